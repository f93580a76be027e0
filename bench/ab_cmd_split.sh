# (bench/flags_ab_run.sh command for mlp_split.hip variants: the wide step and the headline's two-launch / fused
# all-reduce steps, kbench rows)
python bench/kbench.py --hidden 4096 --cols 800 --cfg f32:split3 bf16:split1 --reps 60 &&
python bench/kbench.py --hidden 1024 --cols 800 --cfg bf16:split1 --reps 100 &&
python bench/kbench.py --hidden 100 --cols 800 100 --cfg f32:split3+s0 --reps 200
