# (bench/flags_ab_run.sh command: the wide bf16 steps, kbench rows)
python bench/kbench.py --hidden 4096 --cols 800 --cfg bf16:split1 --reps 60 &&
python bench/kbench.py --hidden 1024 --cols 800 --cfg bf16:split1 --reps 100
