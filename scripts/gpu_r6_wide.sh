# Round-6 wide configs: the bench form (20 warm-up steps, as the VERDICT's targets) and after 600 warm-up steps,
# then the PMC passes of 784-4096-10 fp32 and bf16 (scripts/gpu_pmc_wide.sh) and their tables.
set -o pipefail
O=gpurun_out/r6/wide${TAG:-}
mkdir -p $O
B() { timeout -k 10 300 python bench.py --gpus 1 --steps 200 "$@"; }
B --hidden 4096 --warmup 20 > $O/w4096_f32.json 2> $O/w4096_f32.err &&
B --hidden 4096 --dtype bf16 --warmup 20 > $O/w4096_bf16.json 2> $O/w4096_bf16.err &&
B --hidden 1024 --dtype bf16 --warmup 20 > $O/w1024_bf16.json 2> $O/w1024_bf16.err &&
B --hidden 4096 --warmup 600 > $O/w4096_f32_warm.json 2> $O/w4096_f32_warm.err &&
B --hidden 4096 --dtype bf16 --warmup 600 > $O/w4096_bf16_warm.json 2> $O/w4096_bf16_warm.err &&
B --hidden 1024 --dtype bf16 --warmup 600 > $O/w1024_bf16_warm.json 2> $O/w1024_bf16_warm.err || exit 1
TAG=r6/pmc_wide_f32 CFG=f32:split3 bash scripts/gpu_pmc_wide.sh > $O/pmc_f32.log 2>&1 &&
python3 scripts/pmc_table.py gpurun_out/r6/pmc_wide_f32 --min-us 3 > $O/pmc_f32_table.md &&
TAG=r6/pmc_wide_bf16 CFG=bf16:split1 bash scripts/gpu_pmc_wide.sh > $O/pmc_bf16.log 2>&1 &&
python3 scripts/pmc_table.py gpurun_out/r6/pmc_wide_bf16 --min-us 3 > $O/pmc_bf16_table.md
