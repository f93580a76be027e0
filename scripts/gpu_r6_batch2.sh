# Round-6 batch 2: the wide warm-up with a memory-bound pre-load, then the full GPU tier.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 200 python -u bench/wide_warmup.py --hidden 4096 --dtype f32 --blocks 16 --block 25 --modes walk --prewarm-ms 0 > gpurun_out/r6/wide_warmup_prewarm.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u bench/wide_warmup.py --hidden 4096 --dtype f32 --blocks 16 --block 25 --modes walk --prewarm-ms 300 >> gpurun_out/r6/wide_warmup_prewarm.jsonl 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/ > gpurun_out/r6/pytest_gpu_full.log 2>&1
