# Round-6 batch: xstep prefetch A/B + fine stamps, then the wide-config warm-up probe.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u bench/xstep_ab.py --cols 800 --rounds 2 --bar 1 --pf 0 2 6 --fha-stamps 30 > gpurun_out/r6/xstep_ab_f.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u bench/wide_warmup.py --hidden 4096 --dtype f32 --blocks 20 --block 25 > gpurun_out/r6/wide_warmup_f32.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u bench/wide_warmup.py --hidden 4096 --dtype bf16 --blocks 20 --block 25 --modes walk same > gpurun_out/r6/wide_warmup_bf16.jsonl 2>&1
