#!/bin/bash
# Wide configs on the final tree (bench form and after 600 warm-up steps), no PMC passes.
set -o pipefail
O=gpurun_out/r6/wide4
mkdir -p $O
B() { timeout -k 10 300 python bench.py --gpus 1 --steps 200 "$@"; }
B --hidden 4096 --warmup 20 > $O/w4096_f32.json 2> $O/w4096_f32.err &&
B --hidden 4096 --dtype bf16 --warmup 20 > $O/w4096_bf16.json 2> $O/w4096_bf16.err &&
B --hidden 1024 --dtype bf16 --warmup 20 > $O/w1024_bf16.json 2> $O/w1024_bf16.err &&
B --hidden 4096 --warmup 600 > $O/w4096_f32_warm.json 2> $O/w4096_f32_warm.err &&
B --hidden 4096 --dtype bf16 --warmup 600 > $O/w4096_bf16_warm.json 2> $O/w4096_bf16_warm.err &&
B --hidden 1024 --dtype bf16 --warmup 600 > $O/w1024_bf16_warm.json 2> $O/w1024_bf16_warm.err
