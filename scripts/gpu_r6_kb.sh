#!/bin/bash
# Per-rank steps at n = 800 / 400 / 200 / 100 on the tree with the pipeline's row-major form, then the predicted curve.
set -o pipefail
O=gpurun_out/r6kb; mkdir -p $O
PYTHONPATH=. timeout -k 10 400 python -u bench/kbench.py --cfg f32:split3+s0 --cols 800 400 200 100 --json $O/kbench_headline_r6c.jsonl > $O/kbench.log 2>&1 &&
python bench/predict_scaling.py $O/kbench_headline_r6c.jsonl > $O/predict_scaling_r6c.jsonl 2> $O/predict.err
