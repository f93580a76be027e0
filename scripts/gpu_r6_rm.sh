#!/bin/bash
# The pipeline's row-major form (off-grid steps, n = 100): its tests, then walking steps against the two-launch loop.
set -o pipefail
O=gpurun_out/r6rm; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_xstep.py > $O/pytest_xstep4.log 2>&1 &&
timeout -k 10 240 python -u bench/xstep_ab.py --cols 100 104 256 800 --reps 400 --rounds 2 --json $O/xstep_ab_rm4.jsonl > $O/xstep_ab.log 2>&1
