#!/bin/bash
# Kernel-trace stats of the n = 100 walking steps: the pipeline's row-major form, then the two-launch loop.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r6rm/stats; mkdir -p $O
PYTHONPATH=. timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench/xstep_ab.py --cols 100 --reps 400 --rounds 1 > $O/xstep_ab.log 2>&1
