#!/bin/bash
# The row-major form against the fragment-ordered one on plans both can take (n on the 16-sample grid).
set -o pipefail
O=gpurun_out/r6rm; mkdir -p $O
PYTHONPATH=. timeout -k 10 300 python -u bench/xstep_ab.py --rm --cols 800 400 512 --reps 400 --rounds 2 --json $O/xstep_ab_rm_vs_frag.jsonl > $O/xstep_ab_rm_vs_frag.log 2>&1
