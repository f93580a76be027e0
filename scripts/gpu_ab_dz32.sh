#!/bin/bash
# Headline A/B: the all-gather head's fp32 dZ1 store skipped in training (kbench +s0 = store_a1 off) vs kept.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 300 python bench/kbench.py --hidden 100 --cols 800 --cfg f32:split3 f32:split3+s0 f32:split3 f32:split3+s0 f32:split3 f32:split3+s0 > $O/kbench_dz32.jsonl 2>&1 && grep '^{' $O/kbench_dz32.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['path'], r['fwd_head_us'], r['wgrad_sgd_us'], r['step_fused_us'])" &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_handoff.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_dz32.log 2>&1; tail -2 $O/pytest_dz32.log
