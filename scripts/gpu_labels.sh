#!/bin/bash
# Labels fetched with the first burst in the heads: MLP tests, the wide-head timeline, kernel timings, benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/labels
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench/stamps_hw.py > $O/stamps_hw.jsonl 2>&1 || { tail -5 $O/stamps_hw.jsonl; exit 1; }
grep -v amdgpu $O/stamps_hw.jsonl | tail -2
timeout -k 10 120 python bench/stamps_fha.py > $O/stamps_fha.jsonl 2>&1 || { tail -5 $O/stamps_fha.jsonl; exit 1; }
grep -v amdgpu $O/stamps_fha.jsonl | tail -2
timeout -k 10 120 python bench/stamps_wgrad.py > $O/stamps_wgrad.jsonl 2>&1 || { tail -5 $O/stamps_wgrad.jsonl; exit 1; }
grep -v amdgpu $O/stamps_wgrad.jsonl | tail -2
timeout -k 10 300 python bench/kbench.py --hidden 100 4096 1024 --cols 800 --cfg f32:split3 bf16:split1 > $O/kbench.log 2>&1 \
  || { tail -5 $O/kbench.log; exit 1; }
grep -v amdgpu $O/kbench.log | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print({k:v for k,v in r.items() if k in ('dtype','H','fwd_head_us','wgrad_sgd_us','step_fused_us','step_xgmi1_us')})"
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 4000 --warmup 400" "--hidden 4096 --steps 1000 --warmup 100" "--hidden 1024 --dtype bf16 --steps 1000 --warmup 100"; do
  timeout -k 10 120 python bench.py $args > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('$args', round(r['ms_per_step']*1e3,3), 'us/step')"
done
