#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 200 python bench/kbench.py --hidden 100 300 --cols 800 --cfg f32:split3+a0 f32:split3+a1 f32:split3+a2 f32:split3+a3 f32:split3+a0 f32:split3+a1 f32:split3+a2 f32:split3+a3 > $O/kbench.log 2>&1 \
  || { tail -5 $O/kbench.log; exit 1; }
grep -v amdgpu $O/kbench.log | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print({k:v for k,v in r.items() if k.endswith('_us') or k in ('path','H')})"
for a in 0 1 2 3; do
  echo "== bench a_fp32=$a"
  CME_A_FP32=$a timeout -k 10 120 python bench.py --steps 4000 --warmup 400 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(round(r['ms_per_step']*1e3,3), 'us/step', r['value'])"
done
