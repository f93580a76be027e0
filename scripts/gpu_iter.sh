#!/bin/bash
# One iteration on a GPU box: every GPU test, kernel timings at H = 100 / 300, the driver-form and long
# headline bench.  Each step has its own limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/iter
mkdir -p $O
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== kbench"
timeout -k 10 200 python bench/kbench.py --hidden 100 300 --cols 800 --cfg f32:split3 bf16:split1 > $O/kbench.log 2>&1 \
  || { tail -5 $O/kbench.log; exit 1; }
grep -v amdgpu $O/kbench.log | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print({k:v for k,v in r.items() if k.endswith('_us') or k in ('dtype','H')})"
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 4000 --warmup 400" "--steps 2000 --warmup 200 --dtype bf16"; do
  echo "== bench $args"
  timeout -k 10 120 python bench.py $args > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(round(r['ms_per_step']*1e3,3), 'us/step', r['value'])"
done
