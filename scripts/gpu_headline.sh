#!/bin/bash
# Headline (784-100-10) iteration on one MI355X: step-path tests, the launch-overhead sweep and the
# driver-form bench (20 steps, 5 warm-up) a few times, plus a long run.  Each GPU step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/headline
mkdir -p $O
echo "== tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== kbench"
timeout -k 10 120 python bench/kbench.py --hidden 100 --cols 800 --cfg f32:split3 bf16:split1 > $O/kbench.log 2>&1 || { tail -5 $O/kbench.log; exit 1; }
grep -v amdgpu $O/kbench.log | cut -c1-260
echo "== launch overhead"
timeout -k 10 200 python bench/launch_overhead.py > $O/launch_overhead.jsonl 2>&1 || { tail -5 $O/launch_overhead.jsonl; exit 1; }
grep -v amdgpu $O/launch_overhead.jsonl
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 20 --warmup 5 --executor graph" "--steps 20 --warmup 5 --executor graph" "--steps 4000 --warmup 400"; do
  echo "== bench $args"
  timeout -k 10 120 python bench.py $args > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(round(r['ms_per_step']*1e3,3), 'us/step', r['config']['executor'])"
done
