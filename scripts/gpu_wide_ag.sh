#!/bin/bash
# The fused wide all-gather head on one MI355X: its tests, the head-form A/B, then the end-of-round
# validation (scripts/gpu_final.sh).  Every GPU step has its own time limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/wide_ag
mkdir -p $O
echo "== tests (fused wide head)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "wide_fused_allgather" > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wide_step_matches_torch or wide_engines_agree" > $O/pytest2.log 2>&1
rc=$?; tail -3 $O/pytest2.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B"
timeout -k 10 300 python bench/wide_ag_ab.py --hidden 4096 1024 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep '^{' $O/ab.log
[ "$1" = "--final" ] || exit 0
bash scripts/gpu_final.sh
