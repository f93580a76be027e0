#!/bin/bash
# Iteration loop on the GPU box: tests (optional), smoke, kernel microbench, headline bench.
# Every GPU step has its own time limit; the script stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -5 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
if [ "${RUN_KBENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench/kbench.py ${KBENCH_ARGS:-} > gpurun_out/kbench.log 2>&1; rc=$?
  echo "kbench rc=$rc"; grep -v amdgpu.ids gpurun_out/kbench.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench.log
exit $rc
