#!/bin/bash
# Iteration loop on the GPU box: tests (optional), kernel microbench, headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -4 gpurun_out/pytest_gpu.log
  [ $rc -ge 124 ] && exit $rc
fi
timeout -k 10 300 python bench/kbench.py ${KBENCH_ARGS:-} > gpurun_out/kbench.log 2>&1; echo "kbench rc=$?"; cat gpurun_out/kbench.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; grep -v amdgpu.ids gpurun_out/bench.log
