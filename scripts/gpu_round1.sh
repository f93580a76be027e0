#!/bin/bash
# First end-to-end GPU check: kernel numerics tests, bench, rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 4000 --warmup 400 > gpurun_out/bench1.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench1.log; exit 1; }
cat gpurun_out/bench1.log
timeout -k 10 300 python bench.py --steps 4000 --warmup 400 --no-graphs > gpurun_out/bench1_eager.log 2>&1; tail -2 gpurun_out/bench1_eager.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2000 --warmup 200 > "$GRAFT_REPO_ROOT/gpurun_out/prof1.log" 2>&1; echo "rocprof rc=$?"
find "$GRAFT_REPO_ROOT/gpurun_out/prof1" -name "*stats*" | head
