#!/bin/bash
# End-of-round validation on one MI355X, in the order the driver runs things:
# GPU tests, smoke(), the no-flag bench, the other BASELINE configs at N=1, and a rocprofv3 kernel summary.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
step() { echo "== $*"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
step smoke
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step bench default
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
step bench configs
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driverform.log 2>&1 && tail -1 $O/bench_driverform.log &&
timeout -k 10 300 python bench.py --steps 4000 --warmup 400 > $O/bench_h100_f32.log 2>&1 && tail -1 $O/bench_h100_f32.log &&
timeout -k 10 300 python bench.py --steps 4000 --warmup 400 --dtype bf16 > $O/bench_h100_bf16.log 2>&1 && tail -1 $O/bench_h100_bf16.log &&
timeout -k 10 300 python bench.py --hidden 4096 --steps 2000 --warmup 200 > $O/bench_h4096_f32.log 2>&1 && tail -1 $O/bench_h4096_f32.log &&
timeout -k 10 300 python bench.py --hidden 1024 --dtype bf16 --steps 2000 --warmup 200 > $O/bench_h1024_bf16.log 2>&1 && tail -1 $O/bench_h1024_bf16.log &&
timeout -k 10 300 python bench.py --mode reference --steps 200 --warmup 20 > $O/bench_reference_mode.log 2>&1 && tail -1 $O/bench_reference_mode.log &&
timeout -k 10 300 python -m cme213_sp18_amd.train -g 4 > $O/grade4_gemm.log 2>&1 && grep -A2 "GEMM" $O/grade4_gemm.log || exit 1
step rocprof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2000 --warmup 200 > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1
echo "rocprof rc=$?"
find "$GRAFT_REPO_ROOT/$O/prof" -name "*stats*"
