#!/bin/bash
# Round-2 homework-kernel measurements: suite GPU tests, the even/odd sum on the reference size and on an
# input 8x the 256 MB MALL, and the order-8 stencil variants at 4096^2 (reference) and 12288^2 (two 604 MB
# grids: an HBM-bound number).  Each GPU step has its own limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/suite2"
mkdir -p "$OUT"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAIL:-12}
  return $rc
}
S="python -m cme213_sp18_amd.suite"
run tests 300 python -u -m pytest tests/test_suite_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread &&
run sum 300 $S sum --n 30000000 --hbm 536870912 &&
run stencil_o8 600 $S stencil --params "$GRAFT_REPO_ROOT/configs/params.in" &&
run stencil_o8_12288 900 $S stencil --nx 12288 --ny 12288 --iters 20 --order 8
