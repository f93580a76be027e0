#!/bin/bash
# xGMI bucket sequence diagnostics (the multiprocess test's bucket order, 4 ranks on one GPU) per
# protocol variant, then the grid-barrier microbenchmark
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/diagseq"
mkdir -p "$OUT"
for v in 0; do
  for rep in 1 2 3 4 5; do
    CME_XGMI_VARIANT=$v timeout -k 10 120 python scripts/diag_xgmi.py 4 float32:3 float32:614403 float64:79510 float32:80000 float64:79510 \
      > "$OUT/v${v}_r$rep.log" 2>&1; rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
    echo "variant $v rep $rep: $(grep -c 'bad=' "$OUT/v${v}_r$rep.log") bad lines"; grep 'bad=' "$OUT/v${v}_r$rep.log" | head -4; grep -h "another buffer" "$OUT/v${v}_r$rep.log" | head -2
  done
done
timeout -k 10 60 ./bench/micro/grid_barrier 256 512 2000 && timeout -k 10 60 ./bench/micro/grid_barrier 512 256 2000
