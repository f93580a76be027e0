#!/bin/bash
# End-of-round-5 PMC passes on the headline step kernels (784-100-10, n = 800, split3, training form: no a1 store):
# the row-major operand forms (kbench cfg +z0+y0+a1+v0: fp32 W1 and the pixels row-major, dZ1 as three bf16 planes)
# against the final defaults (fragment-ordered W1 / pixel copies, fp32 dZ1 in fragment order).  Same counter groups
# as scripts/gpu_pmc_headline_r5.sh, one group per rocprofv3 run under its own time limit.  Usage: repo root, GPU box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
for X in rowmajor final; do
  SUF=""
  [ "$X" = rowmajor ] && SUF="+z0+y0+a1+v0"
  OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc_end_$X"
  mkdir -p "$OUT"
  run() {  # name counters...
    local name=$1; shift
    (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT" -o "$name" --output-format csv -- \
      python3 "$GRAFT_REPO_ROOT/bench/kbench.py" --hidden 100 --cols 800 --cfg "f32:split3+s0$SUF" --reps 20 \
      > "$OUT/$name.log" 2>&1)
    local rc=$?
    echo "$X $name rc=$rc"
    return $rc
  }
  run l2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE &&
  run waves SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE &&
  run lat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE &&
  run lds SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE || exit 1
  python3 "$GRAFT_REPO_ROOT/scripts/pmc_table.py" "$OUT" --min-us 1 > "$OUT/table.md" && cat "$OUT/table.md"
done
