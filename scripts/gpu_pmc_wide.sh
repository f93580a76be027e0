#!/bin/bash
# PMC passes on the wide (H=4096) step kernels: L2 hit/miss + HBM reads, wave wait/issue mix, L1->L2
# read latency.  One counter group per rocprofv3 run (no sys/runtime trace), each under its own timeout.
# Env: H (default 4096), CFG (default f32:split3), TAG (output subdir, default pmcw).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmcw}"
mkdir -p "$OUT"
cd /tmp
H=${H:-4096}
CFG=${CFG:-f32:split3}
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT" -o "$name" --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench/kbench.py" --hidden $H --cols 800 --cfg $CFG --reps 20 > "$OUT/$name.log" 2>&1
  echo "$name rc=$?"
}
run l2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE && \
run waves SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE && \
run lat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE && \
run lds SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE
ls "$OUT"
