#!/bin/bash
# Round-6 PMC passes over the XCD-local step pipeline against the two-launch step (784-100-10, n = 800, split3,
# training form): bench/xstep_ab.py runs both forms (one round, the default barrier form), one counter group per
# rocprofv3 run under its own time limit, then scripts/pmc_table.py; then a kernel-trace --stats run of the driver's
# bench form.  Usage (repo root on the GPU box).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/r6/pmc_xstep"
mkdir -p "$OUT"
run() {  # name counters...
  local name=$1; shift
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT" -o "$name" --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench/xstep_ab.py" --cols 800 --rounds 1 --reps 100 > "$OUT/$name.log" 2>&1)
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run l2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE &&
run waves SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE &&
run lat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE &&
run lds SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE || exit 1
python3 "$GRAFT_REPO_ROOT/scripts/pmc_table.py" "$OUT" --min-us 1 > "$OUT/table.md" && cat "$OUT/table.md"
mkdir -p "$GRAFT_REPO_ROOT/gpurun_out/r6/stats"
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r6/stats" -o bench --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 200 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/r6/stats/bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r6/stats/bench.err")
