#!/bin/bash
# Round-5 PMC passes on the headline step kernels (784-100-10, n = 800, split3, training form: no a1 store) with the
# head's dW2 partials off and on (kbench cfg suffix +h0 / +h1; MlpStep.head_dw2): the round-4 counter groups (L2
# hit/miss, wave wait / issue mix with MFMA busy, L1->L2 latency with the TCP pending stall, LDS), one group per
# rocprofv3 run under its own time limit, then scripts/pmc_table.py.  Usage (repo root on the GPU box).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
for X in 0 1; do  # X: MlpStep.head_dw2 (the head's dW2 partials) off / on
  OUT="$GRAFT_REPO_ROOT/gpurun_out/pmch_r5_h$X"
  mkdir -p "$OUT"
  run() {  # name counters...
    local name=$1; shift
    (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT" -o "$name" --output-format csv -- \
      python3 "$GRAFT_REPO_ROOT/bench/kbench.py" --hidden 100 --cols 800 --cfg "f32:split3+s0+h$X" --reps 20 \
      > "$OUT/$name.log" 2>&1)
    local rc=$?
    echo "h$X $name rc=$rc"
    return $rc
  }
  run l2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE &&
  run waves SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE &&
  run lat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE &&
  run lds SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE || exit 1
  python3 "$GRAFT_REPO_ROOT/scripts/pmc_table.py" "$OUT" --min-us 1 > "$OUT/table.md" && cat "$OUT/table.md"
done
