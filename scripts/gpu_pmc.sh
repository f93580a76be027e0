#!/bin/bash
# PMC counter collection for the MLP kernels (counters only with --kernel-trace; no sys/runtime trace).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD -d "$OUT" -o pmc1 --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench/kbench.py" --reps 20 ${KB:-} > "$OUT/pmc1.log" 2>&1; echo "pmc1 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o trace --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench/kbench.py" --reps 20 ${KB:-} > "$OUT/trace.log" 2>&1; echo "trace rc=$?"
ls -R "$OUT" | head -30
