#!/bin/bash
# rocprofv3 evidence for profiles/: kernel stats of the headline bench, and PMC counters
# (kernel-trace only, no sys/runtime trace) for the H=100 and H=4096 steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/prof2"
mkdir -p "$OUT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o bench --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2000 --warmup 200 > "$OUT/bench.log" 2>&1; echo "stats rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o wide --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --hidden 4096 --steps 300 --warmup 30 > "$OUT/wide.log" 2>&1; echo "wide stats rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o bf1024 --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --hidden 1024 --dtype bf16 --steps 500 --warmup 50 > "$OUT/bf1024.log" 2>&1; echo "bf1024 stats rc=$?"
PMC="SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
for H in 100 4096; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $PMC -d "$OUT" -o pmc_h$H --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench/kbench.py" --hidden $H --cols 800 --cfg f32:split3 --reps 20 > "$OUT/pmc_h$H.log" 2>&1
  echo "pmc H=$H rc=$?"
done
ls "$OUT"
