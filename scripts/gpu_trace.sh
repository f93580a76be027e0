#!/bin/bash
# roctx marker trace of a short profiled training run (--profile: per-phase events + roctx ranges),
# kernel trace alongside; summaries land in gpurun_out/trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/trace"
mkdir -p "$OUT"
cd /tmp
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d "$OUT" -o train --output-format csv -- \
  python3 -m cme213_sp18_amd.train --preset 1gpu_fp32 -e 2 --num-train 16000 --num-test 1000 --profile \
  --outdir /tmp/Outputs > "$OUT/train.log" 2>&1
rc=$?; echo "trace rc=$rc"; ls "$OUT"; exit $rc
