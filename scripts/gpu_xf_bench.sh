#!/bin/bash
# fused vs separate xGMI all-reduce: world-1 kernel costs, then 2-rank shared-GPU benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/xfb"
mkdir -p "$OUT"
timeout -k 10 200 python bench/kbench.py --hidden 100 --cols 800 100 --cfg f32:split3 --reps 300 > $OUT/kb.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/kb.log
for fz in 1 0; do
  CME_XGMI_FUSED=$fz CME_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 500 --warmup 50 > "$OUT/b2_$fz.log" 2>&1 || exit $?
  echo "fused=$fz"; grep '"metric"' "$OUT/b2_$fz.log"
done
