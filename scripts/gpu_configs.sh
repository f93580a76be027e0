#!/bin/bash
# BASELINE configs on one GPU (per-GPU slices of the 8-GPU configs) + the reference-equivalent mode.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/configs"
mkdir -p "$OUT"
b() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep '^{' "$OUT/$name.log" | tail -1)"
  [ $rc -ne 0 ] && tail -20 "$OUT/$name.log"
  return $rc
}
b h100_f32 --steps 4000 --warmup 400 &&
b h100_bf16 --dtype bf16 --steps 4000 --warmup 400 &&
b h100_f64 --dtype f64 --steps 2000 --warmup 200 &&
b h1024_bf16 --hidden 1024 --dtype bf16 --steps 2000 --warmup 200 &&
b h1024_f32 --hidden 1024 --steps 2000 --warmup 200 &&
b h4096_f32 --hidden 4096 --steps 1000 --warmup 100 &&
b h100_reference --mode reference --steps 500 --warmup 50 &&
CME_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 2 --mode reference --steps 200 --warmup 20 \
  > "$OUT/shared2_reference.log" 2>&1; rc=$?
echo "shared2_reference rc=$rc: $(grep '^{' "$OUT/shared2_reference.log" | tail -1)"
exit $rc
