#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box (all ranks share cuda:0 over gloo + the xGMI peer kernel),
# then the 1-GPU headline bench and its rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/rehearse"
mkdir -p "$OUT"
for n in 2 4; do
  CME_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 300 --warmup 30 \
    > "$OUT/bench_shared_$n.log" 2>&1; rc=$?
  echo "shared-gpu bench n=$n rc=$rc"; grep -v amdgpu.ids "$OUT/bench_shared_$n.log" | tail -3
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python bench.py > "$OUT/bench1.log" 2>&1; rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids "$OUT/bench1.log"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2000 --warmup 200 > "$OUT/prof_bench.log" 2>&1; rc=$?
echo "prof rc=$rc"; tail -2 "$OUT/prof_bench.log"
exit $rc
