# The driver's multi-GPU bench form on the final tree, rehearsed on the one GPU of a gpurun box (CME_SHARED_GPU=1:
# the N ranks share device 0, so step times are plumbing evidence, not scaling numbers): torch.distributed.run,
# one rank per "GPU", N = 2, 4, 8, exactly the driver's command line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp CME_SHARED_GPU=1
O=gpurun_out/r6/driver_multi
mkdir -p $O
for N in 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29500 + N)) bench.py --gpus $N --steps 20 --warmup 5 > $O/n$N.json 2> $O/n$N.err || exit 1
  echo "N=$N ok"
done
