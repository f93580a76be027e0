set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/final_reh; mkdir -p $O
for n in 2 4; do
  CME_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 300 --warmup 30 > $O/bench_shared_$n.log 2>&1 || { echo "n=$n failed"; tail -20 $O/bench_shared_$n.log; exit 1; }
  echo "n=$n"; tail -1 $O/bench_shared_$n.log
done
CME_BENCH_TEST_FALLBACK=1 CME_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 300 --warmup 30 > $O/bench_shared_2_fallback.log 2>&1 || { echo "fallback failed"; tail -20 $O/bench_shared_2_fallback.log; exit 1; }
echo fallback; tail -1 $O/bench_shared_2_fallback.log
CME_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --hidden 4096 --steps 100 --warmup 10 > $O/bench_shared_2_h4096.log 2>&1 || { echo "h4096 failed"; tail -20 $O/bench_shared_2_h4096.log; exit 1; }
echo h4096; tail -1 $O/bench_shared_2_h4096.log
