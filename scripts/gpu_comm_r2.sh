#!/bin/bash
# Communication-policy data on a one-GPU box (2 ranks sharing GPU 0): the all-reduce sweep with the fp32
# and bf16 xGMI wires, and bench.py at BASELINE config 5's shape (784-1024-10 bf16) through the trainer's
# automatic choice.  Each step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp CME_SHARED_GPU=1 OMP_NUM_THREADS=2
O=gpurun_out/comm
mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29671 bench/allreduce_bench.py --paths xgmi xgmi-bf16 --max-bytes $((16 << 20)) --iters 30 \
  --json $O/allreduce_shared2.json > $O/allreduce.log 2>&1 || { tail -20 $O/allreduce.log; exit 1; }
grep '^{' $O/allreduce.log
for args in "--hidden 1024 --dtype bf16" "--hidden 1024 --dtype bf16 --allreduce rccl" "--hidden 100" "--hidden 100 --scaling strong"; do
  echo "== bench 2 ranks (shared GPU) $args"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29672 bench.py --gpus 2 --steps 200 --warmup 20 $args > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(round(r['ms_per_step']*1e3,2), 'us/step', r['value'], r['config']['allreduce'], r['scaling'], r['config']['global_batch'])"
done
