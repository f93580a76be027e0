#!/bin/bash
# Multi-rank rehearsal on a one-GPU box (ranks share GPU 0 over a gloo group, CME_SHARED_GPU=1): the N > 1
# bench paths the 8-GPU driver run takes -- xGMI-fused (H=100 weak + strong), xGMI bf16 wire (H=1024 bf16),
# the RCCL-bucketed choice at H=4096 (gloo here) -- each with its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp CME_SHARED_GPU=1 OMP_NUM_THREADS=2
O=gpurun_out/rehearsal
mkdir -p $O
port=29700
for cfg in "2|--hidden 100" "4|--hidden 100" "2|--hidden 100 --scaling strong" "4|--hidden 100 --scaling strong" \
           "2|--hidden 1024 --dtype bf16" "4|--hidden 1024 --dtype bf16" "2|--hidden 4096 --steps 20 --warmup 3"; do
  n=${cfg%%|*}; args=${cfg#*|}; port=$((port + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $n --steps 200 --warmup 20 $args > $O/run.log 2>&1 || { tail -30 $O/run.log; exit 1; }
  grep '^{' $O/run.log | python -c "
import json,sys
r=json.loads(sys.stdin.read().splitlines()[-1])
c=r['config']
print('N=$n', '$args', round(r['ms_per_step']*1e3,2), 'us/step', round(r['value']/1e6,2), 'M img/s', c['allreduce'], c['executor'], r['scaling'], 'gb', c['global_batch'], 'agree', c.get('replicas_bitwise_equal'), r.get('invalid'))"
done
