#!/bin/bash
# xGMI hand-off cost on a one-GPU box: the xGMI tests (shared-GPU ranks), the headline kernels with the
# wgrad-fused all-reduce at world 1 (kbench), the all-reduce sweep and bench.py with 2 ranks on GPU 0.
# Each step has its own limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/xflag
mkdir -p $O
echo "== xgmi tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_xgmi.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== kbench H=100"
timeout -k 10 120 python bench/kbench.py --hidden 100 --cols 800 --cfg f32:split3 bf16:split1 > $O/kbench.log 2>&1 \
  || { tail -5 $O/kbench.log; exit 1; }
grep -v amdgpu $O/kbench.log | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print({k:v for k,v in r.items() if k.endswith('_us') or k in ('dtype','H')})"
export CME_SHARED_GPU=1 OMP_NUM_THREADS=2
echo "== allreduce sweep (2 ranks, shared GPU)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29671 bench/allreduce_bench.py --paths xgmi xgmi-bf16 --max-bytes $((16 << 20)) --iters 30 \
  --json $O/allreduce_shared2.json > $O/allreduce.log 2>&1 || { tail -20 $O/allreduce.log; exit 1; }
grep '^{' $O/allreduce.log
for args in "--hidden 100" "--hidden 1024 --dtype bf16"; do
  echo "== bench 2 ranks (shared GPU) $args"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29672 bench.py --gpus 2 --steps 200 --warmup 20 $args > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(round(r['ms_per_step']*1e3,2), 'us/step', r['value'], r['config']['allreduce'], r['config']['replicas_bitwise_equal'])"
done
