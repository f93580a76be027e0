#!/bin/bash
# Wide-config iteration on one MI355X: correctness of the wide GEMM paths, then their kernel timings
# (kbench) and the vendor comparison.  Every GPU step has its own time limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/wide
mkdir -p $O
echo "== tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_dist.py tests/test_tensor_parallel.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== kbench"
timeout -k 10 240 python bench/kbench.py --hidden 4096 1024 --cols 800 --cfg f32:split3 bf16:split1 \
  --json $O/kbench.json > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep -v amdgpu.ids $O/kbench.log | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print({k:v for k,v in r.items() if k.endswith('_us') or k in ('dtype','H')})"
echo "== gemm vs vendor (training shapes)"
timeout -k 10 240 python bench/gemm_vs_vendor.py --only training --json $O/gemm_training.json > $O/gemm.log 2>&1 \
  || { tail -20 $O/gemm.log; exit 1; }
grep -v amdgpu.ids $O/gemm.log
echo "== bench H=4096 f32, H=1024 bf16"
timeout -k 10 120 python bench.py --hidden 4096 --steps 500 --warmup 50 > $O/b4096.log 2>&1 && tail -1 $O/b4096.log &&
timeout -k 10 120 python bench.py --hidden 1024 --dtype bf16 --steps 500 --warmup 50 > $O/b1024.log 2>&1 && tail -1 $O/b1024.log
