#!/bin/bash
# Round-2 measurements on one MI355X: the driver-style short bench (first-replay overhead), and our
# GEMMs against the vendor BLAS (bench/gemm_vs_vendor.py).  Every GPU step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2m
mkdir -p $O
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 20 --warmup 20" "--steps 200 --warmup 5" \
            "--steps 20 --warmup 5 --dtype bf16"; do
  echo "== bench $args"
  timeout -k 10 120 python bench.py $args > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step']*1e3, 'us/step')"
done
echo "== gemm vs vendor"
timeout -k 10 300 python bench/gemm_vs_vendor.py --json $O/gemm_vs_vendor.json > $O/gemm.log 2>&1
rc=$?; cat $O/gemm.log | tail -30; exit $rc
