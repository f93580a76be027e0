#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for ts in 800 1600 8000 54000 800 54000; do
  timeout -k 10 120 python bench.py --steps 4000 --warmup 400 --train-size $ts > gpurun_out/loc.log 2>&1 || { tail -5 gpurun_out/loc.log; exit 1; }
  tail -1 gpurun_out/loc.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('train_size=$ts', round(r['ms_per_step']*1e3,3), 'us/step')"
done
