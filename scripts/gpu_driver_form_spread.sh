#!/bin/bash
# The driver's bench invocation (bench.py --steps 20 --warmup 5), ten fresh processes: the spread of the
# number the driver records.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/spread
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/spread/b.log 2>&1 || { tail -5 gpurun_out/spread/b.log; exit 1; }
  tail -1 gpurun_out/spread/b.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(round(r['ms_per_step']*1e3,3), round(r['value']/1e6,2))"
done
