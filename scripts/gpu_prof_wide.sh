#!/bin/bash
# Per-kernel times of the wide steps (rocprofv3 kernel trace + stats): 784-4096-10 fp32, 784-1024-10 bf16.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/profwide
mkdir -p $O
for cfg in "4096 f32" "1024 bf16"; do
  set -- $cfg
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/h$1 -o run --output-format csv -- python3 bench.py --hidden $1 --dtype $2 \
    --steps 200 --warmup 20 > $O/h$1.log 2>&1 || { tail -20 $O/h$1.log; exit 1; }
  f=$(find $O/h$1 -name "*kernel_stats.csv" | head -1)
  echo "== H=$1 $2: $f"
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:12]: print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1000,2), 'us avg', round(float(r['Percentage']),1), '%')
"
done
