#!/bin/bash
# Weak-scaling sweep of the headline bench on one node: bench.py at N = 1, 2, 4, 8 GPUs (one rank per GPU,
# torchrun, RCCL / xGMI), one JSON line per N appended to ${OUT:-bench_scaling.jsonl}, then a table with the
# scaling efficiency value(N) / (N * value(1)).  Extra arguments go to bench.py, e.g.
#   scripts/bench_scaling.sh --hidden 4096            # BASELINE config 4 (global batch 800 * N)
#   scripts/bench_scaling.sh --hidden 1024 --dtype bf16
#   scripts/bench_scaling.sh --allreduce rccl         # force the RCCL path instead of the xGMI kernel
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=${OUT:-bench_scaling.jsonl}
NGPU=$(python3 -c "import torch; print(torch.cuda.device_count())")
: > "$OUT"
for n in 1 2 4 8; do
  [ "$n" -gt "$NGPU" ] && break
  if [ "$n" = 1 ]; then
    timeout -k 10 600 python3 bench.py --gpus 1 "$@" | grep '"metric"' >> "$OUT" || exit $?
  else
    timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
      --master-port $((29800 + n)) bench.py --gpus "$n" "$@" | grep '"metric"' >> "$OUT" || exit $?
  fi
done
python3 - "$OUT" <<'EOF'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
base = next((r["value"] for r in rows if r["n_gpus"] == 1), None)
print(f"{'N':>2} {'images/s':>14} {'us/step':>9} {'allreduce':>11} {'efficiency':>10}")
for r in rows:
    eff = r["value"] / (r["n_gpus"] * base) if base else float("nan")
    print(f"{r['n_gpus']:>2} {r['value']:>14.0f} {1e3 * r['ms_per_step']:>9.2f} {r['config'].get('allreduce', ''):>11} "
          f"{eff:>10.3f}")
EOF
