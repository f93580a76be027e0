# Kernel-trace statistics of 784-1024-10 bf16 (the bench form with 600 warm-up steps) and a stamped step breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O="$GRAFT_REPO_ROOT/gpurun_out/r6/stats_w1024"
mkdir -p $O
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/w1024" -o bench --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --hidden 1024 --dtype bf16 --steps 400 --warmup 600 > "$O/w1024.json" 2> "$O/w1024.err")
