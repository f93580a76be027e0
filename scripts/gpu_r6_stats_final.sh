# Kernel-trace statistics of the final tree's bench form (N = 1) and of the wide fp32 config.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O="$GRAFT_REPO_ROOT/gpurun_out/r6/stats_final"
mkdir -p $O
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/headline" -o bench --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 500 --warmup 20 > "$O/headline.json" 2> "$O/headline.err") || exit 1
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/wide_f32" -o bench --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --hidden 4096 --steps 200 --warmup 200 > "$O/wide_f32.json" 2> "$O/wide_f32.err")
