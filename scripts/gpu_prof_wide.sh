set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/profw
mkdir -p $O
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/f32" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --hidden 4096 --steps 500 --warmup 50) > $O/f32.log 2>&1 && tail -1 $O/f32.log | cut -c1-200 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/bf1024" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --hidden 1024 --dtype bf16 --steps 1000 --warmup 100) > $O/bf1024.log 2>&1 && tail -1 $O/bf1024.log | cut -c1-200
find $O -name "*kernel_stats.csv"
