#!/bin/bash
# After adopting the fused wide head: every GPU test, the wide bench lines and a kernel profile of H=4096.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/wide_ag2
mkdir -p $O
echo "== pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 200 python bench.py --hidden 4096 --steps 2000 --warmup 200 > $O/b4096.log 2>&1 && tail -1 $O/b4096.log &&
timeout -k 10 200 python bench.py --hidden 4096 --dtype bf16 --steps 2000 --warmup 200 > $O/b4096bf.log 2>&1 && tail -1 $O/b4096bf.log &&
timeout -k 10 200 python bench.py --hidden 1024 --dtype bf16 --steps 2000 --warmup 200 > $O/b1024bf.log 2>&1 && tail -1 $O/b1024bf.log &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bdriver.log 2>&1 && tail -1 $O/bdriver.log || exit 1
echo "== rocprof H=4096"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --hidden 4096 --steps 300 --warmup 30 > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1
echo "rocprof rc=$?"
