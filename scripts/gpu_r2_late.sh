#!/bin/bash
# Late round-2 check: every GPU test, smoke, and the bench lines the wide-head changes touch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/late
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 200 python bench.py --hidden 1024 --dtype bf16 --steps 2000 --warmup 200 > $O/b1024bf.log 2>&1 && tail -1 $O/b1024bf.log &&
timeout -k 10 200 python bench.py --hidden 4096 --steps 2000 --warmup 200 > $O/b4096.log 2>&1 && tail -1 $O/b4096.log &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bdriver.log 2>&1 && tail -1 $O/bdriver.log
