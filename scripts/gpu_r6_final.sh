# Round-6 final validation: the pipeline's tests, the driver's bench form x3 (fresh processes), a long run, the full
# GPU tier, smoke().
set -o pipefail
O=gpurun_out/r6/final${TAG:-}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_xstep.py > $O/pytest_xstep.log 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || exit 1; done
timeout -k 10 300 python bench.py --gpus 1 --steps 2000 --warmup 200 > $O/long.json 2> $O/long.err || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1
