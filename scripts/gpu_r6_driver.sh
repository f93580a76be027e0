set -o pipefail
mkdir -p gpurun_out/r6/driver
for i in 1 2 3; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/driver/driver_$i.json 2> gpurun_out/r6/driver/driver_$i.err || exit 1; done
timeout -k 10 300 python bench.py --gpus 1 --steps 2000 --warmup 200 > gpurun_out/r6/driver/long.json 2> gpurun_out/r6/driver/long.err || exit 1
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/ > gpurun_out/r6/driver/pytest_gpu.log 2>&1
