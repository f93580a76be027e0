set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u bench/wide_warmup.py --hidden 100 --dtype f32 --blocks 20 --block 20 --modes reset --probe-during > gpurun_out/r6/headline_warmup_reset.jsonl 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_xgmi.py tests/test_gpu_xstep.py tests/test_probe_guard.py tests/test_suite_gpu.py tests/test_tensor_parallel.py > gpurun_out/r6/pytest_gpu_rest.log 2>&1
