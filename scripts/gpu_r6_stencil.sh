# The two-step (temporal-blocked) LDS stencil: bitwise tests, then the suite's order-8 runs (every variant checked
# against the CPU oracle, ULP-512).
set -o pipefail
mkdir -p gpurun_out/r6/stencil
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_suite_gpu.py -k stencil > gpurun_out/r6/stencil/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -m cme213_sp18_amd.suite stencil -s -v -t --nx 4096 --ny 4096 --iters 400 --order 8 > gpurun_out/r6/stencil/stencil4096.log 2>&1 || exit 1
timeout -k 10 300 python -m cme213_sp18_amd.suite stencil -s -v -t --nx 12288 --ny 12288 --iters 20 --order 8 > gpurun_out/r6/stencil/stencil12288.log 2>&1
