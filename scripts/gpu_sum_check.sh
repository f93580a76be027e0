set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python -u -m pytest tests/test_suite_gpu.py -m gpu -x -q -k sum --timeout 120 --timeout-method thread 2>&1 | tail -2 &&
timeout -k 10 200 python -m cme213_sp18_amd.suite sum --n 30000000 --hbm 536870912 2>&1 | grep -v amdgpu
