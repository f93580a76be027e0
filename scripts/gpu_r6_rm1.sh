#!/bin/bash
set -o pipefail
O=gpurun_out/r6rm; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_xstep.py -k "row_major and 800" > $O/pytest_rm800.log 2>&1
