#!/bin/bash
# The wide dW1 epilogue through an LDS transpose (16-byte W1 / gradient accesses): tests + step times.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lazy_planes.py tests/test_gpu_mlp.py tests/test_gpu_handoff.py tests/test_tensor_parallel.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_epi.log 2>&1; rc=$?; tail -2 $O/pytest_epi.log; [ $rc -eq 0 ] || { grep -E "^E |^FAILED" $O/pytest_epi.log | head -20; exit $rc; }
timeout -k 10 300 python bench/wide_ag_ab.py --hidden 4096 1024 --cfg f32:split3 bf16:split1 --modes ag_noa1 ag_noa1 > $O/wide_epi.jsonl 2>&1 && grep '^{' $O/wide_epi.jsonl | cut -c1-200
