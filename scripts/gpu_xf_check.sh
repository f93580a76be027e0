#!/bin/bash
# fused wgrad + xGMI: cost (world 1, kbench), stress (separate kernel, 4 ranks; fused, 2 ranks), tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench/kbench.py --hidden 100 --cols 800 --cfg f32:split3 --reps 200 > gpurun_out/kb.log 2>&1 || exit $?
grep -o '"wgrad_sgd_us[^,]*\|"wgrad_grads_us[^,]*\|"wgrad_xgmi1_us[^,]*\|"step_fused_us[^,]*\|"step_xgmi1_us[^,]*\|"xgmi1_err[^,]*' gpurun_out/kb.log | tr '\n' ' '; echo
timeout -k 10 300 python scripts/stress_xgmi.py 4 30 > gpurun_out/stress4.log 2>&1 || exit $?
grep bad_elements gpurun_out/stress4.log
timeout -k 10 300 python scripts/stress_fused.py 2 300 > gpurun_out/stress_fused.log 2>&1 || exit $?
grep bad_elements gpurun_out/stress_fused.log
timeout -k 10 900 python -m pytest tests/test_gpu_xgmi.py -x -q > gpurun_out/xg.log 2>&1; rc=$?
tail -4 gpurun_out/xg.log
exit $rc
