set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 300 python bench/kbench.py --hidden 100 --cols 800 --cfg f32:split3+fh+q0 f32:split3+fh+q1 f32:split3+fh+q0 f32:split3+fh+q1 > $O/kbench_pollskip.jsonl 2>&1 && grep '^{' $O/kbench_pollskip.jsonl | cut -c1-400 &&
timeout -k 10 400 python bench/wide_ag_ab.py --hidden 4096 1024 --modes ag_noa1+q0 ag_noa1 ag_noa1+q0 ag_noa1 > $O/wide_pollskip.jsonl 2>&1 && grep '^{' $O/wide_pollskip.jsonl | cut -c1-300 &&
bash scripts/gpu_check.sh "tests=tests/test_gpu_xgmi.py -k tunes" configs launch prof
