# The device-resident xstep argument block: tests, the kernel A/B, the driver form x3 and the launch-gap trace.
set -o pipefail
mkdir -p gpurun_out/r6/kargs/gap
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_xstep.py > gpurun_out/r6/kargs/pytest_xstep.log 2>&1 || exit 1
timeout -k 10 300 python -u bench/xstep_ab.py --cols 800 400 --rounds 2 --bar 3 > gpurun_out/r6/kargs/xstep_ab.jsonl 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/kargs/driver_$i.json 2> gpurun_out/r6/kargs/driver_$i.err || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/r6/kargs/gap -o gap -- python3 bench/driver_gap.py --steps 20 --reps 6 --out gpurun_out/r6/kargs/gap/regions.json > gpurun_out/r6/kargs/gap/run.log 2>&1 || exit 1
python3 bench/driver_gap.py --analyse gpurun_out/r6/kargs/gap > gpurun_out/r6/kargs/gap/analysis.jsonl 2>&1
