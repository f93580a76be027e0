# Where the driver form's fixed cost goes on the XCD-local pipeline (bench/driver_gap.py under rocprofv3).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6/gap
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/r6/gap -o gap -- python3 bench/driver_gap.py --steps 20 --reps 6 --out gpurun_out/r6/gap/regions.json > gpurun_out/r6/gap/run.log 2>&1 || exit 1
python3 bench/driver_gap.py --analyse gpurun_out/r6/gap > gpurun_out/r6/gap/analysis.jsonl 2>&1
