#!/bin/bash
# End-of-round validation on one MI355X (run through gpurun from the repo root): the GPU test tier, smoke(), the
# driver's exact bench command as fresh processes, a long run, the wide configs and a kernel-trace profile.  Every GPU
# step has its own time limit and the steps are chained: the first failure ends the script.
#   bash bench/final_validation.sh [outdir]
set -o pipefail
OUT=${1:-gpurun_out/final}
mkdir -p "$OUT"
step() {  # step <name> <seconds> <command...>: stdout+stderr to $OUT/<name>.log
  local name=$1 secs=$2
  shift 2
  echo "[$(date +%T)] $name" >&2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >&2
  return $rc
}
step driver1 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 &&
step driver2 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 &&
step driver3 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 &&
step long 180 python3 bench.py --gpus 1 --steps 2000 --warmup 200 &&
step smoke 120 python3 -c "import __graft_entry__ as g; g.smoke()" &&
step pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
step wide4096_f32 180 python3 bench.py --gpus 1 --hidden 4096 --dtype f32 --steps 200 --warmup 20 &&
step wide4096_bf16 180 python3 bench.py --gpus 1 --hidden 4096 --dtype bf16 --steps 200 --warmup 20 &&
step wide1024_bf16 180 python3 bench.py --gpus 1 --hidden 1024 --dtype bf16 --steps 400 --warmup 40 &&
# (the wide configs run 1.8-2.4 us/step slower for their first few hundred steps: the same runs after 600 warm-up steps)
step wide4096_f32_warm 180 python3 bench.py --gpus 1 --hidden 4096 --dtype f32 --steps 400 --warmup 600 &&
step wide4096_bf16_warm 180 python3 bench.py --gpus 1 --hidden 4096 --dtype bf16 --steps 400 --warmup 600 &&
step wide1024_bf16_warm 180 python3 bench.py --gpus 1 --hidden 1024 --dtype bf16 --steps 400 --warmup 600 &&
step headline_bf16 120 python3 bench.py --gpus 1 --dtype bf16 --steps 2000 --warmup 200 &&
step rocprof 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o headline -- python3 bench.py --gpus 1 --steps 400 --warmup 40
