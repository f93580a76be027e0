#!/bin/bash
# User-facing flows on the GPU: CLI training with progress/JSON log/checkpoints and resume, grade presets 1-3
# (fp64 GPU vs fp64 CPU oracle), bf16 training, predict accuracy.  Each step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/cli
rm -rf $O; mkdir -p $O
step() { echo "== $1"; shift; timeout -k 10 300 "$@" > $O/step.log 2>&1 || { tail -30 $O/step.log; exit 1; }; tail -4 $O/step.log; }
step "train f32 + checkpoints" python -m cme213_sp18_amd.train -n 100 -e 3 -p 1 --log-json $O/run.jsonl --ckpt-dir $O/ck --ckpt-every 1
step "resume" python -m cme213_sp18_amd.train -n 100 -e 2 -p 1 --resume $O/ck
step "bf16" python -m cme213_sp18_amd.train -n 300 -e 2 --dtype bf16
step "grade 1" python -m cme213_sp18_amd.train -g 1
step "grade 2" python -m cme213_sp18_amd.train -g 2
step "grade 3" python -m cme213_sp18_amd.train -g 3
echo "cli ok"
