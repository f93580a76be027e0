#!/bin/bash
# Train on 8 MI355X of one node: one process per GPU (torchrun), RCCL / xGMI peer all-reduce.
# The reference's job script ran `mpirun -np 4 ./main -g 2` (fpcode/run.sh); extra args pass through,
# e.g.  scripts/run_8gpu.sh -g 2    or    scripts/run_8gpu.sh --preset 8gpu_wide -e 5
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port ${MASTER_PORT:-29500} -m cme213_sp18_amd.train "$@"
