#!/bin/bash
# Lazy W1-plane A/B at 784-4096-10 fp32, the headline's hand-off poll A/B, then bf16 wide-layer PMC (config 5 at
# H=1024 and the H=4096 bf16 step).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 300 python bench/wide_ag_ab.py --hidden 4096 --cfg f32:split3 --modes ag_noa1 ag_noa1+l1 ag_noa1 ag_noa1+l1 > $O/wide_lazy.jsonl 2>&1 && grep '^{' $O/wide_lazy.jsonl | cut -c1-300 &&
timeout -k 10 300 python bench/kbench.py --hidden 100 --cols 800 --cfg f32:split3+q0 f32:split3+q1 f32:split3+q0 f32:split3+q1 > $O/kbench_pollskip_h100.jsonl 2>&1 && grep '^{' $O/kbench_pollskip_h100.jsonl | cut -c1-330 &&
H=4096 CFG=bf16:split1+s0 TAG=pmc_bf4096 bash scripts/gpu_pmc_wide.sh &&
H=1024 CFG=bf16:split1+s0 TAG=pmc_bf1024 bash scripts/gpu_pmc_wide.sh &&
python scripts/pmc_table.py gpurun_out/pmc_bf4096 --min-us 5 && python scripts/pmc_table.py gpurun_out/pmc_bf1024 --min-us 5
