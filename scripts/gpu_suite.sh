#!/bin/bash
# Homework-suite drivers on the GPU box (numbers for BASELINE/README) + rocprofv3 kernel stats.
# Each GPU step has its own limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/suite"
mkdir -p "$OUT"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAIL:-40}
  return $rc
}
S="python -m cme213_sp18_amd.suite"
run sum 300 $S sum --n 30000000 &&
run radix 300 $S radix --n 4000000 --sweep &&
run shift 300 $S shift --doublings 8 --reps 20 &&
run pagerank 600 $S pagerank &&
run stencil_o8 900 $S stencil --params "$GRAFT_REPO_ROOT/configs/params.in" &&
run stencil_o2 600 $S stencil --nx 4096 --ny 4096 --iters 200 --order 2 &&
run stencil_o4 600 $S stencil --nx 4096 --ny 4096 --iters 200 --order 4 &&
python -c "from cme213_sp18_amd.suite import hw4; open('/tmp/eng.txt','wb').write(hw4.synthetic_english(1235150, 7))" &&
run create_cipher 300 $S create_cipher /tmp/eng.txt 8 --out /tmp/cipher_text.txt &&
run solve_cipher 300 $S solve_cipher /tmp/cipher_text.txt --out /tmp/plain_text.txt &&
cd /tmp && export PYTHONPATH="$GRAFT_REPO_ROOT" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o suite --output-format csv -- \
  python3 -m cme213_sp18_amd.suite stencil --nx 4096 --ny 4096 --iters 50 --order 8 > "$OUT/prof_stencil.log" 2>&1
echo "prof rc=$?"
