#!/bin/bash
# The homework kernel suite on one MI355X, every result checked against its CPU oracle:
#   stencil (order 8: 4096^2 x 400 iterations -- the reference's params.in -- and the HBM-sized 12288^2 x 20),
#   even/odd sum (30M and 2 GB), radix sort, PageRank, shift cipher, Vigenere encrypt + crack.
# Usage (repo root on the GPU box): scripts/gpu_suite.sh   -> gpurun_out/suite/*.log
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/suite_r6
mkdir -p $O
S() { timeout -k 10 "$1" python -m cme213_sp18_amd.suite "${@:2}"; }
S 300 stencil -g -b -s -v -t --nx 4096 --ny 4096 --iters 400 --order 8 > $O/stencil4096.log 2>&1 && tail -6 $O/stencil4096.log &&
S 300 stencil -g -b -s -v -t --nx 12288 --ny 12288 --iters 20 --order 8 > $O/stencil12288.log 2>&1 && tail -6 $O/stencil12288.log &&
S 120 sum --hbm 536870912 > $O/sum.log 2>&1 && tail -2 $O/sum.log &&
S 300 radix > $O/radix.log 2>&1 && tail -4 $O/radix.log &&
S 300 pagerank > $O/pagerank.log 2>&1 && tail -8 $O/pagerank.log &&
S 300 shift > $O/shift.log 2>&1 && tail -12 $O/shift.log &&
S 120 create_cipher - 8 --out $O/cipher.txt > $O/cipher.log 2>&1 && tail -4 $O/cipher.log &&
S 120 solve_cipher $O/cipher.txt > $O/solve.log 2>&1 && tail -4 $O/solve.log
