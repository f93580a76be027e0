#!/bin/bash
# One MI355X check run, made of named stages (run in the order given; the first failure ends the run):
#   tests=<pytest args>  GPU tests of the given files / -k expression (quoted: the string is eval'd)
#   smoke                __graft_entry__.smoke()
#   bench                the driver's form of bench.py (--steps 20 --warmup 5) + a long run
#   configs              the other BASELINE configs at N=1 (H=4096 f32, H=1024 bf16, H=100 bf16)
#   launch               bench.py --gpus 2 on a 1-GPU box: refused without CME_SHARED_GPU, 2 ranks with it
#   prof                 rocprofv3 --kernel-trace --stats of the headline bench
#   probes               launch fixed cost (default and spin-wait device flags) and batch-locality probes
#   wideab               bench/wide_ag_ab.py: the wide fused head vs forward + head kernel (H = 4096, 1024)
#   wideab_lazy          bench/wide_ag_ab.py: lazy W1 planes off / on, alternated (784-4096-10 fp32)
# Usage (from the repo root on the GPU box): scripts/gpu_check.sh tests smoke bench
# Every GPU step has its own time limit; outputs go to gpurun_out/check/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/check
mkdir -p $O
B() { timeout -k 10 "$1" python bench.py "${@:2}"; }
for st in "$@"; do
  echo "== $st"
  case "$st" in
    tests=*)
      eval "timeout -k 10 900 python -u -m pytest ${st#tests=} -m gpu -x -q --timeout 240 --timeout-method thread" \
        > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log
      [ $rc -eq 0 ] || { grep -E "^E |^FAILED" $O/pytest.log | tail -30; exit $rc; } ;;
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
        > $O/pytest_all.log 2>&1; rc=$?; tail -4 $O/pytest_all.log; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      B 300 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 && tail -1 $O/bench_driver.log &&
      B 300 --steps 20 --warmup 5 > $O/bench_driver2.log 2>&1 && tail -1 $O/bench_driver2.log &&
      B 300 --steps 4000 --warmup 400 > $O/bench_long.log 2>&1 && tail -1 $O/bench_long.log || exit 1 ;;
    configs)
      B 300 --hidden 4096 --steps 2000 --warmup 200 > $O/b4096.log 2>&1 && tail -1 $O/b4096.log &&
      B 300 --hidden 4096 --dtype bf16 --steps 2000 --warmup 200 > $O/b4096bf.log 2>&1 && tail -1 $O/b4096bf.log &&
      B 300 --hidden 1024 --dtype bf16 --steps 2000 --warmup 200 > $O/b1024bf.log 2>&1 && tail -1 $O/b1024bf.log &&
      B 300 --dtype bf16 --steps 4000 --warmup 400 > $O/b100bf.log 2>&1 && tail -1 $O/b100bf.log || exit 1 ;;
    launch)
      B 120 --gpus 2 --steps 20 --warmup 5 > $O/launch_refused.log 2>&1; rc=$?
      echo "refused rc=$rc (want non-zero)"; grep -c '^{' $O/launch_refused.log; tail -2 $O/launch_refused.log
      [ $rc -ne 0 ] || exit 1
      CME_SHARED_GPU=1 B 300 --gpus 2 --steps 50 --warmup 10 > $O/launch_shared.log 2>&1 && grep '^{' $O/launch_shared.log || { tail -30 $O/launch_shared.log; exit 1; } ;;
    prof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run \
        --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2000 --warmup 200) > $O/prof.log 2>&1
      echo "rocprof rc=$?"; find $O/prof -name "*kernel_stats*" ;;
    probes)
      timeout -k 10 240 python bench/launch_overhead.py > $O/launch_overhead.jsonl 2>&1 && grep fit $O/launch_overhead.jsonl &&
      timeout -k 10 240 python bench/launch_overhead.py --spin > $O/launch_overhead_spin.jsonl 2>&1 && grep -E "fit|spin" $O/launch_overhead_spin.jsonl &&
      timeout -k 10 240 python bench/batch_locality.py > $O/batch_locality.jsonl 2>&1 && grep '^{' $O/batch_locality.jsonl || exit 1 ;;
    wideab_lazy)
      timeout -k 10 300 python bench/wide_ag_ab.py --hidden 4096 --cfg f32:split3 --modes ag_noa1+l0 ag_noa1+l1 ag_noa1+l0 ag_noa1+l1 \
        > $O/wide_lazy.jsonl 2>&1 || { tail -20 $O/wide_lazy.jsonl; exit 1; }
      grep '^{' $O/wide_lazy.jsonl ;;
    wideab)
      timeout -k 10 300 python bench/wide_ag_ab.py --hidden 4096 1024 > $O/wide_ab.jsonl 2>&1 || { tail -20 $O/wide_ab.jsonl; exit 1; }
      grep '^{' $O/wide_ab.jsonl ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
echo "== done"
