#!/bin/bash
# Shared-GPU rehearsal of the wide configs' multi-rank paths (CME_SHARED_GPU=1: N ranks on the one GPU of a
# gpurun box; the ranks' kernels compete for the same CUs, so the step times are plumbing evidence, not
# scaling numbers).  One bench.py record per line into gpurun_out/rehearse/rows.jsonl.
#   DP  784-4096-10 fp32: two-shot xGMI (reduce-scatter + sharded SGD + all-gather), N = 2, 4
#   TP  784-4096-10 fp32: hidden-sharded, one z2 all-reduce per step (xGMI one-shot), global batch 800 N, N = 2, 4
#   DP  784-1024-10 bf16: the auto policy (one-shot under 2 MB of wire bytes, two-shot at N >= 4), N = 2, 4
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp CME_SHARED_GPU=1
O=gpurun_out/rehearse
mkdir -p $O
: > $O/rows.jsonl
row() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 240 python bench.py "$@" > $O/$name.log 2>&1
  local rc=$?
  case $rc in
    0) ;;
    124|134|137|139) echo "$name: time limit / abort / fault (rc=$rc): stopping"; tail -20 $O/$name.log; exit $rc ;;
    *) echo "$name FAILED (rc=$rc)"; grep -h '"invalid"' $O/$name.log | cut -c1-300; return 1 ;;
  esac
  grep '^{' $O/$name.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); r['rehearsal']='$name'; print(json.dumps(r))" >> $O/rows.jsonl
  echo "$name ok"
}
# (rows run one after another; a row whose bench.py exits with an error of its own is reported and the next
# row still runs; a time limit, an abort or a fault ends the script)
rc=0
for spec in "${ROWS[@]:-dp4096_n2|--gpus 2 --hidden 4096 --allreduce xgmi2
tp4096_n2|--gpus 2 --hidden 4096 --parallel tp --batch 1600
tp4096_n4|--gpus 4 --hidden 4096 --parallel tp --batch 3200
dp1024bf_n2|--gpus 2 --hidden 1024 --dtype bf16
dp1024bf_n4|--gpus 4 --hidden 1024 --dtype bf16
dp4096_n4|--gpus 4 --hidden 4096 --allreduce xgmi2}"; do
  while IFS='|' read -r name args; do
    [ -n "$name" ] || continue
    row "$name" $args --steps 40 --warmup 10 || rc=1
  done <<< "$spec"
done
python - <<'EOF'
import json
for l in open("gpurun_out/rehearse/rows.jsonl"):
    r = json.loads(l); c = r["config"]
    print(r["rehearsal"], r["n_gpus"], round(r["ms_per_step"] * 1e3, 1), "us/step", c.get("parallelism"),
          c.get("allreduce"), c.get("allreduce_us"), c.get("allreduce_bytes"), c.get("comm_ok"))
EOF
exit $rc
