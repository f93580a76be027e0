# A/B: 784-1024-10 bf16 weight gradient with split-K over the batch (CME_SPLITK_KS slices, gate lowered to n >= 512)
# against the one-pass 64 x 64 launch, alternated in fresh processes (bench form after 600 warm-up steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6/splitk_w1024
mkdir -p $O
B() { timeout -k 10 200 python bench.py --gpus 1 --hidden 1024 --dtype bf16 --steps 400 --warmup 600; }
for r in 1 2; do
  B > $O/base_$r.json 2> $O/base_$r.err || exit 1
  CME_SPLITK_KS=2 CME_SPLITK_MIN_N=512 B > $O/ks2_$r.json 2> $O/ks2_$r.err || exit 1
  CME_SPLITK_KS=3 CME_SPLITK_MIN_N=512 B > $O/ks3_$r.json 2> $O/ks3_$r.err || exit 1
done
for f in $O/*.json; do python -c "import json,sys;d=json.load(open('$f'));print('$f',round(d['ms_per_step']*1e3,2),d['config'].get('params_finite'))"; done
