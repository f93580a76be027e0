# Process-alternated A/B of the variant packages under bench/ab (bench/flags_ab_build.py): each round runs $CMD
# (default: bench/xstep_ab.py at n = 800) once per variant (fresh process), the tree's own package as "default".
# Output: gpurun_out/r6/flags${TAG}/<variant>_<round>.jsonl
set -o pipefail
O=gpurun_out/r6/flags${TAG:-}
mkdir -p $O
CMD=${CMD:-"python bench/xstep_ab.py --cols 800 --rounds 1 --reps 200"}
for r in 1 2 3; do
  timeout -k 10 200 $CMD > $O/default_$r.jsonl 2>&1 || exit 1
  for d in bench/ab/*/; do
    n=$(basename $d)
    CME_PKG_ROOT=$d timeout -k 10 200 $CMD > $O/${n}_$r.jsonl 2>&1 || exit 1
  done
done
