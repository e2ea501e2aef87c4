# A/B of bench variants on one box (after gpu_check.sh built the library)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1}
for O in 0 1 3 13 15; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --options $O > gpurun_out/${T}_bench_opt$O.log 2>&1 || exit 1
  echo opt$O-ok
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --patterns 1000000 > gpurun_out/${T}_bench_1m.log 2>&1 && echo 1m-ok
