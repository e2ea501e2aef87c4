# A/B of bench variants on one box (after gpu_check.sh built the library)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1}
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --no-deep-lut > gpurun_out/${T}_bench_nolut.log 2>&1 && echo nolut-ok &&
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --occ blob --no-deep-lut > gpurun_out/${T}_bench_blob.log 2>&1 && echo blob-ok &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --patterns 1000000 > gpurun_out/${T}_bench_1m.log 2>&1 && echo 1m-ok
