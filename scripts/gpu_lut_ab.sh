# deep k-mer table budget A/B on C2 (K=12 at 2 GiB default, K=13 at 16 GiB)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1}
FMX_DEEP_LUT_MB=16384 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/${T}_bench_k13.log 2>&1 && echo k13-ok &&
FMX_DEEP_LUT_MB=16384 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --patterns 1000000 > gpurun_out/${T}_bench_k13_1m.log 2>&1 && echo k13-1m-ok
