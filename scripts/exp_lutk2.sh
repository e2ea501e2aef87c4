# Deeper tables: C2 at K = 17 (128 GiB) vs 16, C5 at K = 16 (64 GiB) vs 15.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r1lk2}
FMX_DEEP_LUT_MB=131072 timeout -k 10 400 python bench.py --no-cpu > gpurun_out/${T}_c2_k17.log 2>&1 && echo c2-k17-ok || exit 1
FMX_DEEP_LUT_MB=40960 timeout -k 10 400 python bench.py --no-cpu > gpurun_out/${T}_c2_k16.log 2>&1 && echo c2-k16-ok || exit 1
FMX_DEEP_LUT_MB=65536 timeout -k 10 600 python bench.py --no-cpu --config c5 --steps 20 --warmup 4 > gpurun_out/${T}_c5_k16.log 2>&1 && echo c5-k16-ok || exit 1
FMX_DEEP_LUT_MB=40960 timeout -k 10 600 python bench.py --no-cpu --config c5 --steps 20 --warmup 4 > gpurun_out/${T}_c5_k15.log 2>&1 && echo c5-k15-ok || exit 1
