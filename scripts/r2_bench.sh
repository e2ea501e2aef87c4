# Default bench (faithful headline + derived leg + CPU baseline), then c3 at N=1.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r2d}
timeout -k 10 600 python bench.py > gpurun_out/${T}_default.log 2>&1 && echo default-ok &&
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_driver.log 2>&1 && echo driver-ok &&
timeout -k 10 600 python bench.py --config c3 --no-derived --no-cpu > gpurun_out/${T}_c3.log 2>&1 && echo c3-ok
