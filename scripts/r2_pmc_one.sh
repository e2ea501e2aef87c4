# One PMC pass (COUNTERS) over a bench command (TAG, BENCH_ARGS from the env).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r2pm}
timeout -k 10 300 rocprofv3 --pmc ${COUNTERS:-TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum} --kernel-trace -d gpurun_out/${T} -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:-} > gpurun_out/${T}.log 2>&1 && echo "$T-ok"
