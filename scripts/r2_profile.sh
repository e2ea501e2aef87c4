# Evidence for one bench command: a kernel-trace + stats run of the command
# itself, then PMC passes (one counter group per run) over the same command
# without its derived-index and CPU legs.  TAG, BENCH_ARGS from the env.
# Summaries: python scripts/traffic.py <TAG> (after the call).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r2e}
ARGS=${BENCH_ARGS:-""}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${T}_trace.log 2>&1 && echo trace-ok &&
pmc() {  # name, counters...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/${T}_$name -o run --output-format csv -- python3 bench.py $ARGS --no-derived --no-cpu > gpurun_out/${T}_$name.log 2>&1 && echo "$name-ok"
} &&
pmc fetch FETCH_SIZE &&
pmc ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum &&
pmc write WRITE_SIZE &&
pmc tcc TCC_HIT_sum TCC_MISS_sum
