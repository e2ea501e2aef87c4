#!/bin/bash
# Round 3 evidence for the default bench command: a kernel-trace + stats run of
# the command itself, the same with one stream (k_search alone per launch, to
# compare with the line's roofline.kernel.avg_us), then PMC passes (one counter
# group per run).  Summaries: python scripts/traffic.py <TAG> (after the call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r3p}
ARGS=${BENCH_ARGS:-""}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${T}_trace.log 2>&1 && echo trace-ok &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_one -o run --output-format csv -- python3 bench.py $ARGS --streams 1 --no-blob-layout --no-cpu > gpurun_out/${T}_one.log 2>&1 && echo one-stream-ok &&
pmc() {  # name, counters...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/${T}_$name -o run --output-format csv -- python3 bench.py $ARGS --no-blob-layout --no-cpu > gpurun_out/${T}_$name.log 2>&1 && echo "$name-ok"
} &&
pmc fetch FETCH_SIZE &&
pmc ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum &&
pmc write WRITE_SIZE &&
pmc tcc TCC_HIT_sum TCC_MISS_sum
