#!/bin/bash
# One parameterised driver for the GPU box (run through gpurun from the repo
# root):  bash scripts/gpu.sh TAG STEP [STEP ...]
#   suite    pytest -m gpu (the driver's round-end command, verbose, 120 s per test)
#   smoke    __graft_entry__.smoke()
#   stress   scripts/stress_grouped.py for 150 s (grouped launches vs the oracle)
#   bench    python bench.py (defaults) and the driver's command (--steps 20 --warmup 5)
#   single   bench.py --single-batch only (one 100k batch per call)
#   trace    rocprofv3 --kernel-trace --stats on bench.py --streams 1 and on the default command
#   pmc      rocprofv3 PMC passes (FETCH/WRITE size, memory-side requests) on bench.py --streams 1
#   configs  bench.py --config c1 / c3 / c4 / c5
# Every step has its own time limit; the first failing step ends the run.
# Output: gpurun_out/TAG/*.
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run NAME SECONDS CMD...: stdout+stderr to $OUT/NAME.log
    local name=$1 secs=$2; shift 2
    echo "[$(date +%T)] $name: $*"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] $name rc=$rc"
    tail -3 "$OUT/$name.log"
    return $rc
}
for step in "$@"; do
    case $step in
        suite) run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1 ;;
        smoke) run smoke 300 python -u -c 'import __graft_entry__ as g; g.smoke()' || exit 1 ;;
        stress) run stress 240 python -u scripts/stress_grouped.py --seconds 150 || exit 1 ;;
        bench)
            run bench_default 400 python -u bench.py || exit 1
            run bench_driver 400 python -u bench.py --steps 20 --warmup 5 || exit 1 ;;
        single) run bench_single 300 python -u bench.py --single-batch-only || exit 1 ;;
        trace)
            run trace_one_stream 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace1" -o run -- \
                python -u bench.py --streams 1 --no-cpu || exit 1
            run trace_default 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace2" -o run -- \
                python -u bench.py --no-cpu || exit 1 ;;
        pmc)
            for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_REQ_sum TCC_HIT_sum"; do
                nm=$(echo "$ctr" | tr ' ' '_')
                run "pmc_$nm" 300 rocprofv3 --pmc $ctr -d "$OUT/pmc_$nm" -o run -- \
                    python -u bench.py --streams 1 --no-cpu || exit 1
            done ;;
        configs)
            for c in c1 c3 c4 c5; do
                run "bench_$c" 600 python -u bench.py --config $c || exit 1
            done ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "ALL_OK"
