# PMC passes over one bench command (each counter group in its own run:
# MI355X_MICROARCH.md, rocprofv3 PMC slots).  TAG and BENCH_ARGS from the env.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r2p}
ARGS=${BENCH_ARGS:-"--steps 40 --warmup 8 --no-cpu --options 1"}
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/${T}_$name -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${T}_$name.log 2>&1 && echo "$name-ok"
}
timeout -k 10 120 rocprofv3 -L > gpurun_out/${T}_counters.txt 2>&1
run fetch FETCH_SIZE &&
run tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum &&
run ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum &&
run tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum &&
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU
