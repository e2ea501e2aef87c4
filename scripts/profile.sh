# rocprofv3 passes over the C2 bench (no CPU leg).  Kernel trace + stats in one
# run; each PMC counter group in its own run (MI355X_MICROARCH.md, rocprofv3).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r1}
ARGS=${BENCH_ARGS:-"--steps 50 --warmup 5 --no-cpu"}
# (the engine is built here, in-tree, before the call; the box only runs it)
timeout -k 10 120 rocprofv3 -L > gpurun_out/${T}_counters.txt 2>&1;
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${T}_trace.log 2>&1 && echo trace-ok &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${T}_pmc1 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${T}_pmc1.log 2>&1 && echo pmc1-ok &&
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/${T}_pmc2 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${T}_pmc2.log 2>&1 && echo pmc2-ok &&
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace -d gpurun_out/${T}_pmc3 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${T}_pmc3.log 2>&1 && echo pmc3-ok
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d gpurun_out/${T}_pmc4 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${T}_pmc4.log 2>&1 && echo pmc4-ok
