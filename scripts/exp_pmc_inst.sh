# Two PMC passes on the C2 default: LDS / instruction-fetch side of k_search.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r1pi}
A="--steps 50 --warmup 5 --no-cpu"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_IFETCH SQ_BUSY_CU_CYCLES --kernel-trace -d gpurun_out/${T}_a -o run --output-format csv -- python3 bench.py $A > gpurun_out/${T}_a.log 2>&1 && echo pa-ok &&
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH_LEVEL --kernel-trace -d gpurun_out/${T}_b -o run --output-format csv -- python3 bench.py $A > gpurun_out/${T}_b.log 2>&1 && echo pb-ok
