# L2 hits/misses and memory-side requests per launch: super vs paired records.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--no-derived --no-cpu --steps 160"
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace -d gpurun_out/r2sp_super -o run --output-format csv -- python3 bench.py $A > gpurun_out/r2sp_super.log 2>&1 && echo super-ok &&
FMX_OCC_SUPER=0 timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace -d gpurun_out/r2sp_paired -o run --output-format csv -- python3 bench.py $A > gpurun_out/r2sp_paired.log 2>&1 && echo paired-ok &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES --kernel-trace -d gpurun_out/r2sp_super_sq -o run --output-format csv -- python3 bench.py $A > gpurun_out/r2sp_super_sq.log 2>&1 && echo super-sq-ok &&
FMX_OCC_SUPER=0 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES --kernel-trace -d gpurun_out/r2sp_paired_sq -o run --output-format csv -- python3 bench.py $A > gpurun_out/r2sp_paired_sq.log 2>&1 && echo paired-sq-ok
