set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/micro/fetch64 > gpurun_out/r2_fetch64.jsonl 2>&1 && echo run-ok &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d gpurun_out/r2_fetch64_pmc -o run --output-format csv -- ./scripts/micro/fetch64 > gpurun_out/r2_fetch64_pmc.log 2>&1 && echo pmc-ok
