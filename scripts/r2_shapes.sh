set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 ./scripts/micro/shapes > gpurun_out/r2_shapes.jsonl 2>&1 && echo shapes-ok &&
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum --kernel-trace -d gpurun_out/r2_shapes_pmc -o run --output-format csv -- ./scripts/micro/shapes > gpurun_out/r2_shapes_pmc.log 2>&1 && echo pmc-ok
