# One kernel-trace + stats run of a bench command (TAG, BENCH_ARGS from the env).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r2t}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:-} > gpurun_out/${T}_trace.log 2>&1 && echo trace-ok
