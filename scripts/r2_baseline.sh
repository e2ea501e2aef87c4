# Round 2 first measurement: the faithful C2 path (options 1 = interleaved occ,
# options 0 = blob layout) on the current build, plus a kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu --options 1 > gpurun_out/r2a_opt1.log 2>&1 && echo opt1-ok &&
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu --options 0 > gpurun_out/r2a_opt0.log 2>&1 && echo opt0-ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2a_trace -o run --output-format csv -- python3 bench.py --steps 200 --warmup 10 --no-cpu --options 1 > gpurun_out/r2a_trace.log 2>&1 && echo trace-ok
