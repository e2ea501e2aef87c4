# Final check of the committed build: smoke, C2 default bench with the CPU
# leg, kernel trace + stats of the same command.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r1f2}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo smoke-ok &&
timeout -k 10 400 python bench.py > gpurun_out/${T}_c2.log 2>&1 && echo c2-ok &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o run --output-format csv -- python3 bench.py > gpurun_out/${T}_trace.log 2>&1 && echo trace-ok
