# One GPU call: smoke, GPU parity tests, C2 bench (with the CPU leg), kernel
# trace + stats, phase stamps.  Every GPU step has its own time limit and the
# steps are chained with && (the first failure ends the call).
#   TAG=r1x SKIP_TESTS=1 STAMPS=1 bash scripts/gpu_round.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r1}
BA=${BENCH_ARGS:-""}
ok=0
run() { echo "== $1"; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo smoke-ok || exit 1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo pytest-ok || exit 1
fi
timeout -k 10 400 python bench.py --steps 50 --warmup 5 $BA > gpurun_out/${T}_bench.log 2>&1 && echo bench-ok || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu $BA > gpurun_out/${T}_trace.log 2>&1 && echo trace-ok || exit 1
if [ -n "$STAMPS" ]; then
  export FMX_LIB=$GRAFT_REPO_ROOT/sview-fmindex_amd/lib/libfmx_stamps.so
  FMX_STAMPS_OUT=gpurun_out/${T}_stamps.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu $BA > gpurun_out/${T}_stamps.log 2>&1 && echo stamps-ok || exit 1
  unset FMX_LIB
fi
if [ -n "$EXTRA" ]; then
  eval "$EXTRA"
fi
