# GPU parity tests, then the faithful C2 bench (options 1 and 0) and a kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r2b}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo pytest-ok &&
timeout -k 10 300 python bench.py --steps 400 --warmup 10 --no-cpu --options 1 > gpurun_out/${T}_opt1.log 2>&1 && echo opt1-ok &&
timeout -k 10 300 python bench.py --steps 400 --warmup 10 --no-cpu --options 0 > gpurun_out/${T}_opt0.log 2>&1 && echo opt0-ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o run --output-format csv -- python3 bench.py --steps 200 --warmup 10 --no-cpu --options 1 > gpurun_out/${T}_trace.log 2>&1 && echo trace-ok
