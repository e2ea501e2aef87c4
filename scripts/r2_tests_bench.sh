# All GPU tests, then the default bench without its derived/CPU legs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2i}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo pytest-ok &&
timeout -k 10 300 python bench.py --no-derived --no-cpu > gpurun_out/${T}_bench.log 2>&1 && echo bench-ok &&
timeout -k 10 300 python bench.py --no-derived --no-cpu --steps 20 --warmup 5 > gpurun_out/${T}_bench20.log 2>&1 && echo bench20-ok
