# GPU tests, then C2 (default) and C5 bench lines without the CPU leg.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1v}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo pytest-ok || exit 1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${T}_c2.log 2>&1 && echo c2-ok || exit 1
timeout -k 10 600 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu > gpurun_out/${T}_c5.log 2>&1 && echo c5-ok || exit 1
