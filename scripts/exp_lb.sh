# GPU tests, C2 default x2, C2 single-batch launches, C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1i}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo pytest-ok || exit 1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${T}_c2a.log 2>&1 && echo c2-ok || exit 1
timeout -k 10 300 python bench.py --no-cpu --steps 400 > gpurun_out/${T}_c2b.log 2>&1 && echo c2b-ok || exit 1
timeout -k 10 300 python bench.py --no-cpu --group 1 --streams 8 > gpurun_out/${T}_c2g1.log 2>&1 && echo c2g1-ok || exit 1
timeout -k 10 600 python bench.py --config c5 --steps 20 --warmup 4 --no-cpu > gpurun_out/${T}_c5.log 2>&1 && echo c5-ok || exit 1
