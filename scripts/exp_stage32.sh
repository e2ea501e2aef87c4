# 32-bit staging positions: GPU tests, smoke, C2 (x2), C4, C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r1s32}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo pytest-ok || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo smoke-ok || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${T}_c2.log 2>&1 && echo c2-ok || exit 1
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/${T}_c2b.log 2>&1 && echo c2b-ok || exit 1
timeout -k 10 400 python bench.py --no-cpu --config c4 > gpurun_out/${T}_c4.log 2>&1 && echo c4-ok || exit 1
timeout -k 10 600 python bench.py --no-cpu --config c5 --steps 20 --warmup 4 > gpurun_out/${T}_c5.log 2>&1 && echo c5-ok || exit 1
