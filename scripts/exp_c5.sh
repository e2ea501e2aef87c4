# GPU tests, C2 and C5 lines (no CPU leg), C5 phase stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1x}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo pytest-ok || exit 1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${T}_c2.log 2>&1 && echo c2-ok || exit 1
timeout -k 10 600 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu > gpurun_out/${T}_c5.log 2>&1 && echo c5-ok || exit 1
timeout -k 10 600 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu --streams 1 > gpurun_out/${T}_c5_s1.log 2>&1 && echo c5s1-ok || exit 1
STAMP_CFGS="c5:--config=c5 default:" bash scripts/stamps.sh
