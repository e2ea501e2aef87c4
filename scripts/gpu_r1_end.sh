# End-of-round measurement: smoke, GPU parity tests, C2 (headline, with the
# CPU leg), C3 on one GPU, C4, C5, then the rocprofv3 trace + PMC passes of
# the C2 default (scripts/profile.sh).  Each GPU step has its own limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r1e}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo smoke-ok || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo pytest-ok || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${T}_c2.log 2>&1 && echo c2-ok || exit 1
timeout -k 10 500 python bench.py --config c3 --steps 32 --warmup 4 > gpurun_out/${T}_c3.log 2>&1 && echo c3-ok || exit 1
timeout -k 10 400 python bench.py --config c4 > gpurun_out/${T}_c4.log 2>&1 && echo c4-ok || exit 1
timeout -k 10 600 python bench.py --config c5 --steps 20 --warmup 4 > gpurun_out/${T}_c5.log 2>&1 && echo c5-ok || exit 1
TAG=$T bash scripts/profile.sh
