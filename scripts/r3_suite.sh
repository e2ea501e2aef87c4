#!/bin/bash
# Full GPU suite + smoke on the current build, then 8 ranks rehearsed on one
# GPU over gloo (the multi-rank Python path at world 8: plan, broadcast,
# in-step gathers, assembly, weak gather).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3s}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
FMX_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 8 --config c3 --text-len 100000000 \
  --verify-job --min-seconds 0.05 --warmup 0 > $O/gloo8_c3.json 2> $O/gloo8_c3.err || exit $?
FMX_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 8 --text-len 100000000 \
  --min-seconds 0.05 --warmup 0 > $O/gloo8_c2.json 2> $O/gloo8_c2.err || exit $?
echo suite-ok
