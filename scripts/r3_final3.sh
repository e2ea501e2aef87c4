#!/bin/bash
# The essentials of scripts/r3_final2.sh: the whole GPU suite, smoke, the
# default bench line and the driver's command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3v}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
echo suite-ok
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || exit $?
echo bench-ok
