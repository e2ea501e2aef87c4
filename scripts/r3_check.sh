#!/bin/bash
# Grouped tests (opt-in path) + the default bench (launch order) on the current build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grouped.py tests/test_gpu_sharded.py tests/test_gpu.py -k "grouped or sharded or group_launch or fixed_len" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
echo check-ok
