#!/bin/bash
# 128 batches per launch: group-launch and grouped tests, then C2 default
# (128 per launch) vs 32 per launch vs launch order, C3 default with the job verified.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3g128}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grouped.py tests/test_gpu.py -k "grouped or group_launch or fixed_len or queue" > $O/pytest.log 2>&1 || exit $?
echo parity-ok
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-blob-layout"
$B > $O/c2_default.json 2> $O/c2_default.err || exit $?
$B --no-cpu --group 32 > $O/c2_g32.json 2> $O/c2_g32.err || exit $?
$B --no-cpu > $O/c2_default2.json 2> $O/c2_default2.err || exit $?
FMX_GROUPED=0 $B --no-cpu > $O/c2_order_g128.json 2> $O/c2_order_g128.err || exit $?
$B --no-cpu --config c3 --verify-job > $O/c3.json 2> $O/c3.err || exit $?
echo ab-ok
