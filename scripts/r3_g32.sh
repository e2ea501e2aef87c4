#!/bin/bash
# 32 batches per launch: group-launch tests (several launches per call), then
# C2 16 vs 32 per launch, C3 16 vs 32 per launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3g32}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grouped.py tests/test_gpu.py -k "grouped or group_launch or fixed_len or queue" > $O/pytest.log 2>&1 || exit $?
echo parity-ok
B="timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-blob-layout --no-cpu"
for i in 1 2; do
  $B --group 16 > $O/c2_g16_$i.json 2> $O/c2_g16_$i.err || exit $?
  $B --group 32 > $O/c2_g32_$i.json 2> $O/c2_g32_$i.err || exit $?
done
FMX_GROUPED=0 $B --group 32 > $O/c2_order_g32.json 2> $O/c2_order_g32.err || exit $?
$B --group 32 --batches 64 > $O/c2_g32_b64.json 2> $O/c2_g32_b64.err || exit $?
$B --config c3 --group 16 > $O/c3_g16.json 2> $O/c3_g16.err || exit $?
$B --config c3 --group 32 --verify-job > $O/c3_g32.json 2> $O/c3_g32.err || exit $?
echo ab-ok
