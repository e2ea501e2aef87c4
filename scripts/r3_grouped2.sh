#!/bin/bash
# Grouped launches after the flush fix: grouped tests, then A/B (2 streams x2,
# one stream), XCD order, larger launches, and a one-stream kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3g4}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grouped.py > $O/pytest_grouped.log 2>&1 || exit $?
echo parity-ok
B="timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout"
for i in 1 2; do
  $B > $O/ab_order_$i.json 2> $O/ab_order_$i.err || exit $?
  FMX_GROUPED=1 $B > $O/ab_grouped_$i.json 2> $O/ab_grouped_$i.err || exit $?
  FMX_GROUPED=1 FMX_GROUPED_XCD=1 $B > $O/ab_grouped_xcd_$i.json 2> $O/ab_grouped_xcd_$i.err || exit $?
done
$B --group 16 > $O/ab_order_g16.json 2> $O/ab_order_g16.err || exit $?
FMX_GROUPED=1 FMX_GROUPED_XCD=1 $B --group 16 > $O/ab_grouped_xcd_g16.json 2> $O/ab_grouped_xcd_g16.err || exit $?
$B --streams 1 > $O/order_s1.json 2> $O/order_s1.err || exit $?
FMX_GROUPED=1 FMX_GROUPED_XCD=1 $B --streams 1 > $O/grouped_xcd_s1.json 2> $O/grouped_xcd_s1.err || exit $?
echo ab-ok
FMX_GROUPED=1 FMX_GROUPED_XCD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_s1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout --streams 1 > $O/trace_s1.log 2>&1 || exit $?
echo trace-ok
