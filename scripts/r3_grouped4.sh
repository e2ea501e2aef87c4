#!/bin/bash
# Grouped launches with the count -> scan -> place passes: grouped tests, A/B
# against launch order (two streams x2, one stream), one-stream trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3g7}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grouped.py > $O/pytest_grouped.log 2>&1 || exit $?
echo parity-ok
B="timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-blob-layout --no-cpu"
for i in 1 2; do
  $B > $O/grouped_$i.json 2> $O/grouped_$i.err || exit $?
  FMX_GROUPED=0 $B > $O/order_$i.json 2> $O/order_$i.err || exit $?
done
$B --streams 1 > $O/grouped_s1.json 2> $O/grouped_s1.err || exit $?
FMX_GROUPED=0 $B --streams 1 > $O/order_s1.json 2> $O/order_s1.err || exit $?
echo ab-ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_s1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout --streams 1 > $O/trace_s1.log 2>&1 || exit $?
echo trace-ok
