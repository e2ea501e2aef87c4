#!/bin/bash
# Grouped launches: parity first (every grouped test), then A/B against launch
# order (FMX_GROUPED=0) on the default C2 workload, then a one-stream
# kernel trace of the grouped launch (the cost of each grouping kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3g1}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grouped.py > $O/pytest_grouped.log 2>&1 || exit $?
echo parity-ok
for i in 1 2; do
  FMX_GROUPED=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout > $O/ab_order_$i.json 2> $O/ab_order_$i.err || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout > $O/ab_grouped_$i.json 2> $O/ab_grouped_$i.err || exit $?
done
for s in 1; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout --streams 1 > $O/grouped_s1.json 2> $O/grouped_s1.err || exit $?
  FMX_GROUPED=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout --streams 1 > $O/order_s1.json 2> $O/order_s1.err || exit $?
done
FMX_GROUPED_XCD=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout > $O/ab_grouped_xcd.json 2> $O/ab_grouped_xcd.err || exit $?
FMX_GROUPED_XCD=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout --streams 1 > $O/grouped_xcd_s1.json 2> $O/grouped_xcd_s1.err || exit $?
echo ab-ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_s1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout --streams 1 > $O/trace_s1.log 2>&1 || exit $?
echo trace-ok
if [ -n "$FULL" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $O/pytest_gpu_full.log 2>&1 || exit $?
  echo full-ok
fi
