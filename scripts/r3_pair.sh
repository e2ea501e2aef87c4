#!/bin/bash
# Two patterns per lane in the grouped search (FMX_GROUPED_PAIR=1): grouped
# tests with it, then A/B against one per lane, and a one-stream trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3p2}
mkdir -p $O
FMX_GROUPED_PAIR=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grouped.py > $O/pytest_grouped_pair.log 2>&1 || exit $?
echo parity-ok
B="timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-blob-layout --no-cpu"
for i in 1 2; do
  $B > $O/one_$i.json 2> $O/one_$i.err || exit $?
  FMX_GROUPED_PAIR=1 $B > $O/pair_$i.json 2> $O/pair_$i.err || exit $?
done
$B --streams 1 > $O/one_s1.json 2> $O/one_s1.err || exit $?
FMX_GROUPED_PAIR=1 $B --streams 1 > $O/pair_s1.json 2> $O/pair_s1.err || exit $?
FMX_GROUPED_PAIR=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-blob-layout > $O/pair_cpu.json 2> $O/pair_cpu.err || exit $?
echo ab-ok
FMX_GROUPED_PAIR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_s1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout --streams 1 > $O/trace_s1.log 2>&1 || exit $?
echo trace-ok
