#!/bin/bash
# Grouped launches on by default (fixed-length DNA launches >= 131,072 patterns,
# XCD order): grouped tests, then A/B against launch order (FMX_GROUPED=0) for
# 8 and 16 batches per launch, C3, C4 (forced), and a one-stream trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3g6}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grouped.py > $O/pytest_grouped.log 2>&1 || exit $?
echo parity-ok
B="timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-blob-layout"
$B > $O/def_g8_1.json 2> $O/def_g8_1.err || exit $?
for i in 1 2; do
  FMX_GROUPED=0 $B --no-cpu > $O/order_g8_$i.json 2> $O/order_g8_$i.err || exit $?
  $B --no-cpu --group 16 > $O/def_g16_$i.json 2> $O/def_g16_$i.err || exit $?
  FMX_GROUPED=0 $B --no-cpu --group 16 > $O/order_g16_$i.json 2> $O/order_g16_$i.err || exit $?
  $B --no-cpu > $O/def_g8_$((i+1)).json 2> $O/def_g8_$((i+1)).err || exit $?
done
$B --group 16 --streams 3 --no-cpu > $O/def_g16_s3.json 2> $O/def_g16_s3.err || exit $?
echo c2-ok
$B --no-cpu --config c3 --verify-job > $O/def_c3.json 2> $O/def_c3.err || exit $?
FMX_GROUPED=0 $B --no-cpu --config c3 > $O/order_c3.json 2> $O/order_c3.err || exit $?
FMX_GROUPED=1 $B --no-cpu --config c4 > $O/grouped_c4.json 2> $O/grouped_c4.err || exit $?
$B --no-cpu --config c4 > $O/def_c4.json 2> $O/def_c4.err || exit $?
echo c34-ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_s1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout --streams 1 --group 16 > $O/trace_s1.log 2>&1 || exit $?
echo trace-ok
