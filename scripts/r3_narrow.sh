#!/bin/bash
# A/B: 8-B grouped search records (NarrowRec, the new default build) against
# the round-3 final build (lib/ab/libfmx_r3t.so, 16-B records), and 256
# batches per launch (lib/ab/libfmx_g256.so, -DFMX_MAX_GROUP=256, narrow
# records) — alternating, C2 two streams and one stream; then the grouped
# parity tests on the g256 build and the whole GPU suite on the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3n}
mkdir -p $O
OLD=sview-fmindex_amd/lib/ab/libfmx_r3t.so
G=sview-fmindex_amd/lib/ab/libfmx_g256.so
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-blob-layout --no-cpu"
for r in 1 2; do
  FMX_LIB=$OLD $B > $O/old_c2_$r.json 2> $O/old_c2_$r.err || exit $?
  $B > $O/new_c2_$r.json 2> $O/new_c2_$r.err || exit $?
  FMX_LIB=$G $B --group 256 > $O/g256_c2_$r.json 2> $O/g256_c2_$r.err || exit $?
done
FMX_LIB=$OLD $B --streams 1 > $O/old_c2_s1.json 2> $O/old_c2_s1.err || exit $?
$B --streams 1 > $O/new_c2_s1.json 2> $O/new_c2_s1.err || exit $?
FMX_LIB=$G $B --streams 1 --group 256 > $O/g256_c2_s1.json 2> $O/g256_c2_s1.err || exit $?
echo ab-ok
FMX_LIB=$G timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "group" tests > $O/g256_pytest_grouped.log 2>&1 || exit $?
echo g256-tests-ok
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
echo suite-ok
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo smoke-ok
