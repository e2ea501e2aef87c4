#!/bin/bash
# A/B: 14-bit group keys (16,384 bins: C2 grouped by its last 7 symbols, build
# lib/ab/libfmx_k14.so, -DFMX_GROUP_KEY_BITS=14) against the default 12-bit
# keys (6 symbols), alternating; then the grouped parity tests on the k14 build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3k14}
mkdir -p $O
K=sview-fmindex_amd/lib/ab/libfmx_k14.so
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-blob-layout --no-cpu"
for r in 1 2; do
  FMX_LIB=$K $B > $O/k14_c2_$r.json 2> $O/k14_c2_$r.err || exit $?
  $B > $O/def_c2_$r.json 2> $O/def_c2_$r.err || exit $?
done
FMX_LIB=$K $B --streams 1 > $O/k14_c2_s1.json 2> $O/k14_c2_s1.err || exit $?
$B --streams 1 > $O/def_c2_s1.json 2> $O/def_c2_s1.err || exit $?
echo ab-ok
FMX_LIB=$K timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "group" tests > $O/k14_pytest_grouped.log 2>&1 || exit $?
echo k14-tests-ok
