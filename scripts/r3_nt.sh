#!/bin/bash
# A/B: non-temporal loads for records only one pattern reads (narrow-interval
# steps, walk steps) — FMX_NT_NARROW=1 build in lib/ab/libfmx_nt.so — against
# the default build, alternating, C2 two streams and one stream, then C5, C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3nt}
mkdir -p $O
NT=sview-fmindex_amd/lib/ab/libfmx_nt.so
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-blob-layout"
FMX_LIB=$NT $B > $O/nt_c2_1.json 2> $O/nt_c2_1.err || exit $?
$B --no-cpu > $O/def_c2_1.json 2> $O/def_c2_1.err || exit $?
FMX_LIB=$NT $B --no-cpu > $O/nt_c2_2.json 2> $O/nt_c2_2.err || exit $?
$B --no-cpu > $O/def_c2_2.json 2> $O/def_c2_2.err || exit $?
FMX_LIB=$NT $B --no-cpu --streams 1 > $O/nt_c2_s1.json 2> $O/nt_c2_s1.err || exit $?
$B --no-cpu --streams 1 > $O/def_c2_s1.json 2> $O/def_c2_s1.err || exit $?
echo c2-ok
for c in c5 c4; do
  FMX_LIB=$NT $B --no-cpu --config $c > $O/nt_$c.json 2> $O/nt_$c.err || exit $?
  $B --no-cpu --config $c > $O/def_$c.json 2> $O/def_$c.err || exit $?
done
echo c45-ok
