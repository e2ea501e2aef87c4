#!/bin/bash
# A/B on one box: the round-2 final build (ab_r2/, commit 90dce67, untracked copy)
# vs this build on C1 (launch-bound) and C4; then the persistent-grid k_search
# (FMX_SEARCH_PERSISTENT=1) vs one workgroup per tile on C2, one and two streams.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3ab2
mkdir -p $O
run() {  # name, dir, args...
  local name=$1 dir=$2; shift 2
  ( cd $dir && timeout -k 10 300 python -u bench.py "$@" ) > $O/$name.json 2> $O/$name.err || exit 1
}
FMX_SEARCH_PERSISTENT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu.py -k "group or queue or fixed_len or split_timers" > $O/persistent_pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  run c1_r2_$i ab_r2 --config c1 --no-derived --no-cpu || exit 1
  run c1_r3_$i . --config c1 --no-cpu --no-blob-layout || exit 1
done
for i in 1 2; do
  run c4_r2_$i ab_r2 --config c4 --no-derived --no-cpu || exit 1
  run c4_r3_$i . --config c4 --no-cpu --no-blob-layout || exit 1
done
for i in 1 2 3; do
  FMX_SEARCH_PERSISTENT=0 run c2_s1_p0_$i . --no-cpu --no-blob-layout --streams 1 || exit 1
  FMX_SEARCH_PERSISTENT=1 run c2_s1_p1_$i . --no-cpu --no-blob-layout --streams 1 || exit 1
done
for i in 1 2; do
  FMX_SEARCH_PERSISTENT=0 run c2_s2_p0_$i . --no-cpu --no-blob-layout || exit 1
  FMX_SEARCH_PERSISTENT=1 run c2_s2_p1_$i . --no-cpu --no-blob-layout || exit 1
done
echo ab2-ok
