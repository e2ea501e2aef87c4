#!/bin/bash
# Every BASELINE config once on the current build (sharded jobs verified
# job-wide against the oracle).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3cf}
mkdir -p $O
for c in c1 c4; do
  timeout -k 10 400 python -u bench.py --config $c > $O/$c.json 2> $O/$c.err || exit $?
done
for c in c3 c5; do
  timeout -k 10 600 python -u bench.py --config $c --verify-job > $O/$c.json 2> $O/$c.err || exit $?
done
echo configs-ok
