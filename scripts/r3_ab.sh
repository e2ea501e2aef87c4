#!/bin/bash
# A/B on the default bench workload: status-word completion events on/off
# (FMX_STATUS_EVENTS), alternating; then one-stream launches of 4/8/16 batches
# (k_search alone per launch: ramp/drain overhead vs launch size).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3b}
mkdir -p $O
for i in 1 2 3; do
  for ev in 1 0; do
    FMX_STATUS_EVENTS=$ev timeout -k 10 300 python -u bench.py --no-blob-layout --no-cpu > $O/ab_ev${ev}_$i.json 2> $O/ab_ev${ev}_$i.err || exit $?
  done
done
for g in 4 8 16; do
  timeout -k 10 300 python -u bench.py --no-blob-layout --no-cpu --streams 1 --group $g --kernel-launches 12 > $O/tail_g$g.json 2> $O/tail_g$g.err || exit $?
done
echo ab-ok
