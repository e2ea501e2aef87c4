#!/bin/bash
# C1 (1 Mbp, 1,000-pattern batches: launch- and latency-bound): batches per
# launch x streams in flight.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3c1
mkdir -p $O
for rep in 1 2; do
  for gs in "8 2" "16 2" "16 4" "8 4" "16 8"; do
    set -- $gs
    timeout -k 10 300 python -u bench.py --config c1 --group $1 --streams $2 --no-cpu --no-blob-layout \
      > $O/g$1_s$2_$rep.json 2> $O/g$1_s$2_$rep.err || exit 1
  done
done
echo sweep-ok
