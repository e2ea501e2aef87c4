#!/bin/bash
# Upper bound of grouping a launch's patterns by their last L symbols (host-side
# presort, stable within a key): which key length captures the cache reuse.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3ps}
mkdir -p $O
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout > $O/ps_base.json 2> $O/ps_base.err || exit $?
for L in 4 6 8 10 14; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-blob-layout --presorted --presort-symbols $L > $O/ps_L$L.json 2> $O/ps_L$L.err || exit $?
done
echo presort-ok
