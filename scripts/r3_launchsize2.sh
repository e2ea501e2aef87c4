#!/bin/bash
# Experiment: 3.2M vs 6.4M vs 12.8M patterns per grouped launch (batch size varied, 32 per launch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3ls2}
mkdir -p $O
B="timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-blob-layout --no-cpu"
$B > $O/l32x100k.json 2> $O/l32x100k.err || exit $?
$B --patterns 200000 > $O/l32x200k.json 2> $O/l32x200k.err || exit $?
$B --patterns 400000 > $O/l32x400k.json 2> $O/l32x400k.err || exit $?
$B > $O/l32x100k_b.json 2> $O/l32x100k_b.err || exit $?
echo ok
