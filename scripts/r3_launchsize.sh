#!/bin/bash
# Experiment: patterns per grouped launch (1.6M default; 3.2M with 200k or 400k batches).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r3ls}
mkdir -p $O
B="timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-blob-layout --no-cpu"
$B > $O/l16x100k.json 2> $O/l16x100k.err || exit $?
$B --patterns 200000 --batches 16 > $O/l16x200k.json 2> $O/l16x200k.err || exit $?
$B --patterns 400000 --batches 8 --group 8 > $O/l8x400k.json 2> $O/l8x400k.err || exit $?
$B --patterns 50000 --batches 64 > $O/l16x50k.json 2> $O/l16x50k.err || exit $?
FMX_GROUPED=0 $B --patterns 200000 --batches 16 > $O/order_l16x200k.json 2> $O/order_l16x200k.err || exit $?
echo ok
