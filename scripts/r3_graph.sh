#!/bin/bash
# HIP-graph replay of whole passes vs per-launch host calls: C1 (launch-bound)
# and C2 (GPU-bound); C1 with the CPU leg (32 batches checked bit-exact).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 300 python -u bench.py --config c1 --graph > $O/c1_graph_cpu.json 2> $O/c1_graph_cpu.err || exit 1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --config c1 --no-cpu --no-blob-layout > $O/c1_plain_$rep.json 2> $O/c1_plain_$rep.err || exit 1
  timeout -k 10 300 python -u bench.py --config c1 --graph --no-cpu --no-blob-layout > $O/c1_graph_$rep.json 2> $O/c1_graph_$rep.err || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu --no-blob-layout > $O/c2_plain_$rep.json 2> $O/c2_plain_$rep.err || exit 1
  timeout -k 10 300 python -u bench.py --graph --no-cpu --no-blob-layout > $O/c2_graph_$rep.json 2> $O/c2_graph_$rep.err || exit 1
done
echo graph-ok
