# Diagnostic: the search alone (k_count) vs the fused count+locate kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1l}
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --streams 1 --count-only --event-every 1 > gpurun_out/${T}_cnt_s1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --streams 1 --count-only --event-every 1 --patterns 1000000 > gpurun_out/${T}_cnt_1m.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --streams 1 --event-every 1 --patterns 1000000 > gpurun_out/${T}_loc_1m.log 2>&1 || exit 1
echo done
