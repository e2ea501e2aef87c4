# A/B: batches in flight (--streams), event sampling, 1M-pattern batches.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1j}
for S in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --streams $S > gpurun_out/${T}_s$S.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --streams 2 --event-every 1 > gpurun_out/${T}_s2_ev1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --streams 2 --no-kernel-timing > gpurun_out/${T}_s2_noev.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --patterns 1000000 --streams 1 > gpurun_out/${T}_1m_s1.log 2>&1 || exit 1
echo done
