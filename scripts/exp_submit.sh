# A/B: native job-queue submission vs one Python call per step; streams; distinct batches.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1r}
for S in 1 2 4; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu --streams $S > gpurun_out/${T}_nat_s$S.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu --streams 2 --submit python > gpurun_out/${T}_py_s2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu --streams 2 --batches 2 > gpurun_out/${T}_nat_s2_nb2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu --streams 4 --no-kernel-timing > gpurun_out/${T}_nat_s4_noev.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu --streams 8 > gpurun_out/${T}_nat_s8.log 2>&1 || exit 1
echo done
