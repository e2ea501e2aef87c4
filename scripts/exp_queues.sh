# A/B: HIP hardware queues per process (GPU_MAX_HW_QUEUES, default 4) x batches in flight.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1u}
for Q in 4 8 16; do
  for S in 8 16; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --steps 400 --warmup 20 --no-cpu --streams $S --batches 16 > gpurun_out/${T}_q${Q}_s$S.log 2>&1 || exit 1
  done
done
echo done
