# A/B: split (k_search + k_emit) vs fused (k_locate) locate kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1m}
for S in 1 2; do
  FMX_LOCATE_SPLIT=1 timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --streams $S > gpurun_out/${T}_split_s$S.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --streams $S > gpurun_out/${T}_fused_s$S.log 2>&1 || exit 1
done
FMX_LOCATE_SPLIT=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --patterns 1000000 --streams 1 > gpurun_out/${T}_split_1m.log 2>&1 || exit 1
FMX_LOCATE_SPLIT=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --patterns 1000000 --streams 2 > gpurun_out/${T}_split_1m_s2.log 2>&1 || exit 1
echo done
