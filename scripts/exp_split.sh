# GPU tests (split default), then A/B: three-kernel split (default) vs fused k_locate (FMX_LOCATE_FUSED=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1o}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo pytest-ok || exit 1
for cfg in "8 2" "8 1" "4 2" "8 3"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu --group $1 --streams $2 > gpurun_out/${T}_split_g$1_s$2.log 2>&1 || exit 1
  FMX_LOCATE_FUSED=1 timeout -k 10 300 python bench.py --no-cpu --group $1 --streams $2 > gpurun_out/${T}_fused_g$1_s$2.log 2>&1 || exit 1
done
timeout -k 10 600 python bench.py --config c5 --steps 20 --warmup 4 --no-cpu > gpurun_out/${T}_split_c5.log 2>&1 && echo c5-ok || exit 1
echo done
