# GPU tests, then A/B of FMX_TILE_PAIRS (k_search2) on C2, C4, C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r1pr}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo pytest-ok || exit 1
for p in 0 1; do
  FMX_TILE_PAIRS=$p timeout -k 10 400 python bench.py --no-cpu > gpurun_out/${T}_c2_p$p.log 2>&1 && echo c2-p$p-ok || exit 1
done
for p in 0 1; do
  FMX_TILE_PAIRS=$p timeout -k 10 400 python bench.py --no-cpu --config c4 > gpurun_out/${T}_c4_p$p.log 2>&1 && echo c4-p$p-ok || exit 1
  FMX_TILE_PAIRS=$p timeout -k 10 600 python bench.py --no-cpu --config c5 --steps 20 --warmup 4 > gpurun_out/${T}_c5_p$p.log 2>&1 && echo c5-p$p-ok || exit 1
done
