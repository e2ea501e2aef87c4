# GPU tests, then grouped launches (batches per launch x streams) on C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1y}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo pytest-ok || exit 1
for cfg in "8 2" "8 4" "4 2" "4 4" "1 8" "8 1"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu --steps 400 --warmup 20 --group $1 --streams $2 > gpurun_out/${T}_g$1_s$2.log 2>&1 || exit 1
done
echo done
