# Grouped launches, 16 distinct batches: sweep (batches per launch, streams).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1z}
for cfg in "4 2" "4 3" "2 4" "8 2" "6 2" "3 3"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu --steps 480 --warmup 24 --batches 18 --group $1 --streams $2 > gpurun_out/${T}_g$1_s$2.log 2>&1 || exit 1
done
echo done
