# Sweep (batches per launch, streams) on C2 with 16+ distinct batches, then profile the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1j}
for cfg in "4 2" "8 2" "2 2" "4 1" "8 1" "2 4" "6 2"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu --steps 480 --warmup 24 --batches 24 --group $1 --streams $2 > gpurun_out/${T}_g$1_s$2.log 2>&1 || exit 1
done
echo sweep-done
TAG=$T bash scripts/profile.sh
