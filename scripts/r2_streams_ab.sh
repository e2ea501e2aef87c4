# Launch-concurrency A/B on the faithful C2 path: streams x batches per launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2s}
for cfg in "2 8" "1 8" "3 8" "4 8" "2 4" "4 4"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-derived --no-cpu --streams $1 --group $2 --min-seconds 0.5 > gpurun_out/${T}_s$1_g$2.log 2>&1 || exit 1
  echo "streams $1 group $2 $(grep -o '"value": [0-9.e+]*' gpurun_out/${T}_s$1_g$2.log | head -1)"
done
