# XCD-partition upper bound: the faithful C2 bench with each launch's
# patterns arranged so that tile t (dispatched to XCD t % 8) holds only
# patterns of class t % 8 (a function of their last 3 symbols), vs the
# default random arrangement; one and two streams.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2x}
for S in 1 2; do
  for mode in plain xcd; do
    extra=""; [ $mode = xcd ] && extra="--xcd-partitioned"
    timeout -k 10 300 python bench.py --no-derived --no-cpu --min-seconds 0.5 --streams $S $extra > gpurun_out/${T}_${mode}_s$S.log 2>&1 || exit 1
    echo "$mode streams=$S $(grep -o '"value": [0-9.e+]*' gpurun_out/${T}_${mode}_s$S.log | head -1)"
  done
done
