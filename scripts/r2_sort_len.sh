# (Needs the suffix-sorted launch code: git branch exp/suffix-sort; FMX_SORT / FMX_SORT_L do not exist on main.)
# Sorted-launch key length sweep (FMX_SORT_L) on the faithful C2 bench, one
# stream (clean kernel times) and the default two.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2sl}
for L in ${LENS:-0 4 6 8 10}; do
  for S in ${STREAMS:-1 2}; do
    FMX_SORT_L=$L timeout -k 10 300 python bench.py --no-derived --no-cpu --min-seconds 0.3 --streams $S > gpurun_out/${T}_L${L}_s${S}.log 2>&1 || exit 1
    echo "L=$L streams=$S $(grep -o '"value": [0-9.e+]*' gpurun_out/${T}_L${L}_s${S}.log | head -1)"
  done
done
