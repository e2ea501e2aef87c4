# (Needs the suffix-sorted launch code: git branch exp/suffix-sort; FMX_SORT / FMX_SORT_L do not exist on main.)
# Suffix-sorted launches: parity (tests/test_gpu_sorted.py), then the faithful
# bench unsorted (FMX_SORT=0) vs the engine's default (sorted launches) on C2,
# C4 and C5, and the presorted upper bound on C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2so}
timeout -k 10 600 python -u -m pytest tests/test_gpu_sorted.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo pytest-ok || exit 1
for cfg in ${CONFIGS:-c2 c4 c5}; do
  for mode in 0 auto; do
    if [ $mode = auto ]; then unset FMX_SORT; else export FMX_SORT=$mode; fi
    timeout -k 10 400 python bench.py --config $cfg --no-derived --no-cpu --min-seconds 0.5 > gpurun_out/${T}_${cfg}_sort${mode}.log 2>&1 || exit 1
    echo "$cfg sort=$mode $(grep -o '"value": [0-9.e+]*' gpurun_out/${T}_${cfg}_sort${mode}.log | head -1)"
  done
done
unset FMX_SORT
if [ -n "$PRESORT" ]; then
  FMX_SORT=0 timeout -k 10 400 python bench.py --no-derived --no-cpu --min-seconds 0.5 --presorted > gpurun_out/${T}_c2_presorted.log 2>&1 || exit 1
  echo "c2 presorted $(grep -o '"value": [0-9.e+]*' gpurun_out/${T}_c2_presorted.log | head -1)"
fi
