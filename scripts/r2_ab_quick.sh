# Quick faithful-C2 A/B: the current build vs the build in $ALT_LIB (FMX_LIB),
# alternating runs, two each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2ab}
for i in $(seq 1 ${REPS:-2}); do
  for v in cur alt; do
    if [ $v = alt ]; then export FMX_LIB=$ALT_LIB; else unset FMX_LIB; fi
    timeout -k 10 300 python bench.py --no-derived --no-cpu --min-seconds 0.5 ${BENCH_ARGS:-} > gpurun_out/${T}_${v}_$i.log 2>&1 || exit 1
    echo "$v run $i $(grep -o '"value": [0-9.e+]*' gpurun_out/${T}_${v}_$i.log | head -1)"
  done
done
