# A/B of the current build against $ALT_LIB on one config, REPS alternations
# (BENCH_ARGS, TAG from the env).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2ab}
for i in $(seq 1 ${REPS:-4}); do
  for v in new alt; do
    if [ $v = alt ]; then export FMX_LIB=$GRAFT_REPO_ROOT/$ALT_LIB; else unset FMX_LIB; fi
    timeout -k 10 300 python bench.py --no-derived --no-cpu ${BENCH_ARGS:-} > gpurun_out/${T}_${v}_$i.log 2>&1 || exit 1
    echo "$v run $i $(grep -o '"value": [0-9.e+]*' gpurun_out/${T}_${v}_$i.log | head -1)"
  done
done
