# Paired-chunk occ records: chunk-count micro, the layout tests, then a
# faithful-C2 A/B (paired default vs FMX_OCC_PAIRED=0), alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2pr}
timeout -k 10 120 ./scripts/micro/chunks > gpurun_out/${T}_chunks.jsonl 2>&1 && echo chunks-ok &&
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "paired or readme or golden" --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo pytest-ok &&
for i in 1 2 3; do
  for v in paired plain; do
    if [ $v = plain ]; then export FMX_OCC_PAIRED=0; else unset FMX_OCC_PAIRED; fi
    timeout -k 10 300 python bench.py --no-derived --no-cpu --min-seconds 0.5 ${BENCH_ARGS:-} > gpurun_out/${T}_${v}_$i.log 2>&1 || exit 1
    echo "$v run $i $(grep -o '"value": [0-9.e+]*' gpurun_out/${T}_${v}_$i.log | head -1)"
  done
done
