# Super occ records: the record-encoding tests, then a faithful-C2 A/B
# (super default vs FMX_OCC_SUPER=0 (paired) vs plain), alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2su}
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "record_encodings or readme or golden or every_layout" --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo pytest-ok &&
for i in 1 2; do
  for v in super paired plain; do
    case $v in
      super) unset FMX_OCC_SUPER FMX_OCC_PAIRED ;;
      paired) export FMX_OCC_SUPER=0; unset FMX_OCC_PAIRED ;;
      plain) export FMX_OCC_SUPER=0 FMX_OCC_PAIRED=0 ;;
    esac
    timeout -k 10 300 python bench.py --no-derived --no-cpu --min-seconds 0.5 ${BENCH_ARGS:-} > gpurun_out/${T}_${v}_$i.log 2>&1 || exit 1
    echo "$v run $i $(grep -o '"value": [0-9.e+]*' gpurun_out/${T}_${v}_$i.log | head -1)"
  done
done
