# rank_pair with the second record's load issued before the first is waited
# for: record-encoding tests, then A/B against the previous build
# (scratch/libfmx_serial.so) on C2, C5, C4, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2dc}
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "record_encodings or readme or golden or every_layout or c1_config" --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo pytest-ok &&
ab() {  # tag-suffix, bench args
  local s=$1; shift
  for i in 1 2; do
    for v in new serial; do
      if [ $v = serial ]; then export FMX_LIB=$GRAFT_REPO_ROOT/scratch/libfmx_serial.so; else unset FMX_LIB; fi
      timeout -k 10 300 python bench.py --no-derived --no-cpu "$@" > gpurun_out/${T}_${s}_${v}_$i.log 2>&1 || return 1
      echo "$s $v run $i $(grep -o '"value": [0-9.e+]*' gpurun_out/${T}_${s}_${v}_$i.log | head -1)"
    done
  done
} &&
ab c2 --min-seconds 0.5 &&
ab c5 --config c5 &&
ab c4 --config c4
