# Per-wave phase timeline of k_locate (diagnostic build, see csrc/Makefile `stamps`).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1}
# (libfmx_stamps.so is built here beforehand: make -C sview-fmindex_amd/csrc stamps)
export FMX_LIB=$GRAFT_REPO_ROOT/sview-fmindex_amd/lib/libfmx_stamps.so
for cfg in ${STAMP_CFGS:-"default:" "1m:--patterns 1000000"} ; do
  name=${cfg%%:*}; args=${cfg#*:}
  extra=""
  if [ "$name" = "k12" ]; then export FMX_DEEP_LUT_MB=8192; fi
  FMX_STAMPS_OUT=gpurun_out/${T}_stamps_$name.json timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu $args > gpurun_out/${T}_stamps_$name.log 2>&1 && echo stamps-$name-ok || exit 1
done
