# Deep-table size A/B on the C2 default: K = 16 (default budget), 15, 14, 13.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r1lk}
for mb in 0 9000 2300 600; do
  if [ $mb = 0 ]; then unset FMX_DEEP_LUT_MB; else export FMX_DEEP_LUT_MB=$mb; fi
  timeout -k 10 400 python bench.py --no-cpu > gpurun_out/${T}_c2_mb$mb.log 2>&1 && echo c2-mb$mb-ok || exit 1
done
