# A/B of the row-context scan limit (FMX_SCAN_ROWS) and of the options on C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1}
for s in ${SCANS:-8 16 64}; do
  FMX_SCAN_ROWS=$s timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/${T}_scan$s.log 2>&1 && echo scan$s-ok || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --options 15 > gpurun_out/${T}_opt15.log 2>&1 && echo opt15-ok || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --options 17 > gpurun_out/${T}_opt17.log 2>&1 && echo opt17-ok || exit 1
