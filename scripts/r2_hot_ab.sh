# A/B of the LF loop's load-hint split (FMX_HOT_ROWS): all plain, the default
# (n >> 20), n >> 18, n >> 22, all non-temporal.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2h}
for h in 0 default 3814 238 18446744073709551615; do
  if [ $h = default ]; then unset FMX_HOT_ROWS; else export FMX_HOT_ROWS=$h; fi
  timeout -k 10 300 python bench.py --no-derived --no-cpu --min-seconds 0.5 > gpurun_out/${T}_$h.log 2>&1 || exit 1
  echo "$h $(grep -o '"value": [0-9.e+]*' gpurun_out/${T}_$h.log | head -1)"
done
