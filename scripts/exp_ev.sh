# Timing-method A/B on the C2 default: event sampling, timed-region length, distinct batches.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1m2}
for cfg in "200 2 32" "200 5 32" "800 5 32" "800 5 16" "800 0 32" "2000 5 32"; do
  set -- $cfg
  if [ "$2" = "0" ]; then EV="--no-kernel-timing"; else EV="--event-every $2"; fi
  timeout -k 10 300 python bench.py --no-cpu --steps $1 $EV --batches $3 > gpurun_out/${T}_k$1_e$2_b$3.log 2>&1 || exit 1
done
echo done
