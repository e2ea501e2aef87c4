# Final-build evidence: kernel trace + stats of the default bench command and
# the PMC passes (scripts/r2_profile.sh), then the default bench line and the
# driver's short command, each on its own.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2f}
TAG=$T bash scripts/r2_profile.sh &&
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.log 2>&1 && echo bench-ok &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench20.log 2>&1 && echo bench20-ok
