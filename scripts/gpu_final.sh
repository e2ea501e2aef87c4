# Round measurement: smoke, C2 (headline, with the CPU leg), C4, C5, then the
# rocprofv3 kernel trace + PMC passes of the C2 default (scripts/profile.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r1f}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo smoke-ok || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${T}_c2.log 2>&1 && echo c2-ok || exit 1
timeout -k 10 400 python bench.py --config c4 > gpurun_out/${T}_c4.log 2>&1 && echo c4-ok || exit 1
timeout -k 10 600 python bench.py --config c5 --steps 20 --warmup 4 > gpurun_out/${T}_c5.log 2>&1 && echo c5-ok || exit 1
[ -z "$SKIP_PROFILE" ] && TAG=$T bash scripts/profile.sh; true
