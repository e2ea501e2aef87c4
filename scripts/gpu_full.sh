# Everything for one measurement point: build, smoke, GPU tests, C2 bench with
# the CPU leg, 1M-pattern bench, rocprofv3 trace + PMC groups.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1}
bash scripts/gpu_check.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --patterns 1000000 > gpurun_out/${T}_bench_1m.log 2>&1 && echo 1m-ok || exit 1
bash scripts/profile.sh
