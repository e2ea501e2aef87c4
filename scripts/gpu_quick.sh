# Fast iteration: build, GPU parity tests, default bench (no CPU leg), then
# the scan-limit / options A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r1}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/${T}_build.log 2>&1 && echo build-ok &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo pytest-ok &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/${T}_bench.log 2>&1 && echo bench-ok &&
bash scripts/gpu_scan_ab.sh
