set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== host"; nproc; grep -m1 "model name" /proc/cpuinfo; rocm-smi --showproductname 2>/dev/null | head -5
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/${TAG:-r1}_smoke.log 2>&1 && echo smoke-ok &&
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG:-r1}_pytest_gpu.log 2>&1 && echo pytest-ok &&
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --text-len 100000000 --cpu-seconds 3 > gpurun_out/${TAG:-r1}_bench_small.log 2>&1 && echo bench-small-ok &&
timeout -k 10 500 python bench.py --steps 20 --warmup 3 > gpurun_out/${TAG:-r1}_bench.log 2>&1 && echo bench-ok
