# A/B of FMX_HINT_FIXED_LEN (bench default = hint on) after the GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r1fx}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo smoke-ok || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo pytest-ok || exit 1
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/${T}_c2_fixed.log 2>&1 && echo c2f-ok || exit 1
timeout -k 10 400 python bench.py --no-cpu --no-fixed-len > gpurun_out/${T}_c2_var.log 2>&1 && echo c2v-ok || exit 1
timeout -k 10 400 python bench.py --no-cpu --config c4 > gpurun_out/${T}_c4_fixed.log 2>&1 && echo c4f-ok || exit 1
timeout -k 10 600 python bench.py --no-cpu --config c5 --steps 20 --warmup 4 > gpurun_out/${T}_c5_fixed.log 2>&1 && echo c5f-ok || exit 1
timeout -k 10 600 python bench.py --no-cpu --config c5 --steps 20 --warmup 4 --no-fixed-len > gpurun_out/${T}_c5_var.log 2>&1 && echo c5v-ok || exit 1
