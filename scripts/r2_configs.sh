# GPU tests, then the faithful bench on C4 and C5 (with parity + CPU legs).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo pytest-ok &&
timeout -k 10 600 python bench.py --config c4 --no-derived > gpurun_out/${T}_c4.log 2>&1 && echo c4-ok &&
timeout -k 10 900 python bench.py --config c5 --no-derived > gpurun_out/${T}_c5.log 2>&1 && echo c5-ok
