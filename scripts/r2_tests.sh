set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2g}
timeout -k 10 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo pytest-ok
