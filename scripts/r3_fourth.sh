#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_cli.py tests/test_gpu_sharded.py > $O/t1.log 2>&1 || exit $?
TAG=r3cf bash scripts/r3_configs.sh || exit $?
echo done
