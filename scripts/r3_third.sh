#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu.py tests/test_gpu_bench.py -k "status or split_timers or gloo or refused" > $O/t1.log 2>&1 || exit $?
TAG=r3p bash scripts/r3_profile.sh || exit $?
TAG=r3k bash scripts/r3_cli.sh || exit $?
echo done
