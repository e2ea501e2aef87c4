#!/bin/bash
# Round 3, first GPU pass: the new GPU tests, the bench-driven tests, the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu.py tests/test_cli.py -k "status_slots or split_timers or status_is_per_stream or load_file or async or sa64_small or builder_and_queries" \
  > $O/t1.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bench.py \
  > $O/t2.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo done
