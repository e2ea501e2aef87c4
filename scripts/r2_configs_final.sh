# Whole GPU suite on the current build, then every BASELINE config once
# (faithful index, no derived / CPU legs) for DESIGN §5's table.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2cf}
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && echo smoke-ok &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && echo pytest-ok &&
for c in c1 c2 c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-derived --no-cpu > gpurun_out/${T}_$c.log 2>&1 || exit 1
  echo "$c $(grep -o '"value": [0-9.e+]*' gpurun_out/${T}_$c.log | head -1)"
done
