# GPU tests, then what bounds the C2 default: streams x group sweep, the
# search alone (k_count), and one PMC pass on where k_search's waves wait.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r1oc}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 && echo pytest-ok || exit 1
for sg in "2 8" "1 8" "3 8" "4 8" "4 4" "8 2"; do
  set -- $sg
  timeout -k 10 400 python bench.py --no-cpu --streams $1 --group $2 > gpurun_out/${T}_c2_s$1_g$2.log 2>&1 && echo c2-s$1-g$2-ok || exit 1
done
timeout -k 10 400 python bench.py --no-cpu --count-only > gpurun_out/${T}_c2_count.log 2>&1 && echo count-ok || exit 1
timeout -k 10 120 rocprofv3 -L > gpurun_out/${T}_counters.txt 2>&1 || true
C=""
for c in SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU; do
  grep -q "\b$c\b" gpurun_out/${T}_counters.txt && C="$C $c"
done
echo "pmc:$C"
[ -n "$C" ] && timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${T}_pmc -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/${T}_pmc.log 2>&1 && echo pmc-ok
true
