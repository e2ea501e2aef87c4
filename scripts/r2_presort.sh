set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-derived --no-cpu --min-seconds 0.5 > gpurun_out/r2ps_base.log 2>&1 && echo "base $(grep -o '"value": [0-9.e+]*' gpurun_out/r2ps_base.log | head -1)" &&
timeout -k 10 300 python bench.py --no-derived --no-cpu --min-seconds 0.5 --presorted > gpurun_out/r2ps_sorted.log 2>&1 && echo "presorted $(grep -o '"value": [0-9.e+]*' gpurun_out/r2ps_sorted.log | head -1)" &&
timeout -k 10 300 python bench.py --no-derived --no-cpu --min-seconds 0.5 --presorted --streams 1 > gpurun_out/r2ps_sorted1.log 2>&1 && echo "presorted 1 stream $(grep -o '"value": [0-9.e+]*' gpurun_out/r2ps_sorted1.log | head -1)"
