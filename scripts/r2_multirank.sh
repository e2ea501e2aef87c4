# Rehearsal of bench.py's multi-rank path on a 1-GPU box: 2 ranks on cuda:0
# over gloo (weak scaling c2 with the post-run gather; strong scaling c3 with
# the in-step overlapped gather), small text to keep two replicas in HBM.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export FMX_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --text-len 100000000 --steps 40 --warmup 5 > gpurun_out/r2m_c2.log 2>&1 && echo c2-ok &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config c3 --text-len 100000000 --total-patterns 3200000 > gpurun_out/r2m_c3.log 2>&1 && echo c3-ok
