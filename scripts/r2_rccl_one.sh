# bench.py's RCCL path on a one-GPU box: one rank under torchrun with the
# process group started anyway (FMX_BENCH_DIST=1, backend nccl = RCCL), so the
# collectives, barriers and SlabGather all-gathers run through RCCL: c2 (weak
# scaling, post-run gather, derived leg aggregated over ranks) at full size
# and c3 (strong scaling, in-step gathers overlapped on a comm stream).
# Then the two-rank gloo rehearsal (scripts/r2_multirank.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2r}
export FMX_BENCH_DIST=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/${T}_c2.log 2>&1 && echo c2-ok &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 1 --config c3 --no-derived --no-cpu > gpurun_out/${T}_c3.log 2>&1 && echo c3-ok &&
unset FMX_BENCH_DIST &&
bash scripts/r2_multirank.sh
