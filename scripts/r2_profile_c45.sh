set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r2p4 BENCH_ARGS="--config c4 --no-derived" bash scripts/r2_profile.sh && TAG=r2p5 BENCH_ARGS="--config c5 --no-derived" bash scripts/r2_profile.sh
