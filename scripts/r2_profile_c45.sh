set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${T4:-r2p4} BENCH_ARGS="--config c4 --no-derived" bash scripts/r2_profile.sh && TAG=${T5:-r2p5} BENCH_ARGS="--config c5 --no-derived" bash scripts/r2_profile.sh
