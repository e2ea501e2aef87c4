# The reference bench's workflow end to end at the README's workload
# (bench/run_benchmark.sh: 1 Gbp text, 100k x 20 bp patterns, Block3, sasr 2,
# klts 3), through sview-fmindex_amd/bench_cli.py: generate, build (GPU),
# locate with both loaders; timings as the reference bench prints them.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2k}
D=${TMPDIR:-/tmp}/fmx_cli
rm -rf $D
CLI="python sview-fmindex_amd/bench_cli.py"
( timeout -k 10 300 $CLI generate-text -d $D -t 1000000000 -s 7 &&
  timeout -k 10 120 $CLI generate-pattern -d $D -p 20 -n 100000 -s 7 &&
  timeout -k 10 300 $CLI build -d $D -a all -s 2 -k 3 &&
  timeout -k 10 300 $CLI locate -d $D -a sview-memory &&
  timeout -k 10 300 $CLI locate -d $D -a sview-mmap &&
  timeout -k 10 300 $CLI locate -d $D -a sview-memory --options 63 &&
  md5sum $D/*-results.txt && wc -l $D/sview-memory-block3-results.txt ) > gpurun_out/${T}_cli.log 2>&1 && echo cli-ok
rm -rf $D
