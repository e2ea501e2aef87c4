#!/bin/bash
# The reference bench's workflow end to end at the README's workload
# (bench/run_benchmark.sh: 1 Gbp text, 100k x 20 bp patterns, Block3, sasr 2,
# klts 3) through sview-fmindex_amd/bench_cli.py, warm (blob in the page cache)
# and cold (--drop-caches: the files evicted from the page cache first, as the
# reference's runs drop caches; --direct: O_DIRECT reads), on a disk-backed
# directory.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r3k}
# the candidate directory with the most free space (the files need ~7 GB)
best=""; bestav=0
for c in "$PWD" /var/tmp /tmp; do
  [ -d "$c" ] && [ -w "$c" ] || continue
  av=$(df --output=avail -B1 "$c" | tail -1)
  if [ "$av" -gt "$bestav" ]; then best=$c; bestav=$av; fi
done
D=${CLI_DIR:-$best/.fmx_cli}
df -T "$PWD" /var/tmp /tmp > gpurun_out/${T}_df.txt 2>&1
echo "CLI dir: $D" >> gpurun_out/${T}_df.txt
rm -rf $D && mkdir -p $D
CLI="python sview-fmindex_amd/bench_cli.py"
( timeout -k 10 300 $CLI generate-text -d $D -t 1000000000 -s 7 &&
  timeout -k 10 120 $CLI generate-pattern -d $D -p 20 -n 100000 -s 7 &&
  timeout -k 10 300 $CLI build -d $D -a all -s 2 -k 3 &&
  echo "== warm sview-memory" && timeout -k 10 300 $CLI locate -d $D -a sview-memory &&
  echo "== warm sview-mmap" && timeout -k 10 300 $CLI locate -d $D -a sview-mmap &&
  echo "== cold sview-memory" && timeout -k 10 300 $CLI locate -d $D -a sview-memory --drop-caches &&
  echo "== cold sview-mmap" && timeout -k 10 300 $CLI locate -d $D -a sview-mmap --drop-caches &&
  echo "== cold sview-mmap O_DIRECT" && timeout -k 10 300 $CLI locate -d $D -a sview-mmap --drop-caches --direct &&
  md5sum $D/*-results.txt && wc -l $D/sview-memory-block3-results.txt ) > gpurun_out/${T}_cli.log 2>&1 && echo cli-ok
rc=$?
rm -rf $D
exit $rc
