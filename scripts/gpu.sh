#!/bin/bash
# One parameterised driver for the GPU box (run through gpurun from the repo
# root):  bash scripts/gpu.sh TAG STEP [STEP ...]
#   suite    pytest -m gpu (the driver's round-end command, verbose, 120 s per test)
#   smoke    __graft_entry__.smoke()
#   stress   scripts/stress_grouped.py for 150 s (grouped launches vs the oracle)
#   bench    python bench.py (defaults) and the driver's command (--steps 20 --warmup 5)
#   single   bench.py --single-batch only (one 100k batch per call)
#   trace    rocprofv3 --kernel-trace --stats on bench.py --streams 1 and on the default command
#   pmc      rocprofv3 PMC passes (FETCH/WRITE size, memory-side requests) on bench.py --streams 1
#            (PMC_CONFIG=c4 / c5 / ...: that config instead of the default c2)
#   configs  bench.py --config c1 / c3 / c4 / c5
#   cli      bench_cli.py: generate, build, locate warm / cold / O_DIRECT (the README workload)
#   c5ab     C5 grouped at 16 per launch (whole job verified) and in launch order
#   grouped  pytest tests/test_gpu_grouped.py only
#   presort  bench.py --presorted (L = 8, 12) and the same command without (upper bound of a longer key)
#   refineab k_group_refine on / off, alternating twice
#   c1ab     C1 at a 2 s and a 0.2 s timed region
#   knobs    headline A/B: no XCD order, 3 streams, 128 x 4 streams, two patterns per lane
#   freshreps  test_every_layout_grouped[4-2-*] in 12 fresh processes, then the grouped file 3 times (FMX_DEBUG=1)
#   countab  the count pass decoding the key's bytes only (this build) vs the whole pattern
#            (build_ab/libfmx_fullcount.so via FMX_LIB), alternating twice
#   wsortab  the grouped search's in-workgroup sort by the next symbols on / off (FMX_GROUPED_WSORT=0), twice
#   emitab   k_emit / k_group_tiles with 4 tiles per workgroup (this build) vs 1 (build_ab/libfmx_e1.so
#            via FMX_LIB, built with -DFMX_EMIT_TILES=1), alternating twice
#   gloo2    bench.py --gpus 2 over gloo on the one GPU (the multi-rank path: in-step gathers)
#   c4presort  C4 at 8 and 256 batches per launch (launch order) and presorted by the last 3-6 residues
#   c4group  C4 grouped (last 3 residues) with and without the refine pass, vs launch order, 256 per launch
#   c4rec    C4 with symbol-mask / paired-chunk / plain occ records (FMX_OCC_ONEHOT=0, FMX_OCC_PAIRED=0), twice
#   launchab C1 on this build vs build_ab/libfmx_prev.so; single batch with 4 vs 1 tiles per k_emit workgroup
#   clitrace the sview-memory loader's stage times (FMX_LOAD_TRACE=1), warm
#   sizesweep  C2's shape on 100 / 250 / 500 Mbp texts, grouped vs launch order (the grouping size floor)
#   c1streams  C1 at its default 256 batches per launch on 2 / 4 / 8 streams
#   c1sweep  C1 at 16 / 64 / 256 batches per launch x 2 / 8 streams (+ 256 in launch order)
#   rawab    C2 grouped with packed vs id-only records (FMX_GROUPED_RAW=1), alternating twice
#   singletrace  rocprofv3 kernel trace of the single-batch leg (one 100k batch per call)
#   fusedtest  only tests/test_gpu_fused.py (the fused launch, k_locate)
#   chainab  C2 (grouped) ended by k_emit_chain vs k_group_tiles + k_emit (FMX_EMIT_CHAIN=0), alternating twice
#   psweep   C2 at 100k / 200k / 400k patterns per batch (256 batches per launch: 25.6 / 51.2 / 102.4 M per launch)
#   groupedtest  tests/test_gpu_grouped.py and tests/test_gpu_fused.py only
#   c4mega   C4 at 1,024 batches per launch: launch order vs grouped (and + refine), and launch order at 256
#   c4ab     C4 at 1,024 per launch: grouped (default) vs launch order, alternating twice
#   streamab C2 on 2 vs 3 streams at 1,024 batches per launch, alternating twice
#   foldab   C2: k_emit's own tile sums vs k_scan first (FMX_EMIT_FOLD=0), and the refine pass, alternating twice
#   slotab   C2 with the per-XCD sub-runs (8 slots) vs one run per key (sview-fmindex_amd/lib/ab/libfmx_s1.so),
#            alternating twice, then a one-stream kernel trace of each
#   megab    C2 at 256 / 512 / 1,024 batches per launch (one grouped launch over 2-4 kernel-argument groups), twice
#   megatest test_gpu_mega.py (1,024-batch grouped launch, two-stream fused launches), test_gpu_fused.py,
#            test_gpu_provenance.py
#   prevab   this build vs lib/ab/libfmx_prev.so (the build before), C2 and C4, alternating twice
#   sampledab  one-row results from the search's sampled row vs the walk (lib/ab/libfmx_walk.so): C2, C4, single
#   c4knobs  C4: in-workgroup sort off, XCD deal off, vs default, alternating twice
#   c4trace  one-stream kernel trace of C4
#   thresh   C3 slabs of 5 M / 2.5 M / 1.6 M / 1.25 M patterns: grouped vs launch order
#   tabab    C2 on this build vs lib/ab/libfmx_prev.so (the previous commit), alternating twice
#   c4       bench.py --config c4 (with the CPU leg)
#   records  the record-encoding, every-layout, golden and README GPU tests
#   m2048ab  C2 at 2,048 batches per launch (the FMX_MAX_MEGA=2048 build) vs 1,024, alternating twice
#   tcc      the TCC hit/miss PMC pass alone (C2, shipped launch shape)
#   c4walk   C4 with vs without the walk line in its multi-line records, alternating twice
#   c4pair   C4 one vs two patterns per lane in the grouped search, alternating twice; C2 two per lane once
#   shapes   the per-rank shapes of C3 (10 M / N) and C5 (1 M / N) at N = 1, 2, 4, 8 on one GPU
#   gloo2g   bench.py --gpus 2 over gloo on the one GPU with --gather all and --gather counts
#   ticketab the fused launch's tickets vs workgroup index order: single batch and C1, alternating twice
#   fusedab  the fused launch vs the two-kernel path (FMX_FUSED=0): single batch, C1, C4, alternating twice;
#            then the single-batch kernel trace of the fused build
# Every step has its own time limit; the first failing step ends the run.
# Output: gpurun_out/TAG/*.
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run NAME SECONDS CMD...: stdout+stderr to $OUT/NAME.log
    local name=$1 secs=$2; shift 2
    echo "[$(date +%T)] $name: $*"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] $name rc=$rc"
    tail -3 "$OUT/$name.log"
    return $rc
}
shrink() {  # a profiler pass's output, small enough to come back (gpurun returns <= 64 MiB)
    find "$1" -name "*kernel_trace.csv" -delete
    find "$1" -name "*counter_collection.csv" -exec gzip -f {} \;
    return 0
}
for step in "$@"; do
    case $step in
        suite) run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1 ;;
        smoke) run smoke 300 python -u -c 'import __graft_entry__ as g; g.smoke()' || exit 1 ;;
        stress) run stress 240 python -u scripts/stress_grouped.py --seconds 150 || exit 1 ;;
        bench)
            run bench_default 400 python -u bench.py || exit 1
            run bench_driver 400 python -u bench.py --steps 20 --warmup 5 || exit 1 ;;
        single) run bench_single 300 python -u bench.py --single-batch-only || exit 1 ;;
        c5ab)  # C5 grouped (id-only records) vs launch order, 8 and 16 batches per launch
            run bench_c5_g16 600 python -u bench.py --config c5 --group 16 --verify-job || exit 1
            FMX_GROUPED=0 run bench_c5_lo 600 python -u bench.py --config c5 || exit 1 ;;
        grouped) run pytest_grouped 600 python -u -m pytest tests/test_gpu_grouped.py -x -v --timeout 300 --timeout-method thread || exit 1 ;;
        presort)  # upper bound of a longer sort key: each launch group pre-sorted by its last L symbols
            for L in 8 12; do
                run "bench_presort$L" 400 python -u bench.py --presorted --presort-symbols $L --no-cpu --no-blob-layout \
                    --no-single-batch || exit 1
            done
            run bench_presort_ref 400 python -u bench.py --no-cpu --no-blob-layout --no-single-batch || exit 1 ;;
        refineab)  # per-key refine sort on / off, alternating, same box
            for r in 1 2; do
                run "bench_refine_on$r" 400 python -u bench.py --no-cpu --no-blob-layout --no-single-batch || exit 1
                FMX_GROUP_REFINE=0 run "bench_refine_off$r" 400 python -u bench.py --no-cpu --no-blob-layout \
                    --no-single-batch || exit 1
            done ;;
        c1ab)  # C1 (launch-bound) at a 2 s and a 0.2 s timed region
            run bench_c1_2s 300 python -u bench.py --config c1 --no-cpu || exit 1
            run bench_c1_02s 300 python -u bench.py --config c1 --no-cpu --min-seconds 0.2 || exit 1 ;;
        knobs)  # launch-shape and grouping knobs on the headline (no CPU / blob / single legs), same box
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            run knob_ref 300 $B || exit 1
            FMX_GROUPED_XCD=0 run knob_noxcd 300 $B || exit 1
            run knob_s3 300 $B --streams 3 || exit 1
            run knob_g128_s4 300 $B --group 128 --streams 4 || exit 1
            FMX_GROUPED_PAIR=1 run knob_pair 300 $B || exit 1
            run knob_ref2 300 $B || exit 1 ;;
        freshreps)
            for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
                FMX_DEBUG=1 run "rep_$i" 120 python -u -m pytest tests/test_gpu_grouped.py -x -q --timeout 60 \
                    --timeout-method thread -k "every_layout_grouped and 4-2" || exit 1
            done
            for i in 1 2 3; do
                FMX_DEBUG=1 run "full_$i" 200 python -u -m pytest tests/test_gpu_grouped.py -x -q --timeout 60 \
                    --timeout-method thread || exit 1
            done ;;
        countab)
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "count_key_$r" 300 $B || exit 1
                FMX_LIB=$PWD/build_ab/libfmx_fullcount.so run "count_full_$r" 300 $B || exit 1
            done ;;
        wsortab)
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "wsort_on_$r" 300 $B || exit 1
                FMX_GROUPED_WSORT=0 run "wsort_off_$r" 300 $B || exit 1
            done
            run wsort_on_c4 400 python -u bench.py --config c4 --no-cpu || exit 1
            FMX_GROUPED_WSORT=0 run wsort_off_c4 400 python -u bench.py --config c4 --no-cpu || exit 1 ;;
        emitab)
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "emit_e4_$r" 300 $B || exit 1
                FMX_LIB=$PWD/build_ab/libfmx_e1.so run "emit_e1_$r" 300 $B || exit 1
            done
            FMX_LIB=$PWD/build_ab/libfmx_e1.so run emit_e1_c1 300 python -u bench.py --config c1 --no-cpu || exit 1
            run emit_e4_c1 300 python -u bench.py --config c1 --no-cpu || exit 1 ;;
        gloo2) FMX_BENCH_BACKEND=gloo run bench_gloo2 600 python -u bench.py --gpus 2 --no-cpu || exit 1 ;;
        c4presort)  # C4 at 256 batches per launch in launch order, and the upper bound of sorting by the last L residues
            B="python -u bench.py --config c4 --no-cpu --no-blob-layout --group 256"
            run c4_g8 400 python -u bench.py --config c4 --no-cpu --no-blob-layout || exit 1
            run c4_g256 400 $B || exit 1
            for L in 3 4 5 6; do
                run "c4_presort$L" 400 $B --presorted --presort-symbols $L || exit 1
            done ;;
        c4group)  # C4 grouped at 256 batches per launch: key = last 3 residues, + refine by the next 3
            B="python -u bench.py --config c4 --no-blob-layout --group 256"
            FMX_GROUPED=1 FMX_GROUP_REFINE_MIN=1 run c4_grouped_refine 500 $B || exit 1
            FMX_GROUPED=1 run c4_grouped 500 $B --no-cpu || exit 1
            run c4_g256_lo 500 $B --no-cpu || exit 1
            FMX_GROUPED=1 FMX_GROUP_REFINE_MIN=1 run c4_grouped_refine2 500 $B --no-cpu || exit 1 ;;
        c4rec)  # C4's occ record encoding: symbol masks (3 lines per block, the default) vs paired chunks vs plain
            B="python -u bench.py --config c4 --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "c4_masks_$r" 400 $B || exit 1
                FMX_OCC_ONEHOT=0 run "c4_paired_$r" 400 $B || exit 1
                FMX_OCC_ONEHOT=0 FMX_OCC_PAIRED=0 run "c4_plain_$r" 400 $B || exit 1
            done ;;
        launchab)  # the launch path's host cost: this build vs build_ab/libfmx_prev.so (C1, launch-bound) and
            # one tile per k_emit workgroup (build_ab/libfmx_e1.so) on the single-batch leg, alternating twice
            for r in 1 2; do
                run "c1_new_$r" 300 python -u bench.py --config c1 --no-cpu || exit 1
                FMX_LIB=$PWD/build_ab/libfmx_prev.so run "c1_prev_$r" 300 python -u bench.py --config c1 --no-cpu || exit 1
                run "single_e4_$r" 300 python -u bench.py --single-batch-only || exit 1
                FMX_LIB=$PWD/build_ab/libfmx_e1.so run "single_e1_$r" 300 python -u bench.py --single-batch-only || exit 1
            done ;;
        clitrace)  # the sview-memory load's stages (FMX_LOAD_TRACE=1): file -> host memory, host -> HBM (pinned stage)
            D=$PWD/.fmx_cli; rm -rf "$D"; mkdir -p "$D"; CLI="python sview-fmindex_amd/bench_cli.py"
            run clitrace_generate 420 bash -c "$CLI generate-text -d $D -t 1000000000 -s 7 && \
                $CLI generate-pattern -d $D -p 20 -n 100000 -s 7 && $CLI build -d $D -a all -s 2 -k 3" || exit 1
            FMX_LOAD_TRACE=1 run clitrace_locate 600 bash -c "$CLI locate -d $D -a sview-memory && \
                $CLI locate -d $D -a sview-memory && $CLI locate -d $D -a sview-mmap" || exit 1
            rm -rf "$D" ;;
        sizesweep)  # where grouping starts to pay: C2's shape on 100 / 250 / 500 Mbp texts, grouped vs launch order
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for n in ${SIZES:-100000000 250000000 500000000}; do
                FMX_GROUPED=1 run "size_${n}_grouped" 300 $B --text-len $n || exit 1
                FMX_GROUPED=0 run "size_${n}_lo" 300 $B --text-len $n || exit 1
            done ;;
        c1streams)  # C1's new default shape (256 batches per launch, launch order) on 2 / 4 / 8 streams
            for st in 2 4 8; do
                run "c1_s${st}" 300 python -u bench.py --config c1 --no-cpu --streams $st || exit 1
            done ;;
        c1sweep)  # C1 (1,000-pattern batches, launch-bound): batches per launch x streams beyond round 3's 8/16
            for g in 16 64 256; do
                for st in 2 8; do
                    run "c1_g${g}_s${st}" 300 python -u bench.py --config c1 --no-cpu --group $g --streams $st || exit 1
                done
            done
            FMX_GROUPED=0 run c1_g256_s2_lo 300 python -u bench.py --config c1 --no-cpu --group 256 --streams 2 || exit 1
            run c1_g16_s8_again 300 python -u bench.py --config c1 --no-cpu --group 16 --streams 8 || exit 1 ;;
        rawab)  # C2 grouped with id-only records (no symbol decode in the place pass) vs packed, alternating
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "packed_$r" 300 $B || exit 1
                FMX_GROUPED_RAW=1 run "raw_$r" 300 $B || exit 1
            done ;;
        fusedtest) run pytest_fused 600 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 300 \
                --timeout-method thread || exit 1 ;;
        chainab)
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "chain_on_$r" 300 $B || exit 1
                FMX_EMIT_CHAIN=0 run "chain_off_$r" 300 $B || exit 1
            done ;;
        groupedtest) run pytest_grouped 900 python -u -m pytest tests/test_gpu_grouped.py tests/test_gpu_fused.py -x -v \
                --timeout 300 --timeout-method thread || exit 1 ;;
        slotab)
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "slots8_$r" 400 $B || exit 1
                FMX_LIB=$PWD/sview-fmindex_amd/lib/ab/libfmx_s1.so run "slots1_$r" 400 $B || exit 1
            done
            run slots8_trace 400 rocprofv3 --kernel-trace --stats -d "$OUT/s8" -o run --output-format csv -- \
                python3 -u bench.py --streams 1 --no-cpu --no-blob-layout --no-single-batch || exit 1
            shrink "$OUT/s8"
            FMX_LIB=$PWD/sview-fmindex_amd/lib/ab/libfmx_s1.so run slots1_trace 400 rocprofv3 --kernel-trace --stats \
                -d "$OUT/s1" -o run --output-format csv -- \
                python3 -u bench.py --streams 1 --no-cpu --no-blob-layout --no-single-batch || exit 1
            shrink "$OUT/s1" ;;
        c4mega)  # C4 at 1,024 batches per launch: launch order vs grouped (keyed on 3 residues; + refine)
            B="python -u bench.py --config c4 --no-cpu --no-blob-layout --no-single-batch"
            FMX_GROUPED=0 run c4_lo_g256 400 $B --group 256 || exit 1
            FMX_GROUPED=0 run c4_lo_g1024 400 $B --group 1024 || exit 1
            FMX_GROUPED=1 run c4_grouped_g1024 400 $B --group 1024 || exit 1
            FMX_GROUPED=1 FMX_GROUP_REFINE_MIN=1 run c4_refine_g1024 400 $B --group 1024 || exit 1 ;;
        c4ab)  # C4 at 1,024 per launch: grouped (the default) vs launch order (FMX_GROUPED=0), alternating twice
            B="python -u bench.py --config c4 --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "c4_grouped_$r" 400 $B || exit 1
                FMX_GROUPED=0 run "c4_order_$r" 400 $B || exit 1
            done ;;
        streamab)  # C2 on 2 vs 3 streams (1,024 batches per launch), alternating twice
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "streams2_$r" 400 $B || exit 1
                run "streams3_$r" 400 $B --streams 3 || exit 1
            done ;;
        foldab)  # C2: k_emit's own tile sums vs k_scan first (FMX_EMIT_FOLD=0); the refine pass on (all launches)
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "fold_$r" 400 $B || exit 1
                FMX_EMIT_FOLD=0 run "scan_$r" 400 $B || exit 1
                FMX_GROUP_REFINE_MIN=1 run "refine_$r" 400 $B || exit 1
            done ;;
        megab)
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                for g in 256 512 1024; do run "mega_g${g}_$r" 400 $B --group $g || exit 1; done
            done ;;
        psweep)
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for p in 100000 200000 400000; do run "patterns_$p" 300 $B --patterns $p || exit 1; done ;;
        fusedab)
            for r in 1 2; do
                run "single_fused_$r" 300 python -u bench.py --single-batch-only || exit 1
                FMX_FUSED=0 run "single_split_$r" 300 python -u bench.py --single-batch-only || exit 1
                run "c1_fused_$r" 300 python -u bench.py --config c1 --no-cpu || exit 1
                FMX_FUSED=0 run "c1_split_$r" 300 python -u bench.py --config c1 --no-cpu || exit 1
                run "c4_fused_$r" 400 python -u bench.py --config c4 --no-cpu --no-blob-layout --no-single-batch || exit 1
                FMX_FUSED=0 run "c4_split_$r" 400 python -u bench.py --config c4 --no-cpu --no-blob-layout \
                    --no-single-batch || exit 1
            done
            run single_trace_fused 400 rocprofv3 --kernel-trace --stats -d "$OUT/single" -o run --output-format csv -- \
                python3 -u bench.py --single-batch-only || exit 1 ;;
        singletrace)  # where one 100k batch per call spends its time
            run single_trace 400 rocprofv3 --kernel-trace --stats -d "$OUT/single" -o run --output-format csv -- \
                python3 -u bench.py --single-batch-only || exit 1 ;;
        trace)
            run trace_one_stream 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace1" -o run --output-format csv -- \
                python3 -u bench.py --streams 1 --no-cpu --no-blob-layout --no-single-batch || exit 1
            run trace_default 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace2" -o run --output-format csv -- \
                python3 -u bench.py --no-cpu || exit 1
            shrink "$OUT/trace1"; shrink "$OUT/trace2" ;;
        pmcw)  # the WRITE_SIZE pass alone (a pass that hangs can be re-run on its own)
            P="--config ${PMC_CONFIG:-c2} --streams 1 --no-cpu --no-blob-layout --no-single-batch --min-seconds 0.5"
            run pmc_write 170 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run \
                --output-format csv -- python3 -u bench.py $P || exit 1
            shrink "$OUT/pmc_write" ;;
        pmcfe)  # the FETCH_SIZE and request-split passes
            P="--config ${PMC_CONFIG:-c2} --streams 1 --no-cpu --no-blob-layout --no-single-batch --min-seconds 0.5"
            run pmc_fetch 170 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run \
                --output-format csv -- python3 -u bench.py $P || exit 1
            shrink "$OUT/pmc_fetch"
            run pmc_ea 170 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
                --kernel-trace -d "$OUT/pmc_ea" -o run --output-format csv -- python3 -u bench.py $P || exit 1
            shrink "$OUT/pmc_ea" ;;
        pmc)
            P="--config ${PMC_CONFIG:-c2} --streams 1 --no-cpu --no-blob-layout --no-single-batch --min-seconds 0.5"
            run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run \
                --output-format csv -- python3 -u bench.py $P || exit 1
            run pmc_ea 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
                --kernel-trace -d "$OUT/pmc_ea" -o run --output-format csv -- python3 -u bench.py $P || exit 1
            run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run \
                --output-format csv -- python3 -u bench.py $P || exit 1
            [ "${PMC_SKIP_TCC:-0}" = 1 ] && continue
            run pmc_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$OUT/pmc_tcc" -o run \
                --output-format csv -- python3 -u bench.py $P || exit 1 ;;
        pmcsq)  # one SQ pass (instruction mix and wait cycles per kernel), C2 and C4
            for c in c2 c4; do
                P="--config $c --streams 1 --no-cpu --no-blob-layout --no-single-batch --min-seconds 0.5"
                run "pmc_sq_$c" 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU \
                    SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace \
                    -d "$OUT/pmc_sq_$c" -o run --output-format csv -- python3 -u bench.py $P || exit 1
                shrink "$OUT/pmc_sq_$c"
            done ;;
        pmctlb)  # first-level address translation hits / misses per kernel, C2 and C4
            for c in c2 c4; do
                P="--config $c --streams 1 --no-cpu --no-blob-layout --no-single-batch --min-seconds 0.5"
                run "pmc_tlb_$c" 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum \
                    --kernel-trace -d "$OUT/pmc_tlb_$c" -o run --output-format csv -- python3 -u bench.py $P || exit 1
                shrink "$OUT/pmc_tlb_$c"
            done ;;
        walkab2)  # C4 walk-line records (default) vs without, now that most one-row results skip the walk
            B="--config c4 --no-cpu --no-blob-layout --no-single-batch"
            for i in 1 2 3; do
                run "c4_walk_$i" 400 python -u bench.py $B || exit 1
                FMX_OCC_WALK=0 run "c4_nowalk_$i" 400 python -u bench.py $B || exit 1
            done ;;
        contigab)  # records in physically contiguous memory (FMX_OCC_CONTIG=1) vs hipMalloc's, same box, alternating;
            # then the translation pass on C4 with them
            B="--no-cpu --no-blob-layout --no-single-batch"
            for i in 1 2; do
                for c in c4 c2; do
                    run "${c}_heap_$i" 400 python -u bench.py --config $c $B || exit 1
                    FMX_OCC_CONTIG=1 run "${c}_contig_$i" 400 python -u bench.py --config $c $B || exit 1
                done
            done
            P="--config c4 --streams 1 --no-cpu --no-blob-layout --no-single-batch --min-seconds 0.5"
            FMX_OCC_CONTIG=1 run pmc_tlb_c4_contig 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_HIT_sum \
                TCP_UTCL1_TRANSLATION_MISS_sum --kernel-trace -d "$OUT/pmc_tlb_c4_contig" -o run --output-format csv \
                -- python3 -u bench.py $P || exit 1
            shrink "$OUT/pmc_tlb_c4_contig" ;;
        configs)
            for c in c1 c3 c4 c5; do
                run "bench_$c" 600 python -u bench.py --config $c || exit 1
            done ;;
        cli)  # the reference bench's workflow end to end at the README workload, warm and cold
            D=$PWD/.fmx_cli; rm -rf "$D"; mkdir -p "$D"; CLI="python sview-fmindex_amd/bench_cli.py"
            run cli_generate 420 bash -c "$CLI generate-text -d $D -t 1000000000 -s 7 && \
                $CLI generate-pattern -d $D -p 20 -n 100000 -s 7 && $CLI build -d $D -a all -s 2 -k 3" || exit 1
            run cli_locate 900 bash -c "$CLI locate -d $D -a sview-memory && $CLI locate -d $D -a sview-mmap && \
                $CLI locate -d $D -a sview-memory --drop-caches && $CLI locate -d $D -a sview-mmap --drop-caches && \
                $CLI locate -d $D -a sview-mmap --drop-caches --direct && md5sum $D/*-results.txt" || exit 1
            rm -rf "$D" ;;
        megatest)  # round 6: the 1,024-batch grouped launch and the two-stream fused launches vs the oracle,
            # the fused file, full-size blob provenance (GPU builder vs the oracle builder's SHA-256)
            run pytest_mega 900 python -u -m pytest tests/test_gpu_mega.py tests/test_gpu_fused.py \
                tests/test_gpu_provenance.py -x -v --timeout 300 --timeout-method thread || exit 1 ;;
        ticketab)  # the fused launch's per-batch tickets (default) vs workgroup index order (FMX_FUSED_TICKETS=0):
            # single batch and C1 (fused launches), alternating twice
            for r in 1 2; do
                run "single_tk_$r" 300 python -u bench.py --single-batch-only || exit 1
                FMX_FUSED_TICKETS=0 run "single_idx_$r" 300 python -u bench.py --single-batch-only || exit 1
                run "c1_tk_$r" 300 python -u bench.py --config c1 --no-cpu || exit 1
                FMX_FUSED_TICKETS=0 run "c1_idx_$r" 300 python -u bench.py --config c1 --no-cpu || exit 1
            done ;;
        c4pair)  # C4 (grouped, 1,024 per launch): one vs two patterns per lane in the grouped search
            # (FMX_GROUPED_PAIR=1), alternating twice; then C2 with two per lane once
            B="python -u bench.py --config c4 --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "c4_k1_$r" 400 $B || exit 1
                FMX_GROUPED_PAIR=1 run "c4_k2_$r" 400 $B || exit 1
            done
            FMX_GROUPED_PAIR=1 run c2_k2 400 python -u bench.py --no-cpu --no-blob-layout --no-single-batch || exit 1
            run c2_k1 400 python -u bench.py --no-cpu --no-blob-layout --no-single-batch || exit 1 ;;
        shapes)  # the per-rank shapes JobPlan deals at N = 1/2/4/8, each run on this one GPU (no gathers):
            # C3 10 M / N and C5 1 M / N patterns; and C3's N = 8 slab in launch order
            B="--no-cpu --no-blob-layout --no-single-batch"
            for t in 10000000 5000000 2500000 1250000; do
                run "c3_t$t" 400 python -u bench.py --config c3 --total-patterns $t $B || exit 1
            done
            FMX_GROUPED=0 run c3_t1250000_lo 400 python -u bench.py --config c3 --total-patterns 1250000 $B || exit 1
            for t in 1000000 500000 250000 125000; do
                run "c5_t$t" 500 python -u bench.py --config c5 --total-patterns $t $B || exit 1
            done ;;
        shapes2)  # the per-rank shapes of gathered strong runs: two launch groups per rank (--strong-groups 2)
            B="--no-cpu --no-blob-layout --no-single-batch --strong-groups 2"
            for t in 10000000 5000000 2500000 1250000; do
                run "c3sg2_t$t" 400 python -u bench.py --config c3 --total-patterns $t $B || exit 1
            done
            for t in 500000 250000 125000; do
                run "c5sg2_t$t" 500 python -u bench.py --config c5 --total-patterns $t $B || exit 1
            done ;;
        sgab)  # same box, alternating: one vs two launch groups per rank at the N = 1 and N = 8 shapes
            B="--no-cpu --no-blob-layout --no-single-batch"
            for i in 1 2; do
                for sg in 1 2; do
                    run "c3_sg${sg}_t10000000_$i" 400 python -u bench.py --config c3 $B --strong-groups $sg || exit 1
                    run "c3_sg${sg}_t1250000_$i" 400 python -u bench.py --config c3 --total-patterns 1250000 $B \
                        --strong-groups $sg || exit 1
                    run "c5_sg${sg}_t1000000_$i" 500 python -u bench.py --config c5 $B --strong-groups $sg || exit 1
                done
            done ;;
        c5trace)  # C5's per-rank slabs at N = 4 and 8 under the kernel trace (why 250 k runs slower than 125 k)
            B="--no-cpu --no-blob-layout --no-single-batch"
            for t in 250000 125000; do
                run "c5trace_t$t" 400 rocprofv3 --kernel-trace --stats -d "$OUT/c5trace_$t" -o run --output-format csv -- \
                    python3 -u bench.py --config c5 --total-patterns $t $B || exit 1
                shrink "$OUT/c5trace_$t"
            done ;;
        gloo2g)  # two gloo ranks on the one GPU, c2 weak, both gather policies
            FMX_BENCH_BACKEND=gloo run bench_gloo2_all 600 python -u bench.py --gpus 2 --no-cpu --gather all || exit 1
            FMX_BENCH_BACKEND=gloo run bench_gloo2_counts 600 python -u bench.py --gpus 2 --no-cpu --gather counts \
                || exit 1 ;;
        c4walk)  # C4 (grouped, 1,024 per launch): multi-line symbol masks with a walk line (FMX_OCC_WALK=1,
            # 4 x 128 B per 64 rows) vs without (3 x 128 B: the walk reads the planes, then the symbol's unit),
            # alternating twice; then one-stream kernel traces of each
            B="python -u bench.py --config c4 --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                FMX_OCC_WALK=0 run "c4_nowalk_$r" 400 $B || exit 1
                FMX_OCC_WALK=1 run "c4_walk_$r" 400 $B || exit 1
            done ;;
        m2048ab)  # C2: 2,048 batches per grouped launch (sview-fmindex_amd/lib/ab/libfmx_m2048.so, -DFMX_MAX_MEGA=2048)
            # vs the shipped 1,024, alternating twice (same box)
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "g1024_$r" 400 $B || exit 1
                FMX_LIB=$PWD/sview-fmindex_amd/lib/ab/libfmx_m2048.so run "g2048_$r" 400 $B --group 2048 || exit 1
            done ;;
        tcc)  # the L2 hit / miss pass alone on C2 at the shipped launch shape (PMC_CONFIG for another config)
            P="--config ${PMC_CONFIG:-c2} --streams 1 --no-cpu --no-blob-layout --no-single-batch --min-seconds 0.5"
            run pmc_tcc 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$OUT/pmc_tcc" -o run \
                --output-format csv -- python3 -u bench.py $P || exit 1
            shrink "$OUT/pmc_tcc" ;;
        thresh)  # where grouping starts to pay for C3's per-rank slabs: grouped (FMX_GROUPED=1) vs launch order
            # (FMX_GROUPED=0) at 5 M / 2.5 M / 1.6 M / 1.25 M patterns per launch (256 batches)
            B="--no-cpu --no-blob-layout --no-single-batch"
            for t in 5000000 2500000 1600000 1250000; do
                FMX_GROUPED=1 run "c3g_t$t" 400 python -u bench.py --config c3 --total-patterns $t $B || exit 1
                FMX_GROUPED=0 run "c3o_t$t" 400 python -u bench.py --config c3 --total-patterns $t $B || exit 1
            done ;;
        tabab)  # C2: this build (compact GroupTab copies) vs sview-fmindex_amd/lib/ab/libfmx_prev.so, alternating twice
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "tab_new_$r" 400 $B || exit 1
                FMX_LIB=$PWD/sview-fmindex_amd/lib/ab/libfmx_prev.so run "tab_prev_$r" 400 $B || exit 1
            done ;;
        c4)  run bench_c4 400 python -u bench.py --config c4 || exit 1 ;;
        paritycore) run pytest_core 1100 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_mega.py \
                tests/test_gpu_grouped.py tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread || exit 1 ;;
        r6tests) run pytest_r6 900 python -u -m pytest tests/test_gpu_mega.py tests/test_gpu_bench.py -x -v \
                --timeout 300 --timeout-method thread || exit 1 ;;
        records) run pytest_records 600 python -u -m pytest tests/test_gpu.py -k "record or every_layout or golden or readme" \
                -x -v --timeout 300 --timeout-method thread || exit 1 ;;
        c4knobs)  # C4 grouped: the in-workgroup sort off (FMX_GROUPED_WSORT=0) and the XCD deal off (FMX_GROUPED_XCD=0)
            # vs the default, alternating twice
            B="python -u bench.py --config c4 --no-cpu --no-blob-layout --no-single-batch"
            for r in 1 2; do
                run "c4_def_$r" 400 $B || exit 1
                FMX_GROUPED_WSORT=0 run "c4_nowsort_$r" 400 $B || exit 1
                FMX_GROUPED_XCD=0 run "c4_noxcd_$r" 400 $B || exit 1
            done ;;
        c4trace)  # one-stream kernel trace of C4 (where a grouped launch's time goes)
            run c4_trace 400 rocprofv3 --kernel-trace --stats -d "$OUT/c4trace" -o run --output-format csv -- \
                python3 -u bench.py --config c4 --streams 1 --no-cpu --no-blob-layout --no-single-batch || exit 1
            shrink "$OUT/c4trace" ;;
        sampledab)  # one-row results located from the search's latest sampled row (this build) vs by the walk
            # (sview-fmindex_amd/lib/ab/libfmx_walk.so, -DFMX_SAMPLED_ROW=0): C2, C4, single batch, alternating twice
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            W=$PWD/sview-fmindex_amd/lib/ab/libfmx_walk.so
            for r in 1 2; do
                run "sr_c2_$r" 400 $B || exit 1
                FMX_LIB=$W run "walk_c2_$r" 400 $B || exit 1
                run "sr_c4_$r" 400 $B --config c4 || exit 1
                FMX_LIB=$W run "walk_c4_$r" 400 $B --config c4 || exit 1
                run "sr_single_$r" 300 python -u bench.py --single-batch-only || exit 1
                FMX_LIB=$W run "walk_single_$r" 300 python -u bench.py --single-batch-only || exit 1
            done ;;
        prevab)  # this tree's libfmx.so vs sview-fmindex_amd/lib/ab/libfmx_prev.so (the build before), C2 and C4,
            # alternating twice
            B="python -u bench.py --no-cpu --no-blob-layout --no-single-batch"
            X=$PWD/sview-fmindex_amd/lib/ab/libfmx_prev.so
            for r in 1 2; do
                run "cur_c2_$r" 400 $B || exit 1
                FMX_LIB=$X run "prev_c2_$r" 400 $B || exit 1
                run "cur_c4_$r" 400 $B --config c4 || exit 1
                FMX_LIB=$X run "prev_c4_$r" 400 $B --config c4 || exit 1
            done ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "ALL_OK"
