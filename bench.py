#!/usr/bin/env python3
"""Benchmark: patterns/sec (count + locate) on BASELINE.json's headline config.

Default workload (BASELINE.json configs[1], "C2"): 1 Gbp uniform ACGT text,
symbols ACGTN (N = wildcard, sigma 5), layout u32 / Block3<u64> /
EncodingTable, SA sampling 2, k-mer table k = 3; 100,000 x 20 bp patterns cut
from the text at uniform random starts (bench/src/generate.rs:105-113, cold
ratio 1.0), per GPU.  `--config c1|c3|c4|c5` selects the other BASELINE
configs (c3/c5: one job sharded over the GPUs, results all-gathered).

The headline runs the reference's algorithm on the reference's index: the
blob, re-laid out at load as one interleaved record per occ block
(FMX_OCC_INTERLEAVED: the same planes and checkpoints), the blob's k = 3
seed, the LF loop over the bit planes, the sr = 2 sampled-SA walk.  The same
workload over the blob's arrays exactly as laid out (`--options 0`, the
reference's zero-copy view, bwm/mod.rs:157-189) is measured after it and
reported as "blob_layout".  `--derived` adds the derived-index leg (deep
K-mer table, full SA, text: ~147 GB of HBM at C2), outside SURVEY §8.

One step = one full count+locate pass over one batch: k-mer seed + LF loop
for every pattern, the walk of every occurrence row, output offsets and all
locations written to that batch's own HBM outputs.  Many steps' batches
share one kernel launch (fmx_locate_group_async; `--group`, at most 2,048):
C2 and C4 1,024 per (grouped) launch, C1 and C3 256, C5 8.  Launches
alternate over two streams, each stream with its own launch group of
distinct batches (C2: 2,048 distinct batches, ~20 GB of patterns and
outputs), so that no pass finds the previous pass's index lines in cache.
Inputs (text, blob, index, patterns)
are resident in HBM before the timed region.  The K steps are timed as a
whole and repeated until the timed region lasts at least --min-seconds
(0.2 s): a few-hundred-microsecond region is noise.

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) this process
is one rank; `--gpus N` without torchrun starts the N ranks itself (a
torchrun child process, started before this process touches the GPU).  With
RCCL every rank needs a GPU of its own: N above the visible GPUs is refused.
Each rank builds its own replica of the blob on its GPU (deterministic).
c2 (weak scaling): each rank runs its own batches with no collective in the
timed region; every batch's counts and locations are then all-gathered.
c3/c5 (strong scaling): the job is dealt out by distributed.JobPlan — rank r
takes a contiguous slab of the job, cut into the same number of near-equal
batches on every rank — and each launch group's results are gathered with
ONE all_gather_into_tensor into an exactly sized slab (distributed.JobGather)
on a communication stream while the next launch computes, inside the timed
step (`value`); the compute alone is timed too (gather.value_compute_only).
The job's flat (offsets, locations) is assembled on the device afterwards.

Also reported: the roofline (algorithmic bytes per pattern x patterns/s per
GPU; plus k_search alone on one stream, HIP events around that kernel), the
CPU baseline (the oracle restatement on this host's usable cores, rank 0),
and a bit-exact check of the GPU results against it (`--verify-job`: every
pattern of a sharded job).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# G dependent random 128-B line reads/s over a 0.5-1 GB buffer (the C2 occ records: 1 GB), 0.5-2 M
# chains: 52-54 (profiles/r2_footprint.jsonl, profiles/r2_shapes.jsonl; scripts/micro/shapes.hip).
RANDOM_LINE_CEILING = 52.0
METRIC = "patterns/sec (count+locate), 1 Gbp text / 20 bp patterns, 1/2/4/8 MI355X"
FAITHFUL = 1  # FMX_OCC_INTERLEAVED: the blob's own planes and checkpoints, one record per block
BLOB_LAYOUT = 0  # FMX_OCC_BLOB: the blob's arrays as laid out (the reference's zero-copy view)
DERIVED = 63  # + deep K-mer table, full SA, text, row contexts, single-row entries

ACGTN = [b"Aa", b"Cc", b"Gg", b"Tt", b"Nn"]
AMINO = b"ACDEFGHIKLMNPQRSTVWY"
CONFIGS = {
    # BASELINE.json configs[0]: the reference's CPU-runnable plumbing case (T is the wildcard)
    # (1,000-pattern batches: launch-bound below ~64 batches per launch; 256 per launch on 2 streams in
    # launch order runs 8.17e9 vs 1.1e9 at round 3's 16 x 8 — the 1 Mbp index lives in cache, so the
    # engine does not group it; profiles/r5/r5p_*)
    "c1": dict(text_len=1_000_000, alphabet=b"ACGT", symbols=[b"Aa", b"Cc", b"Gg", b"Tt"], pos=4, planes=2,
               vec=64, k=3, sr=2, patterns=1_000, m=20, total=0, group=256, streams=2,
               desc="C1: 1 Mbp ACGT, 1,000 x 20 bp, u32/Block2<u64>, sr 2, k 3"),
    # configs[1]: the headline (metric quoted on it).  1,024 batches per launch (one launch group
    # per stream, 2,048 distinct batches): a grouped launch of 102.4 M patterns shares more of its
    # first LF steps than one of 51.2 M or 25.6 M (4.04 vs 3.92 vs 3.60-3.66e9, profiles/r5/r5y_mega_*;
    # and 25.6 M more than 12.8 M, 3.2 M, 1.6 M or 0.8 M: 3.42 vs 3.28 vs 2.84 vs ~2.7 vs ~2.6e9 in
    # round 3; launch order ~2.58; profiles/r3/narrow, profiles/r3/grouped/r3ls2, r3g32, r3g6)
    "c2": dict(text_len=1_000_000_000, alphabet=b"ACGT", symbols=ACGTN, pos=4, planes=3, vec=64, k=3, sr=2,
               patterns=100_000, m=20, total=0, group=1024,
               desc="C2: 1 Gbp ACGT (ACGTN, N wildcard), 100,000 x 20 bp per GPU, u32/Block3<u64>, sr 2, k 3"),
    # configs[2]: 10 M patterns sharded over the GPUs
    "c3": dict(text_len=1_000_000_000, alphabet=b"ACGT", symbols=ACGTN, pos=4, planes=3, vec=64, k=3, sr=2,
               patterns=100_000, m=20, total=10_000_000, group=256,
               desc="C3: 1 Gbp ACGT, 10,000,000 x 20 bp sharded over the GPUs, u32/Block3<u64>, sr 2, k 3"),
    # configs[3]: large-alphabet occ path.  1,024 batches per launch, grouped (the engine's default from
    # 2^26 patterns for a 3-residue key): 3.68e9 vs 3.42-3.45 in launch order at 256 or 1,024 per launch
    # (profiles/r5/r5c4m_*); at 256 per launch grouping lost (3.29 vs 3.59e9, r5f_*: the permutation's
    # scattered writes cost more than 25.6 M patterns share)
    "c4": dict(text_len=1_000_000_000, alphabet=AMINO, symbols=[bytes([c, c + 32]) for c in AMINO] + [b"Xx"],
               pos=4, planes=5, vec=64, k=3, sr=2, patterns=100_000, m=12, total=0, group=1024,
               desc="C4: 1 G-residue protein text (20 aa + X wildcard), 100,000 x 12 aa, u32/Block5<u64>, sr 2, k 3"),
    # configs[4]: long patterns, wide blocks, u64 positions (1 M patterns over the GPUs)
    "c5": dict(text_len=3_000_000_000, alphabet=b"ACGT", symbols=ACGTN, pos=8, planes=3, vec=128, k=3, sr=2,
               patterns=100_000, m=150, total=1_000_000,
               desc="C5: 3 Gbp ACGT, 1,000,000 x 150 bp sharded over the GPUs, u64/Block3<u128>, sr 2, k 3"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one GPU each (default: WORLD_SIZE under torchrun, else 1); without torchrun, "
                         "N > 1 starts the N ranks itself")
    ap.add_argument("--steps", type=int, default=0,
                    help="batches per timed pass (default: 800, or the whole sharded job for c3/c5)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--text-len", type=int, default=0, help="override the config's text length")
    ap.add_argument("--patterns", type=int, default=0, help="patterns per batch (target, for sharded jobs)")
    ap.add_argument("--total-patterns", type=int, default=-1,
                    help="> 0: one global job of this many patterns dealt out over the GPUs in batches")
    ap.add_argument("--pattern-len", type=int, default=0)
    ap.add_argument("--options", type=int, default=FAITHFUL,
                    help="fmx_load options of the headline index (1 = FMX_OCC_INTERLEAVED, 0 = blob layout)")
    ap.add_argument("--no-blob-layout", action="store_true", help="skip the blob-layout (options 0) leg")
    ap.add_argument("--blob-source", choices=("broadcast", "build"), default="broadcast",
                    help="several ranks: rank 0 builds the blob and broadcasts it over RCCL (SURVEY 8(e)), or "
                         "every rank builds its own (deterministic)")
    ap.add_argument("--derived", action="store_true", help="also run the derived-index leg (~147 GB at C2)")
    ap.add_argument("--derived-options", type=int, default=DERIVED)
    ap.add_argument("--no-derived", action="store_true", help=argparse.SUPPRESS)  # (the default now)
    ap.add_argument("--min-seconds", type=float, default=2.0,
                    help="minimum timed region (passes repeated; >= 2 s so that an outside sampler sees the GPU busy)")
    ap.add_argument("--event-every", type=int, default=5,
                    help="bracket every k-th launch of the timed region with HIP events")
    ap.add_argument("--kernel-launches", type=int, default=8,
                    help="single-stream launches whose k_search is timed alone (roofline.kernel)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline budget per leg")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: all usable cores)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline / parity leg")
    ap.add_argument("--verify-job", action="store_true",
                    help="sharded jobs: rank 0 checks every count and location of the assembled job "
                         "against the CPU oracle")
    ap.add_argument("--no-fixed-len", action="store_true",
                    help="A/B: do not pass FMX_HINT_FIXED_LEN (the kernels read each tile's offsets first)")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-single-batch", action="store_true",
                    help="skip the single_batch leg (one 100k batch per fmx_locate_batch_async call)")
    ap.add_argument("--single-batch-only", action="store_true",
                    help="run only the headline setup and the single_batch leg (no other legs)")
    ap.add_argument("--streams", type=int, default=None, help="launches in flight (HIP streams; default 2)")
    ap.add_argument("--batches", type=int, default=32,
                    help="distinct batches cycled (weak-scaling configs; at least one launch group per stream)")
    ap.add_argument("--group", type=int, default=None, help="batches per launch (at most 2,048; fmx_locate_group_async; c2, c4: 1,024; c1, c3: 256; c5: 8)")
    ap.add_argument("--graph", action="store_true",
                    help="capture one pass (every launch, forked over the streams) in a HIP graph and replay it: "
                         "one host call per pass instead of one per launch (launch-bound configs)")
    ap.add_argument("--gather", choices=("all", "counts"), default="all",
                    help="N > 1 (and FMX_BENCH_DIST=1): what each launch group's in-step all-gather moves — all: "
                         "counts and locations (north_star's single all-gather, default); counts: the count slabs "
                         "alone (the job's offsets on every rank), the locations gathered once after the timed "
                         "region")
    ap.add_argument("--strong-groups", type=int, default=None,
                    help="c3/c5: launch groups per rank, each of --group / this many batches (default with gathers — "
                         "N > 1, or FMX_BENCH_DIST=1 — one per stream, so that one group's all-gather runs under "
                         "the other's search; without: 1, the rank's batches in one launch group)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--xcd-partitioned", action="store_true",
                    help="experiment (weak configs): each launch group's patterns arranged so that workgroup "
                         "tile t (XCD t %% 8) holds only patterns whose last 3 symbols fall in class t %% 8 "
                         "(upper bound of an XCD-aware partition; not a valid headline workload)")
    ap.add_argument("--presorted", action="store_true",
                    help="experiment (weak configs): each launch group's patterns pre-sorted by reversed "
                         "suffix (upper bound of the cache reuse a suffix sort would buy; not a valid headline)")
    ap.add_argument("--presort-symbols", type=int, default=14,
                    help="--presorted: the sort key is the last this many symbols (order within a key kept)")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def maybe_spawn(args):
    """`--gpus N` (N > 1) without torchrun: start the N ranks as a torchrun
    child process and exit with its status.  This process has not touched the
    GPU (torch.cuda.device_count() does not initialise it on this image) and
    does not exec: the ranks are children."""
    if "WORLD_SIZE" in os.environ or not args.gpus or args.gpus <= 1:
        return
    import torch
    backend = os.environ.get("FMX_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and args.gpus > ndev:
        log(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs (one per RCCL rank) but {ndev} "
            f"{'is' if ndev == 1 else 'are'} visible; refusing to oversubscribe (FMX_BENCH_BACKEND=gloo "
            f"rehearses several ranks on one GPU)")
        sys.exit(2)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"bench.py: starting {args.gpus} ranks: {' '.join(cmd[1:6])} ...")
    sys.exit(subprocess.call(cmd))


def usable_cores():
    """Cores this process may use: the affinity mask, capped by a cgroup CPU
    quota and by OMP_NUM_THREADS when set (a GPU box shows the whole
    machine's CPUs but grants a share of them)."""
    n, src = len(os.sched_getaffinity(0)), "sched_getaffinity"
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max" and math.ceil(int(q) / int(p)) < n:
            n, src = max(1, math.ceil(int(q) / int(p))), "cgroup cpu.max"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < n:
        n, src = int(omp), "OMP_NUM_THREADS"
    return n, src


def cut_patterns(torch, d_text, starts, m):
    """The patterns at `starts` (device int64), m bytes each, packed (device
    uint8[len(starts) * m]); built in chunks to bound the index temporaries."""
    out = torch.empty(starts.numel() * m, dtype=torch.uint8, device=d_text.device)
    ar = torch.arange(m, device=d_text.device)
    step = max(1, (1 << 25) // m)
    for a in range(0, starts.numel(), step):
        b = min(starts.numel(), a + step)
        out[a * m:b * m] = d_text[(starts[a:b, None] + ar[None, :]).reshape(-1)]
    return out


class Workload:
    """The batches of one rank: patterns cut from the device text at the given
    starts, per-batch outputs and workspaces; launch groups of up to GR
    batches, group q on stream q % S.  Batches may differ in size (a
    JobPlan's).  Outputs start as private buffers with room for B + B/8 +
    4096 locations; `rebind` points them at other buffers (a JobGather's
    slots) once the warm-up has sized every batch."""

    def __init__(self, torch, ix, d_text, m, starts_list, P, S, GR, fixed, dev):
        self.torch, self.ix, self.m, self.P, self.GR = torch, ix, m, P, GR
        self.pdt = torch.int32 if P == 4 else torch.int64
        self.streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
        self.stage_kb = min(56, -(-256 * m // 1024))  # FMX_HINT_STAGE_KB: a tile spans 256 * m bytes
        self.fixed = fixed
        self.batches = []
        # one allocation per kind, each batch a view (a few kernels instead of ~10 per batch: 2,048 batches
        # under rocprofv3's counter passes, which serialise every dispatch, took minutes): the patterns back
        # to back (+64 B: the key passes read whole words), offsets shared by batches of one size, the
        # workspaces 256-B aligned
        sizes = [int(st.numel()) for st in starts_list]
        caps = [b + b // 8 + 4096 for b in sizes]
        wss = [-(-ix.locate_workspace_size(max(b, 1)) // 256) * 256 for b in sizes]
        pat_all = torch.zeros(sum(sizes) * m + 64, dtype=torch.uint8, device=dev)
        if sizes:
            pat_all[:sum(sizes) * m] = cut_patterns(torch, d_text, torch.cat(starts_list), m)
        loff_all = torch.zeros(sum(sizes) + len(sizes), dtype=torch.int64, device=dev)
        need_all = torch.zeros(max(len(sizes), 1), dtype=torch.int64, device=dev)
        ws_all = torch.zeros(sum(wss) + 256, dtype=torch.uint8, device=dev)
        ws_base = (-ws_all.data_ptr()) % 256
        cnt_all = torch.zeros(sum(max(b, 1) for b in sizes), dtype=self.pdt, device=dev)
        locs_all = torch.zeros(sum(caps), dtype=self.pdt, device=dev)
        offs = {}
        po = lo = wo = co = ao = 0
        for k, starts in enumerate(starts_list):
            b, cap, wsz = sizes[k], caps[k], wss[k]
            g, j = divmod(k, GR)
            if b not in offs:
                offs[b] = (torch.arange(b + 1, device=dev, dtype=torch.int64) * m).contiguous()
            bt = dict(k=k, group=g, slot=j, n=b, starts=starts, pat=pat_all[po:po + b * m], off=offs[b],
                      loff=loff_all[lo:lo + b + 1], need=need_all[k:k + 1],
                      ws_t=ws_all[ws_base + wo:ws_base + wo + wsz], cnt=cnt_all[co:co + max(b, 1)],
                      locs=locs_all[ao:ao + cap], cap=cap)
            po, lo, wo, co, ao = po + b * m, lo + b + 1, wo + wsz, co + max(b, 1), ao + cap
            self.batches.append(bt)
        self.n_groups = -(-len(self.batches) // GR)
        self.bind()
        self.cursor = 0
        # the batches were made on torch's stream; the launches use self.streams
        torch.cuda.synchronize()

    def bind(self):
        """(Re)build each launch group's job queue from the batches' current buffers."""
        ix = self.ix
        self.groups = []
        for g in range(self.n_groups):
            sel = self.batches[g * self.GR:(g + 1) * self.GR]
            q = ix.job_queue([ix.locate_job(b["pat"].data_ptr(), b["off"].data_ptr(), b["n"], b["loff"].data_ptr(),
                                            b["locs"].data_ptr(), b["cap"], b["need"].data_ptr(),
                                            b["ws_t"].data_ptr(), b["ws_t"].numel(), d_counts=b["cnt"].data_ptr(),
                                            stage_kb=self.stage_kb, fixed_len=self.fixed) for b in sel])
            self.groups.append(dict(queue=q, stream=self.streams[g % len(self.streams)], batches=sel,
                                    patterns=sum(b["n"] for b in sel)))

    def rebind(self, outputs):
        """outputs[k] = (counts view, locations view) for batch k."""
        for bt, (c, l) in zip(self.batches, outputs):
            bt["cnt"], bt["locs"], bt["cap"] = c, l, int(l.numel())
        self.bind()
        self.torch.cuda.synchronize()

    def launch(self, g, stream=None):
        grp = self.groups[g]
        self.ix.locate_group_async(grp["queue"], stream=(stream or grp["stream"]).cuda_stream)
        return grp

    def launch_next(self):
        """The next launch group in a cycle that runs on across passes (so the
        streams keep alternating however many launches a pass has)."""
        g = self.cursor % self.n_groups
        self.cursor += 1
        return g, self.launch(g)

    def sync(self):
        for s in self.streams:
            self.ix.sync(s.cuda_stream)

    def needs(self):
        """Every batch's location total (synchronises)."""
        self.sync()
        return [int(x) for x in self.torch.cat([b["need"] for b in self.batches]).cpu().tolist()]

    def check_capacity(self):
        need = self.needs()
        bad = [(k, nd, b["cap"]) for k, (nd, b) in enumerate(zip(need, self.batches)) if nd > b["cap"]]
        if bad:
            raise SystemExit(f"location buffer too small: batch {bad[0][0]} needs {bad[0][1]} > {bad[0][2]}")
        return need

    def release(self):
        for s in self.streams:
            self.ix.release_stream(s.cuda_stream)


def timed_passes(torch, dist, dist_on, w, launches, warmup, min_seconds, event_every, on_launch=None,
                 pre_launch=None, drain=None):
    """Warm up (`warmup` launches, every launch group at least once), then time
    passes of `launches` launches (groups cycled) until the region lasts
    min_seconds.  Returns (elapsed_s, passes, batches_per_pass,
    patterns_per_pass, timing)."""
    ix = w.ix
    for q in range(max(warmup, w.n_groups)):
        w.launch(q % w.n_groups)
    torch.cuda.synchronize()
    w.check_capacity()
    w.cursor = 0
    count = [0, 0]

    def one_pass():
        for _ in range(launches):
            g = w.cursor % w.n_groups
            if pre_launch:
                pre_launch(g, w.groups[g])
            gi, grp = w.launch_next()
            count[0] += len(grp["batches"])
            count[1] += grp["patterns"]
            if on_launch:
                on_launch(gi, grp)
        if drain:
            drain()

    # calibrate the pass count (untimed), the same on every rank
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    one_pass()
    torch.cuda.synchronize()
    t1 = time.perf_counter() - t0
    # (the calibration pass runs colder than the timed ones: a 30 % margin keeps
    # the timed region at or above min_seconds)
    passes = max(1, math.ceil(1.3 * min_seconds / max(t1, 1e-6)))
    if dist_on:
        pt = torch.tensor([passes], dtype=torch.int64, device="cuda")
        dist.all_reduce(pt, op=dist.ReduceOp.MAX)
        passes = int(pt.item())
    ix.timing_read()
    ix.timing_enable(True, every=event_every)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    count[0] = count[1] = 0
    t0 = time.perf_counter()
    for _ in range(passes):
        one_pass()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist_on:
        dist.barrier()
    ix.timing_enable(False)
    return elapsed, passes, count[0] // passes, count[1] // passes, ix.timing_read()


def capture_pass(torch, w, launches):
    """One pass — `launches` launches, group q on its own stream q % S — captured
    in a HIP graph: the other streams fork from the first and join it at the
    end, so the replay keeps the launches' concurrency.  The engine's launch
    path is capture-safe (no synchronous call; timing must be off)."""
    g = torch.cuda.CUDAGraph()
    s0 = w.streams[0]
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s0):
        fork = torch.cuda.Event()
        fork.record(s0)
        for st in w.streams[1:]:
            st.wait_event(fork)
        w.cursor = 0
        for _ in range(launches):
            w.launch_next()
        for st in w.streams[1:]:
            join = torch.cuda.Event()
            join.record(st)
            s0.wait_event(join)
    w.cursor = 0
    return g


def timed_graph(torch, dist, dist_on, w, launches, warmup, min_seconds):
    """timed_passes with every pass a replay of one captured graph."""
    for q in range(max(warmup, w.n_groups)):
        w.launch(q % w.n_groups)
    torch.cuda.synchronize()
    w.check_capacity()
    w.ix.timing_enable(False)
    g = capture_pass(torch, w, launches)
    per = sum(w.groups[q % w.n_groups]["patterns"] for q in range(launches))
    nbat = sum(len(w.groups[q % w.n_groups]["batches"]) for q in range(launches))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    passes = max(1, math.ceil(1.3 * min_seconds / max(time.perf_counter() - t0, 1e-6)))
    if dist_on:
        pt = torch.tensor([passes], dtype=torch.int64, device="cuda")
        dist.all_reduce(pt, op=dist.ReduceOp.MAX)
        passes = int(pt.item())
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(passes):
        g.replay()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist_on:
        dist.barrier()
    return elapsed, passes, nbat, per, {}


def kernel_pass(torch, w, launches):
    """k_search alone: `launches` launches one after another on one stream
    with nothing else in flight, each bracketed by HIP events around its two
    kernels (timers locate.search / locate.emit).  Per-launch averages."""
    ix = w.ix
    torch.cuda.synchronize()
    ix.timing_read()
    ix.timing_enable(True, every=1)
    for q in range(launches):
        w.launch(q % w.n_groups, stream=w.streams[0])
    torch.cuda.synchronize()
    t = ix.timing_read()
    ix.timing_enable(False)
    return t


def self_location(w, P):
    """Size-independent property at full size, every batch: pattern i was cut
    at starts[i], so starts[i] is among its locations (and counts >= 1)."""
    ok = True
    pdt_np = np.uint32 if P == 4 else np.uint64
    for bt in w.batches:
        if bt["n"] == 0:
            continue
        bo = bt["loff"].cpu().numpy().view(np.uint64)
        bl = bt["locs"][:int(bo[-1])].cpu().numpy().view(pdt_np)
        st = bt["starts"].cpu().numpy()
        cnt = np.diff(bo).astype(np.int64)
        owner = np.repeat(np.arange(bt["n"]), cnt)
        hit = np.zeros(bt["n"], dtype=bool)
        hit[owner[bl.astype(np.int64) == st[owner]]] = True
        ok = ok and bool(hit.all() and (cnt >= 1).all())
    return ok


def traffic_of(path, key):
    if not os.path.exists(path):
        return None
    try:
        return json.load(open(path)).get("runs", {}).get(key)
    except (OSError, ValueError):
        return None


def per_launch_ms(timing):
    return {k: v["total_ms"] / max(v["launches"], 1) for k, v in timing.items()}


def oracle_index(O, d_blob, blob_len, P, cfg):
    host_blob = O.aligned_zeros(blob_len, 16)
    host_blob[:] = d_blob.cpu().numpy()
    return O.OracleIndex(host_blob, O.layout(P, cfg["planes"], cfg["vec"], 0))


def main():
    args = parse()
    maybe_spawn(args)
    import torch
    import torch.distributed as dist

    import __graft_entry__ as g
    pkg = g.load_package()
    D = pkg.distributed
    cfg = dict(CONFIGS[args.config])

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch {args.gpus} ranks "
            f"(torchrun --nproc-per-node {args.gpus}) or drop --gpus")
        sys.exit(2)
    # FMX_BENCH_BACKEND=gloo: a rehearsal of the multi-rank path with several
    # ranks on one GPU (RCCL needs one device per rank)
    backend = os.environ.get("FMX_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > 1 and local >= ndev:
        log(f"bench.py: rank {rank} has LOCAL_RANK {local} but {ndev} GPU(s) are visible; RCCL needs one GPU "
            f"per rank, refusing to share a device")
        sys.exit(2)
    gpu = local % max(ndev, 1)
    # FMX_BENCH_DIST=1: start the process group even for one rank, so that a
    # one-GPU box drives the RCCL calls (collectives, barriers, in-step gathers)
    dist_on = world > 1 or os.environ.get("FMX_BENCH_DIST") == "1"
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{gpu}"))
        else:
            dist.init_process_group(backend)
    dev = torch.device(f"cuda:{gpu}")
    torch.cuda.set_device(dev)
    # the distinct devices the ranks run on (one node: device index + uuid)
    props = torch.cuda.get_device_properties(gpu)
    me = (socket.gethostname(), gpu, str(getattr(props, "uuid", "")))
    if dist_on:
        everyone = [None] * world
        dist.all_gather_object(everyone, me)
    else:
        everyone = [me]
    n_devices = len(set(everyone))

    n = args.text_len or cfg["text_len"]
    m = args.pattern_len or cfg["m"]
    B = args.patterns or cfg["patterns"]
    total = args.total_patterns if args.total_patterns >= 0 else cfg["total"]
    P = cfg["pos"]
    S = max(1, args.streams or cfg.get("streams", 2))
    GR = max(1, min(args.group or cfg.get("group", 8), 2048))
    BLK = cfg["planes"] * cfg["vec"] // 8
    position = pkg.u32 if P == 4 else pkg.u64
    block = getattr(pkg.blocks, f"Block{cfg['planes']}")(pkg.Vector(cfg["vec"]))
    pdt_t = torch.int32 if P == 4 else torch.int64
    pdt_np = np.uint32 if P == 4 else np.uint64

    # ---- synthetic text (same on every rank: the blob is replicated) -------
    t0 = time.time()
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed)
    alpha = torch.tensor(list(cfg["alphabet"]), dtype=torch.uint8, device=dev)
    d_text = torch.empty(n, dtype=torch.uint8, device=dev)
    chunk = 1 << 28
    for c0 in range(0, n, chunk):  # bounded int64 temporaries
        c1 = min(n, c0 + chunk)
        d_text[c0:c1] = alpha[torch.randint(0, len(cfg["alphabet"]), (c1 - c0,), device=dev, dtype=torch.int64,
                                            generator=gen)]
    table = pkg.text_encoders.EncodingTable.from_symbols(cfg["symbols"])
    builder = (pkg.FmIndexBuilder(n, table.symbol_count(), table, position, block)
               .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(cfg["k"]))
               .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(cfg["sr"])))
    blob_len = builder.blob_size()
    d_blob = torch.empty(blob_len, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t1 = time.time()
    # (one rank with FMX_BENCH_DIST=1: the broadcast runs too — a self-broadcast that drives the RCCL path)
    bcast = dist_on and args.blob_source == "broadcast"
    if rank == 0 or not bcast:
        builder.build_device(d_text.data_ptr(), d_blob.data_ptr(), blob_len, device=gpu)
    torch.cuda.synchronize()
    build_s = time.time() - t1
    log(f"[rank {rank}] text {n:,} B generated in {t1 - t0:.2f}s, blob {blob_len:,} B built on GPU in {build_s:.2f}s")
    replicate = None
    if bcast:
        # one replica per GPU: rank 0's blob broadcast over RCCL (xGMI), then
        # every rank's copy checksummed and compared across ranks
        replicate = D.replicate_blob(d_blob, src=0)
        replicate["gbs"] = blob_len / replicate["seconds"] / 1e9
        if not replicate["identical"]:
            raise SystemExit(f"rank {rank}: the broadcast blob differs across ranks")

    # PCIe: what loading this blob from host memory costs (pinned -> HBM)
    upload_s = None
    if rank == 0 and blob_len <= (16 << 30):
        h_blob = torch.empty(blob_len, dtype=torch.uint8, pin_memory=True)
        h_blob.copy_(d_blob)
        d_tmp = torch.empty_like(d_blob)
        torch.cuda.synchronize()
        tu = time.perf_counter()
        d_tmp.copy_(h_blob, non_blocking=True)
        torch.cuda.synchronize()
        upload_s = time.perf_counter() - tu
        del d_tmp, h_blob

    def load(options):
        tl = time.time()
        ixl = pkg.FmIndex.load_device(d_blob.data_ptr(), blob_len, position, block,
                                      pkg.text_encoders.EncodingTable, device=gpu, options=options)
        torch.cuda.synchronize()
        return ixl, time.time() - tl

    ix, load_s = load(args.options)
    info = ix.info()
    log(f"[rank {rank}] index loaded in {load_s:.3f}s: options={info['options']} device_bytes={info['device_bytes']:,}")

    fixed = 0 if args.no_fixed_len else m
    strong = total > 0

    def weak_starts(nbatches):
        # (one draw for all of this rank's batches; each batch a view)
        pg = torch.Generator(device=dev)
        pg.manual_seed(args.seed * 1000 + 7 + 7919 * rank)
        allst = torch.randint(0, n - m + 1, (nbatches, B), device=dev, dtype=torch.int64, generator=pg)
        return [allst[bi] for bi in range(nbatches)]

    NB = -(-max(S * GR, args.batches) // (S * GR)) * (S * GR)  # weak: whole groups on every stream
    plan = job_starts = None
    if strong:
        # the global job (the same on every rank), dealt out by JobPlan
        # with gathers (N > 1): one launch group per stream (each of GR / S batches), so that a group's
        # gather runs under the other group's search; without, one group (same box, profiles/r6/r6q_*: C3
        # 10 M 3.39 vs 3.28 x 10^9 and C5 1 M 3.50 vs 3.34 x 10^8 for one group, but C3's N = 8 slab
        # 2.93 vs 2.61 x 10^9 for two)
        SG = max(1, args.strong_groups if args.strong_groups is not None else (S if dist_on else 1))
        if SG > 1:
            GR = max(1, GR // SG)
        plan = D.JobPlan(total, world, B, GR, min_groups=SG)
        jg_gen = torch.Generator(device=dev)
        jg_gen.manual_seed(args.seed * 1000 + 7)
        job_starts = torch.randint(0, n - m + 1, (total,), device=dev, dtype=torch.int64, generator=jg_gen)
        my = plan.batches(rank)
        w = Workload(torch, ix, d_text, m, [job_starts[a:b] for a, b in my], P, S, GR, fixed, dev)
        launches = w.n_groups
        steps = len(my)
    else:
        w = Workload(torch, ix, d_text, m, weak_starts(NB), P, S, GR, fixed, dev)
        if args.presorted or args.xcd_partitioned:
            arrange(torch, w, B, m, GR, dev, args.presorted, args.presort_symbols, cfg["alphabet"])
        steps = args.steps or 800
        launches = -(-steps // GR)
    torch.cuda.synchronize()

    jg = None
    if strong or dist_on:
        # size every batch's location slot from the warm-up (the same batches
        # run in the timed region), exchange the sizes once, and point the
        # kernels' outputs straight into the gather slabs: a sharded job's
        # (c3/c5), or every rank's own batches (c2 weak scaling), so that the
        # results are concatenated on every rank inside the timed step
        for q in range(max(args.warmup, w.n_groups)):
            w.launch(q % w.n_groups)
        torch.cuda.synchronize()
        needs = w.check_capacity()
        all_needs = D.all_gather_ints(needs, device=dev)
        sizes = plan.sizes() if strong else np.full((world, len(w.batches)), B, dtype=np.int64)
        jg = D.JobGather(sizes, all_needs, GR, rank, pdt_t, dev, collective=dist_on)
        w.rebind([(jg.counts_slot(k), jg.locs_slot(k)) for k in range(len(w.batches))])

    # ---- timed region: compute ----------------------------------------------
    if args.graph:
        elapsed, passes, per_pass, pats_pass, timing = timed_graph(torch, dist, dist_on, w, launches, args.warmup,
                                                                   args.min_seconds)
    else:
        elapsed, passes, per_pass, pats_pass, timing = timed_passes(torch, dist, dist_on, w, launches, args.warmup,
                                                                    args.min_seconds, args.event_every)
    if dist_on:
        elapsed = D.max_over_ranks(elapsed, device=dev)
    # every pattern a launch ran counts (a pass of K steps runs ceil(K / GR) whole launches)
    pt = torch.tensor([pats_pass * passes], dtype=torch.int64, device=dev)
    if dist_on:
        dist.all_reduce(pt)
    value_compute = int(pt.item()) / elapsed

    # ---- gathers -------------------------------------------------------------
    gather = None
    value = value_compute
    if strong:
        needs_after = w.needs()
        gather = {"plan": {"batches_per_rank": plan.nb, "launch_groups": plan.groups,
                           "patterns_per_rank": [e - s for s, e in plan.spans],
                           "batch_patterns_min": int(plan.sizes().min()), "batch_patterns_max": plan.max_batch()},
                  "needs_stable": needs_after == needs}
    if dist_on:
        # the same passes with each launch group's results all-gathered (one
        # collective) on a communication stream while the next launch computes
        # (strong: the job's slab of that group; weak: every rank's batches of
        # that group) — the north star's "single RCCL all-gather over xGMI to
        # concatenate results", inside the timed step
        comm = torch.cuda.Stream(device=dev)
        works, gathered = [], {}

        def pre_launch(gi, grp):
            ev = gathered.get(gi)  # the slab may be rewritten only once its last gather has read it
            if ev is not None:
                grp["stream"].wait_event(ev)

        def on_launch(gi, grp):
            ev = torch.cuda.Event()
            ev.record(grp["stream"])
            comm.wait_event(ev)
            with torch.cuda.stream(comm):
                works.append(jg.gather(gi, async_op=True, part=args.gather))
                done = torch.cuda.Event()
                done.record(comm)
                gathered[gi] = done

        def drain():
            for wk in works:
                if wk is not None:
                    wk.wait()
            works.clear()
            torch.cuda.current_stream().wait_stream(comm)

        e2, p2, _, pats2, _ = timed_passes(torch, dist, dist_on, w, launches, 0, args.min_seconds,
                                           args.event_every, on_launch=on_launch, pre_launch=pre_launch,
                                           drain=drain)
        e2 = D.max_over_ranks(e2, device=dev)
        pt2 = torch.tensor([pats2 * p2], dtype=torch.int64, device=dev)
        dist.all_reduce(pt2)
        value = int(pt2.item()) / e2
        if gather is None:
            gather = {}
        # what each policy moves per pass and the xGMI rate per GPU it needs to
        # hide behind the compute (bytes every rank receives / the compute-only
        # time of a pass), at this N and, for the same per-rank shape, at N = 8
        pass_s = elapsed / max(passes, 1)
        per_rank_slab = {pol: jg.bytes_per_pass(pol) / max(world, 1) for pol in ("all", "counts")}
        gather.update({"inside_timed_step": True, "value_compute_only": value_compute,
                       "policy": args.gather, "collectives_per_launch": 1,
                       "bytes_gathered_per_pass": jg.bytes_per_pass(args.gather),
                       "bytes_per_pass": {pol: jg.bytes_per_pass(pol) for pol in ("all", "counts")},
                       "required_gbs_per_gpu": {pol: jg.bytes_per_pass(pol) / pass_s / 1e9
                                                for pol in ("all", "counts")},
                       "required_gbs_per_gpu_at_n8": {pol: 8 * per_rank_slab[pol] / pass_s / 1e9
                                                      for pol in ("all", "counts")} if not strong else None,
                       "result_bytes_per_pass": jg.result_bytes(),
                       "gathered_over_result": jg.bytes_per_pass() / max(jg.result_bytes(), 1)})
        if args.gather == "counts":
            jg.gather_all()  # the locations once, after the timed region (assemble below)
            torch.cuda.synchronize()
    if jg is not None:
        # the job's flat (offsets, locations) on the device; this rank's part
        # must equal what its own launches wrote
        offs_job, locs_job = jg.assemble()
        s0, e0 = plan.spans[rank] if strong else (rank * len(w.batches) * B, (rank + 1) * len(w.batches) * B)
        mine = torch.cat([bt["cnt"] for bt in w.batches]).to(torch.int64)
        if gather is None:
            gather = {}
        gather["assembled_patterns"] = int(offs_job.numel() - 1)
        gather["assembled_locations"] = int(locs_job.numel())
        gather["assembly_ok"] = bool(offs_job.numel() == int(jg.sizes.sum()) + 1 and
                                     int(offs_job[-1].item()) == locs_job.numel() == int(jg.needs.sum()) and
                                     torch.equal(torch.diff(offs_job[s0:e0 + 1]), mine))

    # what `value` was timed over (N > 1: the passes with the in-step gathers)
    region_s, passes_timed = (e2, p2) if dist_on else (elapsed, passes)
    steps_timed = per_pass * passes_timed

    # ---- roofline --------------------------------------------------------------
    # Algorithmic bytes: per pattern m + 2P (k-mer seed) +
    # L*2*(P+|B|) (two rank queries per LF step) + P (count), per occurrence
    # w*(P+|B|) (walk, E[w] = sr-1) + P (sampled SA) + P (location out).
    k, sr = info["kmer_size"], info["sampling_ratio"]
    my_pats = sum(bt["n"] for bt in w.batches)
    my_occ = sum(w.needs())
    # every pattern is cut from the text, so its interval never empties and the
    # reference's LF loop runs exactly m - k steps (with_slice.rs:27-31)
    L = m - k
    per_pattern = m + 2 * P + L * 2 * (P + BLK) + P
    per_occ = (sr - 1) * (P + BLK) + 2 * P
    alg_per_pattern = per_pattern + per_occ * my_occ / max(my_pats, 1)
    per_gpu = value_compute / max(world, 1)
    achieved = alg_per_pattern * per_gpu / 1e9
    fused0 = ix.info().get("launches_fused", 0)
    kt = kernel_pass(torch, w, max(1, args.kernel_launches))
    # launches in launch order of small batches run as one kernel (k_locate): its "search phase" is the whole launch
    fused = ix.info().get("launches_fused", 0) > fused0
    ks, ke, kl = (kt.get(x, {}) for x in ("locate.search", "locate.emit", "locate"))
    ppl = ks.get("units", 0) / max(ks.get("launches", 1), 1)
    search_us = ks["total_ms"] / ks["launches"] * 1e3 if ks.get("launches") else float("nan")
    k_achieved = alg_per_pattern * ppl / (search_us * 1e-6) / 1e9
    key = f"{args.config}:{n}:{B}:{m}:{info['options']}:g{GR}"
    # (the engine's policy: packable fixed-length launches from grouped_min patterns; longer patterns only
    # when FMX_GROUPED=1 / FMX_GROUPED_RAW=1 ask for it)
    packs = m * table.symbol_count().bit_length() <= 96 and os.environ.get("FMX_GROUPED_RAW") != "1"
    grouped = bool(info.get("group_key_len")) and max(grp["patterns"] for grp in w.groups) >= info["grouped_min"] \
        and bool(fixed) and os.environ.get("FMX_GROUPED") != "0" and \
        (packs or os.environ.get("FMX_GROUPED") == "1" or os.environ.get("FMX_GROUPED_RAW") == "1")
    tr = traffic_of(args.traffic_json, key)
    roof = {
        "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
        # memory-side bytes per launch (reads from the request split + writes), rocprofv3 PMC passes of this
        # build under this profile key (scripts/gpu.sh pmc + scripts/traffic.py)
        "traffic": tr.get("traffic_bytes_per_launch", tr.get("fabric_bytes_per_launch")) if tr else None,
        "achieved_basis": "per-step cost: the reference algorithm's bytes per pattern (SURVEY.md 8(d), "
                          "alg_bytes_per_pattern) x the timed region's patterns/s per GPU",
        "alg_bytes_per_pattern": alg_per_pattern,
        "kernel": {
            "name": ("search phase of a grouped launch: k_group_key + k_group_scan + k_group_place + "
                     "k_search_grouped + k_group_tiles" if grouped else
                     "k_locate (fused: search, tile-count hand-off, offsets and locations in one kernel)" if fused
                     else "k_search"),
            "avg_us": search_us, "patterns_per_launch": ppl,
            "achieved": k_achieved, "frac": k_achieved / HBM_PEAK_GBS,
            "emit_avg_us": ke["total_ms"] / ke["launches"] * 1e3 if ke.get("launches") else None,
            "launch_avg_us": kl["total_ms"] / kl["launches"] * 1e3 if kl.get("launches") else None,
            "launches": ks.get("launches", 0),
            "basis": "alg bytes x patterns per launch / the search phase's average duration: launches one after "
                     "another on one stream, nothing else in flight, HIP events around the search phase (k_search, "
                     "or a grouped launch's five kernels before k_emit) alone (compare the sum of those kernels in "
                     "rocprofv3 --kernel-trace --stats of bench.py --streams 1)",
        },
    }
    if tr:
        req = tr.get("fabric_requests_per_launch")
        tppl = tr.get("patterns_per_launch", ppl or 1)
        tpp = roof["traffic"] / tppl
        roof.update({
            "traffic_what": "memory-side bytes per launch of the headline's launch shape (a launch = "
                            "patterns_per_launch patterns; every kernel of the launch): reads = TCC_EA0_RDREQ "
                            "requests x their size (32/64/128 B), writes = WRITE_SIZE; on gfx950 these include "
                            "Infinity Cache hits (MI355X_MICROARCH.md, HBM section), so they bound HBM bytes from "
                            "above",
            "traffic_source": f"{os.path.relpath(args.traffic_json, ROOT)} [{key}] ({tr.get('source')})",
            "traffic_patterns_per_launch": tppl,
            "traffic_bytes_per_pattern": tpp,
            "traffic_over_alg": tpp / alg_per_pattern,
            "fabric_read_bytes_per_pattern": tr["fabric_bytes_per_launch"] / tppl,
            "traffic_frac_effective": tpp * per_gpu / 1e9 / HBM_PEAK_GBS,
        })
        if tr.get("search_kernel"):
            roof["kernel"]["traffic_bytes_per_pattern"] = tr["search_kernel"].get("traffic_bytes_per_pattern")
            roof["kernel"]["fabric_requests_per_pattern"] = tr["search_kernel"].get("fabric_requests_per_pattern")
        if req:
            rpp = req / tr.get("patterns_per_launch", ppl or 1)
            roof.update({"fabric_requests_per_pattern": rpp, "fabric_grequests_per_s": rpp * per_gpu / 1e9,
                         "random_line_ceiling_grequests_per_s": RANDOM_LINE_CEILING})

    b0 = w.batches[0]
    offs_h = b0["loff"].cpu().numpy().view(np.uint64)
    total_occ = int(offs_h[-1])
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "patterns/s",
        "n_gpus": n_devices,
        "ranks": world,
        "rccl_world_size": world if (dist_on and backend == "nccl") else None,
        "backend": backend if dist_on else None,
        "steps": steps_timed,
        "steps_requested": args.steps or None,
        "warmup": args.warmup,
        "ms_per_step": region_s / steps_timed * 1e3,
        "timed_passes": passes_timed,
        "batches_per_pass": per_pass,
        "timed_region_s": region_s,
        "steps_what": "batches (steps) timed: whole launches of up to batches_per_launch batches, passes repeated "
                      "until the region lasts >= --min-seconds; the requested --steps is rounded up to whole "
                      "launches per pass" + ("; N > 1: the passes with the in-step all-gathers" if dist_on else ""),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u32" if P == 4 else "u64",
        "data": f"synthetic: seeded uniform {cfg['alphabet'].decode()} text; patterns cut from it at uniform "
                f"random starts",
        "config": {
            "workload": cfg["desc"] if (n == cfg["text_len"] and m == cfg["m"] and B == cfg["patterns"]) else
            f"{args.config} variant: {n:,}-symbol text, {B:,} x {m} patterns per batch",
            "config": args.config, "text_len": n, "patterns_per_batch": B, "pattern_len": m,
            "global_batch": total if strong else B * world,
            "layout": f"u{P * 8}/Block{cfg['planes']}<u{cfg['vec']}>/EncodingTable(sigma={table.symbol_count()})",
            "load_options": info["options"],
            "index": {0: "the blob as laid out", 1: "the blob + its planes and checkpoints as one record per block"}
            .get(info["options"], "derived structures"),
            "index_hbm_bytes": blob_len + info["device_bytes"],
            "parallelism": f"dp{world} (patterns sharded, blob replicated)",
            "streams": S, "fixed_len_hint": fixed, "batches_per_launch": GR, "distinct_batches": len(w.batches),
            "hip_graph": bool(args.graph),
            "launch_order": f"grouped by the last {info['group_key_len']} symbols" if grouped else "as given",
        },
        "roofline": roof,
        "kernels_ms_per_launch_timed_region": per_launch_ms(timing),
        "occurrences_batch0": total_occ,
        "self_location_check": self_location(w, P),
        "build_s": build_s,
        "load_s": load_s,
        "upload_s": upload_s,
        "upload_gbs": None if upload_s is None else blob_len / upload_s / 1e9,
        # the README's workload (100 k patterns, bench/run_benchmark.sh) end to
        # end from a host-resident blob: upload + load + locate
        "readme_workload_s": None if upload_s is None else upload_s + load_s + 100_000 / per_gpu,
        "gather": gather,
        # what this rank holds in HBM (distributed.hbm_per_rank: the same accounting tests/test_distributed.py
        # checks for 8 ranks against 288 GB), beside torch's measured peak (+ the index's own allocations)
        "hbm_per_rank": dict(D.hbm_per_rank(blob=blob_len, records=info["device_bytes"], text=n,
                                            batch_sizes=[bt["n"] for bt in w.batches], m=m, pos_bytes=P,
                                            world=world, group=GR, loc_cap=[bt["cap"] for bt in w.batches],
                                            gather=jg is not None and jg.collective),
                             measured_torch_peak=int(torch.cuda.max_memory_allocated(dev)),
                             measured_index=int(info["device_bytes"])),
        "blob_replication": replicate if replicate else
        {"how": "each rank builds the blob from the same seeded text" if world > 1 else "one rank"},
        "profile_key": key,
    }

    # ---- whole-job parity (sharded jobs, rank 0) -------------------------------
    if strong and args.verify_job and rank == 0:
        from oracle import oracle as O
        orc = oracle_index(O, d_blob, blob_len, P, cfg)
        pats_h = cut_patterns(torch, d_text, job_starts, m).cpu().numpy()
        offs_in = np.arange(total + 1, dtype=np.uint64) * m
        cores, _ = usable_cores()
        tv = time.perf_counter()
        ooff, olocs = orc.locate_batch(pats_h, offs_in, threads=cores, cap=int(jg.needs.sum()) + 4096)
        job_off = offs_job.cpu().numpy().view(np.uint64)
        job_loc = locs_job.cpu().numpy().view(pdt_np)
        result["parity"] = {"bit_exact_vs_cpu": bool(np.array_equal(ooff, job_off) and np.array_equal(olocs, job_loc)),
                            "patterns": total, "occurrences": int(olocs.size), "scope": "every pattern of the job",
                            "oracle_s": time.perf_counter() - tv, "oracle_threads": cores}
        if not result["parity"]["bit_exact_vs_cpu"]:
            log("PARITY FAILURE: the assembled job differs from the CPU oracle")
        del orc

    # ---- one batch per call (the config's own batch, N = 1) ------------------
    if rank == 0 and world == 1 and not strong and not args.no_single_batch:
        result["single_batch"] = single_batch_leg(torch, ix, load, d_text, n, m, B, fixed, dev, args.seed,
                                                  min(args.min_seconds, 1.0), pdt_t, P, GR, S)
    if args.single_batch_only:
        args.no_blob_layout = args.no_cpu = True
        args.derived = False

    # ---- the blob's own layout (options 0, N = 1) -----------------------------
    # the GPU's answers for the CPU leg to check (32 batches spread evenly over
    # the workload's distinct batches — at C2's 2,048: every 66th, so every
    # kernel-argument group of 256 of both grouped launches is sampled; host copies)
    host_batches, host_idx, n_distinct = [], [], len(w.batches)
    if rank == 0 and world == 1 and not args.no_cpu:
        host_idx = sorted({int(round(x)) for x in np.linspace(0, n_distinct - 1, min(32, n_distinct))})
        for bi in host_idx:
            bt = w.batches[bi]
            bo = bt["loff"].cpu().numpy().view(np.uint64).copy()
            host_batches.append((bt["pat"].cpu().numpy(), bt["n"], bo,
                                 bt["locs"][:int(bo[-1])].cpu().numpy().view(pdt_np).copy()))
    if world == 1 and not args.no_blob_layout and args.options != BLOB_LAYOUT:
        w.release()
        w = None
        ixb, load_b = load(BLOB_LAYOUT)
        infob = ixb.info()
        wb = Workload(torch, ixb, d_text, m, weak_starts(NB), P, S, GR, fixed, dev)
        bsteps = args.steps or 800
        eb, pb, _, patsb, tb = timed_passes(torch, dist, dist_on, wb, -(-bsteps // GR), args.warmup,
                                            args.min_seconds, args.event_every)
        ktb = kernel_pass(torch, wb, max(1, args.kernel_launches)).get("locate.search", {})
        result["blob_layout"] = {
            "value": patsb * pb / eb, "unit": "patterns/s", "options": infob["options"],
            "index_hbm_bytes": blob_len + infob["device_bytes"], "load_s": load_b,
            "k_search_avg_us": ktb["total_ms"] / ktb["launches"] * 1e3 if ktb.get("launches") else None,
            "self_location_check": self_location(wb, P),
            "what": "the same weak-scaling workload over the blob's rank_checkpoints and blocks arrays exactly as "
                    "laid out (the reference's zero-copy view, bwm/mod.rs:157-189; 2 lines per rank): no HBM "
                    "beyond the blob",
        }
        wb.release()
        wb = None
        ixb.close()

    # ---- derived-index mode (labelled variant, opt-in, N = 1) ----------------
    if world == 1 and args.derived:
        if w is not None:
            w.release()
            w = None
        ixd, load_d = load(args.derived_options)
        infod = ixd.info()
        wd = Workload(torch, ixd, d_text, m, weak_starts(NB), P, S, GR, fixed, dev)
        dsteps = args.steps or 800
        ed, pd, _, patsd, td_t = timed_passes(torch, dist, dist_on, wd, -(-dsteps // GR), args.warmup,
                                              args.min_seconds, args.event_every)
        vd = patsd * pd / ed
        dt = 1.0 / value_compute - 1.0 / vd  # seconds saved per pattern
        result["derived"] = {
            "value": vd, "unit": "patterns/s", "options": infod["options"], "deep_lut_k": infod["deep_lut_k"],
            "index_hbm_bytes": blob_len + infod["device_bytes"], "load_s": load_d,
            "breakeven_patterns": (load_d - load_s) / dt if dt > 0 else None,
            "kernels_ms_per_launch": per_launch_ms(td_t),
            "self_location_check": self_location(wd, P),
            "what": "outside SURVEY 8: the same queries over structures derived from the blob at load (a K-mer "
                    "interval table, single-row entries, row records, the full SA)",
        }
        wd.release()
        wd = None
        ixd.close()

    # ---- CPU baseline + bit-exact check (rank 0, N=1 only) -------------------
    # The oracle answers the GPU's batches in turn (whole batches, cycled) for
    # >= cpu_seconds per leg; every batch it answers is compared with the GPU.
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import oracle as O
        orc = oracle_index(O, d_blob, blob_len, P, cfg)
        cores, src = usable_cores()
        threads = args.cpu_threads or cores
        legs = {}
        checked, exact = set(), True
        for th in sorted({1, threads}):
            done, q, tc = 0, 0, time.perf_counter()
            while True:
                pats_h, nb_, offs_g, locs_g = host_batches[q % len(host_batches)]
                offs_in = np.arange(nb_ + 1, dtype=np.uint64) * m
                ooff, olocs = orc.locate_batch(pats_h, offs_in, threads=th, cap=4 * nb_ + 4096)
                if q % len(host_batches) not in checked:
                    exact = exact and bool(np.array_equal(ooff, offs_g) and np.array_equal(olocs, locs_g))
                    checked.add(q % len(host_batches))
                done += nb_
                q += 1
                if time.perf_counter() - tc >= args.cpu_seconds:
                    break
            legs[th] = (done / (time.perf_counter() - tc), done)
        try:
            model = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
        except (OSError, IndexError):
            model = "unknown"
        nck = sum(host_batches[i][1] for i in checked)
        result["cpu_baseline"] = {
            "value": legs[threads][0], "unit": "patterns/s", "cores": threads, "kind": "port",
            "sample": f"{legs[threads][1]:,} patterns = whole batches of the GPU's workload ({len(host_batches)} "
                      f"batches of {host_batches[0][1]:,} cycled) for >= {args.cpu_seconds:.0f} s on {threads} "
                      f"threads, oracle/fmx_oracle.c (C restatement of the reference query path), blob in RAM",
            "value_1_thread": legs[1][0], "cores_source": src, "cpu_model": model,
            "host_cpus_visible": os.cpu_count(),
        }
        idx_checked = [host_idx[i] for i in sorted(checked)]
        groups = sorted({bi // 256 for bi in idx_checked})
        result.setdefault("parity", {"bit_exact_vs_cpu": exact, "patterns": nck, "batches": len(checked),
                                     "scope": f"{len(checked)} of the workload's {n_distinct} batches, spread "
                                              f"over its kernel-argument groups of 256 {groups}, every count and "
                                              f"location", "batch_indices": idx_checked})
        result["parity_cpu_leg"] = {"bit_exact": exact, "batches": len(checked), "patterns": nck,
                                    "batch_indices": idx_checked}
        result["speedup_vs_cpu"] = value / legs[threads][0]
        result["speedup_vs_cpu_1_thread"] = value / legs[1][0]
        if not exact:
            log("PARITY FAILURE: GPU results differ from the CPU oracle")

    if rank == 0:
        print(json.dumps(result), flush=True)
    if w is not None:
        w.release()
    ix.close()
    if dist_on:
        dist.destroy_process_group()


def single_batch_leg(torch, ix, load, d_text, n, m, B, fixed, dev, seed, min_seconds, pdt_t, P, GR, S):
    """BASELINE configs[1] as a caller of the reference's per-batch loop gets
    it (bench/src/locate/sview_memory.rs:32: one batch of 100,000 patterns per
    call): one fmx_locate_batch_async call per batch on one stream, calls back
    to back (each waits only for the stream), 32 distinct batches cycled for
    >= min_seconds — in launch order (FMX_GROUPED=0) and grouped
    (FMX_GROUPED=1: the batch dealt out by its last symbols on its own), each
    on an index of its own (the policy is read at load)."""
    out = {"what": f"one {B:,}-pattern batch per fmx_locate_batch_async call, one stream, calls back to back; "
                   f"the headline instead runs {GR:,} batches per launch (fmx_locate_group_async) on {S} streams"}
    stage_kb = min(56, -(-256 * m // 1024))
    for mode, name in (("0", "launch_order"), ("1", "grouped")):
        saved = os.environ.get("FMX_GROUPED")
        os.environ["FMX_GROUPED"] = mode
        try:
            ixs, _ = load(FAITHFUL)
        finally:
            if saved is None:
                del os.environ["FMX_GROUPED"]
            else:
                os.environ["FMX_GROUPED"] = saved
        stream = torch.cuda.Stream(device=dev)
        bats = []
        for bi in range(32):
            pg = torch.Generator(device=dev)
            pg.manual_seed(seed * 1000 + 50021 * bi + 13)
            st = torch.randint(0, n - m + 1, (B,), device=dev, dtype=torch.int64, generator=pg)
            cap = B + B // 8 + 4096
            bats.append(dict(starts=st, pat=cut_patterns(torch, d_text, st, m),
                             off=torch.arange(B + 1, device=dev, dtype=torch.int64) * m,
                             loff=torch.zeros(B + 1, dtype=torch.int64, device=dev),
                             need=torch.zeros(1, dtype=torch.int64, device=dev),
                             locs=torch.zeros(cap, dtype=pdt_t, device=dev), cap=cap,
                             ws=torch.zeros(ixs.locate_workspace_size(B), dtype=torch.uint8, device=dev),
                             cnt=torch.zeros(B, dtype=pdt_t, device=dev)))
        torch.cuda.synchronize()

        def call(b):
            ixs.locate_batch_async(b["pat"].data_ptr(), b["off"].data_ptr(), B, b["loff"].data_ptr(),
                                   b["locs"].data_ptr(), b["cap"], b["need"].data_ptr(), b["ws"].data_ptr(),
                                   b["ws"].numel(), d_counts=b["cnt"].data_ptr(), stream=stream.cuda_stream,
                                   stage_kb=stage_kb, fixed_len=fixed)

        for b in bats:
            call(b)
        ixs.sync(stream.cuda_stream)
        calls, t0 = 0, time.perf_counter()
        while True:
            for b in bats:
                call(b)
            calls += len(bats)
            if time.perf_counter() - t0 >= min_seconds:
                break
        ixs.sync(stream.cuda_stream)
        el = time.perf_counter() - t0
        need = [int(b["need"].item()) for b in bats]
        if any(nd > b["cap"] for nd, b in zip(need, bats)):
            raise SystemExit("single_batch: location buffer too small")
        w1 = type("W", (), {})()
        w1.batches = [dict(n=B, loff=b["loff"], locs=b["locs"], starts=b["starts"]) for b in bats[:4]]
        out[name] = {"value": calls * B / el, "unit": "patterns/s", "us_per_batch": el / calls * 1e6,
                     "calls": calls, "self_location_check": self_location(w1, P)}
        ixs.release_stream(stream.cuda_stream)
        del bats
        ixs.close()
    return out


def arrange(torch, w, B, m, GR, dev, presorted, key_symbols=14, alphabet=b"ACGT"):
    """Experiments (weak configs, uniform batches): rearrange each launch
    group's patterns — sorted by reversed suffix (`presorted`: the last
    key_symbols symbols, digits over the text's alphabet), or so that
    workgroup tile t holds class-(t % 8) patterns (XCD-partitioned)."""
    if presorted:
        code = torch.zeros(256, dtype=torch.int64, device=dev)
        for i, c in enumerate(alphabet):
            code[c] = i
        base = len(alphabet)
        for g in range(w.n_groups):
            sel = w.batches[g * GR:(g + 1) * GR]
            st = torch.cat([b["starts"] for b in sel])
            pats = torch.stack([b["pat"].view(B, m) for b in sel]).view(-1, m).long()
            key = torch.zeros(st.numel(), dtype=torch.int64, device=dev)
            for q in range(min(m, key_symbols, int(62 / math.log2(base)))):
                key = key * base + code[pats[:, m - 1 - q]]
            order = torch.argsort(key, stable=True)
            st, pats = st[order], pats[order].to(torch.uint8)
            for j, b in enumerate(sel):
                b["starts"] = st[j * B:(j + 1) * B].contiguous()
                b["pat"].copy_(pats[j * B:(j + 1) * B].reshape(-1))
        return
    code = np.zeros(256, np.int64)
    code[list(b"ACGT")] = [0, 1, 2, 3]
    T = -(-B // 256)
    for g in range(w.n_groups):
        sel = w.batches[g * GR:(g + 1) * GR]
        st = torch.cat([b["starts"] for b in sel]).cpu().numpy()
        pats = torch.stack([b["pat"].view(B, m) for b in sel]).view(-1, m).cpu().numpy()
        cls = (code[pats[:, m - 1]] * 16 + code[pats[:, m - 2]] * 4 + code[pats[:, m - 3]]) % 8
        want = ((np.arange(len(sel))[:, None] * T + np.arange(B)[None, :] // 256) % 8).reshape(-1)
        order = np.empty(cls.size, np.int64)
        pools = [list(np.flatnonzero(cls == c)[::-1]) for c in range(8)]
        spill = []
        for u in range(cls.size):
            pool = pools[want[u]]
            if pool:
                order[u] = pool.pop()
            else:
                order[u] = -1
                spill.append(u)
        rest = [x for pl in pools for x in pl]
        order[spill] = rest
        st, pats = st[order], pats[order]
        for j, b in enumerate(sel):
            b["starts"] = torch.from_numpy(st[j * B:(j + 1) * B].copy()).to(dev)
            b["pat"].copy_(torch.from_numpy(pats[j * B:(j + 1) * B].reshape(-1).copy()).to(dev))


if __name__ == "__main__":
    main()
