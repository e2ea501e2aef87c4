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
seed, the LF loop over the bit planes, the sr = 2 sampled-SA walk
(`--options 0` reads the blob's arrays as they lie).  The derived-index mode
(deep K-mer table, full SA, text: ~147 GB of HBM at C2) is measured after it
and reported as the labelled sub-object "derived".

One step = one full count+locate pass over one batch: k-mer seed + LF loop
for every pattern, the walk of every occurrence row, output offsets and all
locations written to that batch's own HBM outputs.  Eight steps' batches share
one kernel launch (fmx_locate_group_async) and launches alternate over two
streams; 32 distinct batches are cycled so that no pass finds the previous
pass's index lines in cache.  Inputs (text, blob, index, patterns) are
resident in HBM before the timed region.  The K steps are timed as a whole
and repeated until the timed region lasts at least --min-seconds (0.2 s):
a few-hundred-microsecond region is noise.

Multi-GPU: one process per GPU (torchrun); each rank builds its own replica of
the blob on its GPU (deterministic).  c2 (weak scaling): each rank runs its
own batches with no collective in the timed region; every batch's counts and
locations are then all-gathered over RCCL (gather.gather_ms).  c3/c5 (strong
scaling): the job is dealt out in 100 k batches, rank r taking batches
r, r+N, ...; each launch's results are all-gathered on a communication stream
while the next launch computes, inside the timed step (`value`), and the
compute alone is timed too (gather.value_compute_only).

Also reported: the locate launch's roofline (HIP events on the engine's
streams), the CPU baseline (the oracle restatement on this host's usable
cores, rank 0), and a bit-exact check of the GPU results against it.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# G dependent random 128-B line reads/s over a 0.5-1 GB buffer (the C2 occ records: 1 GB), 0.5-2 M
# chains: 52-54 (profiles/r2_footprint.jsonl, profiles/r2_shapes.jsonl; scripts/micro/shapes.hip).
# Round 1 quoted 47 from 8-128 GB buffers (profiles/r01_randline.jsonl), where TLB reach costs more.
RANDOM_LINE_CEILING = 52.0
METRIC = "patterns/sec (count+locate), 1 Gbp text / 20 bp patterns, 1/2/4/8 MI355X"
FAITHFUL = 1  # FMX_OCC_INTERLEAVED: the blob's own planes and checkpoints, one record per block
DERIVED = 63  # + deep K-mer table, full SA, text, row contexts, single-row entries

ACGTN = [b"Aa", b"Cc", b"Gg", b"Tt", b"Nn"]
AMINO = b"ACDEFGHIKLMNPQRSTVWY"
CONFIGS = {
    # BASELINE.json configs[0]: the reference's CPU-runnable plumbing case (T is the wildcard)
    "c1": dict(text_len=1_000_000, alphabet=b"ACGT", symbols=[b"Aa", b"Cc", b"Gg", b"Tt"], pos=4, planes=2,
               vec=64, k=3, sr=2, patterns=1_000, m=20, total=0,
               desc="C1: 1 Mbp ACGT, 1,000 x 20 bp, u32/Block2<u64>, sr 2, k 3"),
    # configs[1]: the headline (metric quoted on it)
    "c2": dict(text_len=1_000_000_000, alphabet=b"ACGT", symbols=ACGTN, pos=4, planes=3, vec=64, k=3, sr=2,
               patterns=100_000, m=20, total=0,
               desc="C2: 1 Gbp ACGT (ACGTN, N wildcard), 100,000 x 20 bp per GPU, u32/Block3<u64>, sr 2, k 3"),
    # configs[2]: 10 M patterns sharded over the GPUs
    "c3": dict(text_len=1_000_000_000, alphabet=b"ACGT", symbols=ACGTN, pos=4, planes=3, vec=64, k=3, sr=2,
               patterns=100_000, m=20, total=10_000_000,
               desc="C3: 1 Gbp ACGT, 10,000,000 x 20 bp sharded over the GPUs, u32/Block3<u64>, sr 2, k 3"),
    # configs[3]: large-alphabet occ path
    "c4": dict(text_len=1_000_000_000, alphabet=AMINO, symbols=[bytes([c, c + 32]) for c in AMINO] + [b"Xx"],
               pos=4, planes=5, vec=64, k=3, sr=2, patterns=100_000, m=12, total=0,
               desc="C4: 1 G-residue protein text (20 aa + X wildcard), 100,000 x 12 aa, u32/Block5<u64>, sr 2, k 3"),
    # configs[4]: long patterns, wide blocks, u64 positions (1 M patterns over the GPUs)
    "c5": dict(text_len=3_000_000_000, alphabet=b"ACGT", symbols=ACGTN, pos=8, planes=3, vec=128, k=3, sr=2,
               patterns=100_000, m=150, total=1_000_000,
               desc="C5: 3 Gbp ACGT, 1,000,000 x 150 bp sharded over the GPUs, u64/Block3<u128>, sr 2, k 3"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=0,
                    help="batches per timed pass (default: 800, or the whole sharded job for c3/c5)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--text-len", type=int, default=0, help="override the config's text length")
    ap.add_argument("--patterns", type=int, default=0, help="patterns per batch")
    ap.add_argument("--total-patterns", type=int, default=-1,
                    help="> 0: one global job of this many patterns dealt out over the GPUs in batches")
    ap.add_argument("--pattern-len", type=int, default=0)
    ap.add_argument("--options", type=int, default=FAITHFUL,
                    help="fmx_load options of the headline index (1 = FMX_OCC_INTERLEAVED, 0 = blob layout)")
    ap.add_argument("--derived-options", type=int, default=DERIVED,
                    help="options of the derived-index leg (reported under 'derived')")
    ap.add_argument("--no-derived", action="store_true", help="skip the derived-index leg")
    ap.add_argument("--min-seconds", type=float, default=0.2, help="minimum timed region (passes repeated)")
    ap.add_argument("--event-every", type=int, default=5,
                    help="bracket every k-th launch of the timed region with HIP events")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline budget per leg")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: all usable cores)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline / parity leg")
    ap.add_argument("--no-fixed-len", action="store_true",
                    help="A/B: do not pass FMX_HINT_FIXED_LEN (the kernels read each tile's offsets first)")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--streams", type=int, default=2, help="launches in flight (HIP streams)")
    ap.add_argument("--batches", type=int, default=32, help="distinct batches cycled (weak-scaling configs)")
    ap.add_argument("--group", type=int, default=8, help="batches per kernel launch (at most 16)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--xcd-partitioned", action="store_true",
                    help="experiment: each launch group's patterns arranged so that workgroup tile t (XCD t %% 8) "
                         "holds only patterns whose last 3 symbols fall in class t %% 8 (upper bound of an "
                         "XCD-aware partition; not a valid headline workload)")
    ap.add_argument("--presorted", action="store_true",
                    help="experiment: each launch group's patterns pre-sorted by reversed suffix (upper bound of "
                         "the cache reuse a suffix sort would buy; not a valid headline workload)")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


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


class Workload:
    """The batches of one rank: patterns cut from the device text, per-batch
    outputs and workspaces; launch groups of up to GR batches, group q on
    stream q % S.  With `slabs`, batch k writes its counts and locations
    straight into slot k % GR of gather slab k // GR."""

    def __init__(self, torch, ix, d_text, n, m, B, batch_ids, P, S, GR, fixed, dev, seed, rank, slabs=None,
                 presorted=False, xcd_partitioned=False):
        self.ix, self.B = ix, B
        pdt = torch.int32 if P == 4 else torch.int64
        self.cap = B + B // 8 + 4096  # checked against every batch's total at warmup
        self.ws = ix.locate_workspace_size(B)
        self.streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
        stage_kb = min(56, -(-256 * m // 1024))  # FMX_HINT_STAGE_KB: a tile spans 256 * m bytes
        self.batches = []
        for k, bi in enumerate(batch_ids):
            pg = torch.Generator(device=dev)
            # a sharded job's batch bi is the same on any rank; weak-scaling ranks differ
            pg.manual_seed(seed * 1000 + 7 + 100003 * bi + (0 if slabs else 7919 * rank))
            starts = torch.randint(0, n - m + 1, (B,), device=dev, dtype=torch.int64, generator=pg)
            g, j = divmod(k, GR)
            bt = dict(id=bi, group=g, slot=j, starts=starts,
                      pat=d_text[(starts[:, None] + torch.arange(m, device=dev)[None, :]).reshape(-1)].contiguous(),
                      off=(torch.arange(B + 1, device=dev, dtype=torch.int64) * m).contiguous(),
                      loff=torch.zeros(B + 1, dtype=torch.int64, device=dev),
                      need=torch.zeros(1, dtype=torch.int64, device=dev),
                      ws_t=torch.zeros(self.ws, dtype=torch.uint8, device=dev))
            if slabs is not None:
                bt["cnt"], bt["locs"] = slabs[g].counts_slot(j), slabs[g].locs_slot(j)
            else:
                bt["cnt"] = torch.zeros(B, dtype=pdt, device=dev)
                bt["locs"] = torch.zeros(self.cap, dtype=pdt, device=dev)
            self.batches.append(bt)
        if presorted:  # experiment: sort each group's patterns by their reversed last 14 symbols
            code = torch.zeros(256, dtype=torch.int64, device=dev)
            for i, c in enumerate(b"ACGT"):
                code[c] = i
            for g in range(-(-len(self.batches) // GR)):
                sel = self.batches[g * GR:(g + 1) * GR]
                st = torch.cat([b["starts"] for b in sel])
                pats = torch.stack([b["pat"].view(B, m) for b in sel]).view(-1, m).long()
                key = torch.zeros(st.numel(), dtype=torch.int64, device=dev)
                for q in range(min(m, 14)):
                    key = key * 4 + code[pats[:, m - 1 - q]]
                order = torch.argsort(key)
                st, pats = st[order], pats[order].to(torch.uint8)
                for j, b in enumerate(sel):
                    b["starts"] = st[j * B:(j + 1) * B].contiguous()
                    b["pat"].copy_(pats[j * B:(j + 1) * B].reshape(-1))
        if xcd_partitioned:  # experiment: tile t of a launch holds class-(t % 8) patterns only
            import numpy as np
            code = np.zeros(256, np.int64)
            code[list(b"ACGT")] = [0, 1, 2, 3]
            T = -(-B // 256)
            for g in range(-(-len(self.batches) // GR)):
                sel = self.batches[g * GR:(g + 1) * GR]
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
        self.groups = []
        for g in range(-(-len(self.batches) // GR)):
            sel = self.batches[g * GR:(g + 1) * GR]
            q = ix.job_queue([ix.locate_job(b["pat"].data_ptr(), b["off"].data_ptr(), B, b["loff"].data_ptr(),
                                            b["locs"].data_ptr(), self.cap, b["need"].data_ptr(),
                                            b["ws_t"].data_ptr(), self.ws, d_counts=b["cnt"].data_ptr(),
                                            stage_kb=stage_kb, fixed_len=fixed) for b in sel])
            self.groups.append(dict(queue=q, stream=self.streams[g % S], batches=sel))
        self.cursor = 0

    def launch(self, g):
        grp = self.groups[g]
        self.ix.locate_group_async(grp["queue"], stream=grp["stream"].cuda_stream)
        return grp

    def launch_next(self):
        """The next launch group in a cycle that runs on across passes (so the
        streams keep alternating however many launches a pass has)."""
        g = self.cursor % len(self.groups)
        self.cursor += 1
        return g, self.launch(g)

    def check_capacity(self):
        for grp in self.groups:
            self.ix.sync(grp["stream"].cuda_stream)
        need = max(int(b["need"].item()) for b in self.batches)
        if need > self.cap:
            raise SystemExit(f"location buffer too small: {need} > {self.cap}")


def timed_passes(torch, dist, dist_on, w, steps, warmup, min_seconds, event_every, on_launch=None, drain=None):
    """Warm up (every launch group at least once), then time passes of
    `steps` batches (ceil(steps / GR) launches of GR batches, groups cycled)
    until the region lasts min_seconds.  Returns (elapsed_s, passes,
    batches_per_pass, timing)."""
    ix = w.ix
    ng = len(w.groups)
    GR = len(w.groups[0]["batches"])
    per_pass = -(-steps // GR)
    for q in range(max(-(-warmup // GR), ng)):
        w.launch(q % ng)
    torch.cuda.synchronize()
    w.check_capacity()
    w.cursor = 0
    batches = 0

    def one_pass():
        nonlocal batches
        for _ in range(per_pass):
            gi, grp = w.launch_next()
            batches += len(grp["batches"])
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
    batches = 0
    t0 = time.perf_counter()
    for _ in range(passes):
        one_pass()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist_on:
        dist.barrier()
    ix.timing_enable(False)
    return elapsed, passes, batches // passes, ix.timing_read()


def self_location(w, P):
    """Size-independent property at full size, every batch: pattern i was cut
    at starts[i], so starts[i] is among its locations (and counts >= 1)."""
    ok = True
    pdt_np = np.uint32 if P == 4 else np.uint64
    for bt in w.batches:
        bo = bt["loff"].cpu().numpy().view(np.uint64)
        bl = bt["locs"][:int(bo[-1])].cpu().numpy().view(pdt_np)
        st = bt["starts"].cpu().numpy()
        cnt = np.diff(bo).astype(np.int64)
        owner = np.repeat(np.arange(w.B), cnt)
        hit = np.zeros(w.B, dtype=bool)
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


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import __graft_entry__ as g
    pkg = g.load_package()
    D = pkg.distributed
    cfg = dict(CONFIGS[args.config])

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # FMX_BENCH_BACKEND=gloo: a rehearsal of the multi-rank path with several
    # ranks on one GPU (RCCL needs one device per rank)
    backend = os.environ.get("FMX_BENCH_BACKEND", "nccl")
    gpu = local % max(torch.cuda.device_count(), 1)
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
    local = gpu

    n = args.text_len or cfg["text_len"]
    m = args.pattern_len or cfg["m"]
    B = args.patterns or cfg["patterns"]
    total = args.total_patterns if args.total_patterns >= 0 else cfg["total"]
    P = cfg["pos"]
    S = max(1, args.streams)
    GR = max(1, min(args.group, 8))
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
    builder.build_device(d_text.data_ptr(), d_blob.data_ptr(), blob_len, device=local)
    torch.cuda.synchronize()
    build_s = time.time() - t1
    log(f"[rank {rank}] text {n:,} B generated in {t1 - t0:.2f}s, blob {blob_len:,} B built on GPU in {build_s:.2f}s")

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

    t2 = time.time()
    ix = pkg.FmIndex.load_device(d_blob.data_ptr(), blob_len, position, block, pkg.text_encoders.EncodingTable,
                                 device=local, options=args.options)
    torch.cuda.synchronize()
    load_s = time.time() - t2
    info = ix.info()
    log(f"[rank {rank}] index loaded in {load_s:.3f}s: options={info['options']} device_bytes={info['device_bytes']:,}")

    fixed = 0 if args.no_fixed_len else m
    strong = total > 0
    slabs = None
    if strong:
        # the global job: nb batches of B, batch b on rank b % world
        nb = -(-total // B)
        if nb * B != total:
            raise SystemExit(f"--total-patterns must be a multiple of the batch size {B}")
        my_ids = list(range(rank, nb, world))
        n_groups = -(-(-(-nb // world)) // GR)  # launch groups of the rank with the most batches
        cap_b = B + B // 8 + 4096
        slabs = [D.SlabGather(world, GR, B, cap_b, pdt_t, pdt_t, dev) for _ in range(n_groups)]
        w = Workload(torch, ix, d_text, n, m, B, my_ids, P, S, GR, fixed, dev, args.seed, rank, slabs=slabs)
        steps = len(my_ids)
        if len(w.groups) < n_groups:
            raise SystemExit("every rank needs the same number of launch groups (use a job of world * GR batches)")
    else:
        NB = -(-max(S * GR, args.batches) // (S * GR)) * (S * GR)  # whole groups on every stream
        w = Workload(torch, ix, d_text, n, m, B, list(range(NB)), P, S, GR, fixed, dev, args.seed, rank,
                     presorted=args.presorted, xcd_partitioned=args.xcd_partitioned)
        steps = args.steps or 800
    torch.cuda.synchronize()

    # ---- timed region: compute ----------------------------------------------
    elapsed, passes, per_pass, timing = timed_passes(torch, dist, dist_on, w, steps, args.warmup, args.min_seconds,
                                                     args.event_every)
    if dist_on:
        elapsed = D.max_over_ranks(elapsed, device=dev)
    # every batch a launch ran counts (a pass of K steps runs ceil(K / GR) whole launches)
    pt = torch.tensor([per_pass * B * passes], dtype=torch.int64, device=dev)
    if dist_on:
        dist.all_reduce(pt)
    value_compute = int(pt.item()) / elapsed

    # ---- gathers -------------------------------------------------------------
    gather = None
    value = value_compute
    if dist_on and strong:
        # the same passes with each launch's results all-gathered on a
        # communication stream while the next launch computes
        comm = torch.cuda.Stream(device=dev)
        works = []

        def on_launch(gi, grp):
            ev = torch.cuda.Event()
            ev.record(grp["stream"])
            comm.wait_event(ev)
            with torch.cuda.stream(comm):
                works.append(slabs[gi].gather(async_op=True))

        def drain():
            for ws in works:
                for wk in ws:
                    if wk is not None:
                        wk.wait()
            works.clear()
            torch.cuda.current_stream().wait_stream(comm)

        e2, p2, _, _ = timed_passes(torch, dist, dist_on, w, steps, 0, args.min_seconds, args.event_every,
                                    on_launch=on_launch, drain=drain)
        e2 = D.max_over_ranks(e2, device=dev)
        value = total * p2 / e2
        # check: every rank's batches arrived (rank 0 reads the last rank's first slot)
        o, l = slabs[0].result(world - 1, 0, B)
        gather = {"inside_timed_step": True, "value_compute_only": value_compute,
                  "bytes_gathered_per_pass": sum(s.bytes_per_gather() for s in slabs),
                  "slot_check": bool(int(o[-1].item()) == l.numel() and l.numel() >= B)}
    elif dist_on:
        # weak scaling: every batch's counts and locations, after the timed region
        slab = D.SlabGather(world, len(w.batches), B, w.cap, pdt_t, pdt_t, dev)
        torch.cuda.synchronize()
        tg = time.perf_counter()
        for j, bt in enumerate(w.batches):
            slab.counts_slot(j).copy_(bt["cnt"], non_blocking=True)
            slab.locs_slot(j).copy_(bt["locs"][:w.cap], non_blocking=True)
        slab.gather()
        torch.cuda.synchronize()
        gather = {"inside_timed_step": False, "gather_ms": (time.perf_counter() - tg) * 1e3,
                  "bytes_gathered": slab.bytes_per_gather(), "batches": len(w.batches)}
        o, l = slab.result(rank, 0, B)  # this rank's batch 0 came back intact
        gather["roundtrip_ok"] = bool(torch.equal(o, w.batches[0]["loff"]) and
                                      torch.equal(l, w.batches[0]["locs"][:l.numel()]))

    # ---- roofline of the locate launch ----------------------------------------
    # Algorithmic bytes: per pattern m + 2P (k-mer seed) +
    # L*2*(P+|B|) (two rank queries per LF step) + P (count), per occurrence
    # w*(P+|B|) (walk, E[w] = sr-1) + P (sampled SA) + P (location out).
    k, sr = info["kmer_size"], info["sampling_ratio"]
    b0 = w.batches[0]
    offs_h = b0["loff"].cpu().numpy().view(np.uint64)
    total_occ = int(offs_h[-1])
    # every pattern is cut from the text, so its interval never empties and the
    # reference's LF loop runs exactly m - k steps (with_slice.rs:27-31)
    L = m - k
    per_pattern = m + 2 * P + L * 2 * (P + BLK) + P
    per_occ = (sr - 1) * (P + BLK) + 2 * P
    alg_per_pattern = per_pattern + per_occ * total_occ / B
    t_loc = timing.get("locate", {})
    launch_ms = t_loc["total_ms"] / t_loc["launches"] if t_loc.get("launches") else float("nan")
    pats_per_launch = t_loc["units"] / t_loc["launches"] if t_loc.get("launches") else B * GR
    achieved = alg_per_pattern * pats_per_launch / (launch_ms * 1e-3) / 1e9
    per_gpu = value_compute / max(world, 1)
    key = f"{args.config}:{n}:{B}:{m}:{info['options']}:g{GR}"
    tr = traffic_of(args.traffic_json, key)
    roof = {
        "bound": "hbm", "kernel": "locate launch (k_search + k_emit)", "achieved": achieved, "peak": HBM_PEAK_GBS,
        "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
        "traffic": tr["hbm_bytes_per_launch"] if tr else None,
        "achieved_basis": "reference algorithm's bytes per pattern (SURVEY.md 8(d)) x patterns per launch / "
                          "average launch duration (HIP events on the launch streams; with 2 streams in flight a "
                          "launch shares the GPU with the other stream's, so this understates the rate, see "
                          "achieved_effective = bytes per pattern x the timed region's patterns/s per GPU)",
        "alg_bytes_per_pattern": alg_per_pattern, "patterns_per_launch": pats_per_launch,
        "avg_launch_ms": launch_ms,
        "achieved_effective": alg_per_pattern * per_gpu / 1e9,
        "frac_effective": alg_per_pattern * per_gpu / 1e9 / HBM_PEAK_GBS,
    }
    if tr:
        req = tr.get("hbm_requests_per_launch")
        tpp = tr["hbm_bytes_per_launch"] / tr.get("patterns_per_launch", pats_per_launch)
        roof.update({
            "traffic_source": f"{os.path.relpath(args.traffic_json, ROOT)} [{key}] ({tr.get('source')})",
            "traffic_bytes_per_pattern": tpp,
            "traffic_frac_effective": tpp * per_gpu / 1e9 / HBM_PEAK_GBS,
        })
        if req:
            rpp = req / tr.get("patterns_per_launch", pats_per_launch)
            roof.update({"hbm_requests_per_pattern": rpp, "hbm_grequests_per_s": rpp * per_gpu / 1e9,
                         "random_line_ceiling_grequests_per_s": RANDOM_LINE_CEILING})

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "patterns/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / (per_pass * passes) * 1e3,
        "timed_passes": passes,
        "batches_per_pass": per_pass,
        "timed_region_s": elapsed,
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
        },
        "roofline": roof,
        "kernels_ms_per_launch": per_launch_ms(timing),
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
        "profile_key": key,
    }

    # ---- derived-index mode (labelled variant, N = 1) ------------------------
    if world == 1 and not args.no_derived:
        keep_b0 = b0
        w = None
        torch.cuda.synchronize()
        td = time.time()
        ixd = pkg.FmIndex.load_device(d_blob.data_ptr(), blob_len, position, block, pkg.text_encoders.EncodingTable,
                                      device=local, options=args.derived_options)
        torch.cuda.synchronize()
        load_d = time.time() - td
        infod = ixd.info()
        NB = -(-max(S * GR, args.batches) // (S * GR)) * (S * GR)
        wd = Workload(torch, ixd, d_text, n, m, B, list(range(NB)), P, S, GR, fixed, dev, args.seed, rank)
        dsteps = 800 if strong else steps
        ed, pd, dpp, td_t = timed_passes(torch, dist, dist_on, wd, dsteps, args.warmup, args.min_seconds,
                                         args.event_every)
        done_d = torch.tensor([dpp * B * pd], dtype=torch.int64, device=dev)
        if dist_on:  # whole job, like the headline: every rank's work over the slowest rank's time
            ed = D.max_over_ranks(ed, device=dev)
            dist.all_reduce(done_d)
        vd = int(done_d.item()) / ed
        dt = 1.0 / value_compute - 1.0 / vd  # seconds saved per pattern
        result["derived"] = {
            "value": vd, "unit": "patterns/s", "options": infod["options"], "deep_lut_k": infod["deep_lut_k"],
            "index_hbm_bytes": blob_len + infod["device_bytes"], "load_s": load_d,
            "breakeven_patterns": (load_d - load_s) / dt if dt > 0 else None,
            "kernels_ms_per_launch": per_launch_ms(td_t),
            "self_location_check": self_location(wd, P),
            "what": "the same queries over structures derived from the blob at load: a K-mer interval table "
                    "replaces the first LF steps, single-row entries and row records settle most patterns with "
                    "one or two reads, the full SA replaces the walk",
        }
        wd = None
        ixd.close()
        b0 = keep_b0

    # ---- CPU baseline + bit-exact check (rank 0, N=1 only) -------------------
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import oracle as O
        host_blob = O.aligned_zeros(blob_len, 16)
        host_blob[:] = d_blob.cpu().numpy()
        orc = O.OracleIndex(host_blob, O.layout(P, cfg["planes"], cfg["vec"], 0))
        pats_h = b0["pat"].cpu().numpy()
        offs_in = np.arange(B + 1, dtype=np.uint64) * m
        cores, src = usable_cores()
        threads = args.cpu_threads or cores
        legs = {}
        ooff = olocs = None
        for th in sorted({1, threads}):
            done, tc = 0, time.perf_counter()
            while True:
                ooff, olocs = orc.locate_batch(pats_h, offs_in, threads=th, cap=4 * B + 4096)
                done += B
                if time.perf_counter() - tc >= args.cpu_seconds:
                    break
            legs[th] = (done / (time.perf_counter() - tc), done)
        locs_h = b0["locs"][:total_occ].cpu().numpy().view(pdt_np)
        exact = bool(np.array_equal(ooff, offs_h) and np.array_equal(olocs, locs_h))
        try:
            model = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
        except (OSError, IndexError):
            model = "unknown"
        result["cpu_baseline"] = {
            "value": legs[threads][0], "unit": "patterns/s", "cores": threads, "kind": "port",
            "sample": f"{legs[threads][1]:,} patterns = whole passes over the GPU's batch 0 ({B:,} patterns) "
                      f"for >= {args.cpu_seconds:.0f} s on {threads} threads, oracle/fmx_oracle.c (C restatement "
                      f"of the reference query path), blob in RAM",
            "value_1_thread": legs[1][0], "cores_source": src, "cpu_model": model,
            "host_cpus_visible": os.cpu_count(),
        }
        result["parity"] = {"bit_exact_vs_cpu": exact, "patterns": B, "occurrences": total_occ}
        result["speedup_vs_cpu"] = value / legs[threads][0]
        result["speedup_vs_cpu_1_thread"] = value / legs[1][0]
        if not exact:
            log("PARITY FAILURE: GPU results differ from the CPU oracle")

    if rank == 0:
        print(json.dumps(result), flush=True)
    ix.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
