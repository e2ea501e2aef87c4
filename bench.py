#!/usr/bin/env python3
"""Benchmark: patterns/sec (count + locate) on BASELINE.json's headline config.

Default workload (BASELINE.json configs[1], "C2"): 1 Gbp uniform ACGT text,
symbols ACGTN (N = wildcard, sigma 5), layout u32 / Block3<u64> /
EncodingTable, SA sampling 2, k-mer table k = 3; 100,000 x 20 bp patterns cut
from the text at uniform random starts (bench/src/generate.rs:105-113, cold
ratio 1.0), per GPU.  `--config c1|c3|c4|c5` selects the other BASELINE configs.

One step = one full count+locate pass over one batch in the fused k_locate
kernel: k-mer seed + LF loop, single-pass look-back scan of the counts into
output offsets, locations — every count (as offsets) and every location of
every pattern, written to that batch's own HBM outputs.  By default eight
steps' batches share one launch (fmx_locate_group_async; --group 1: one
launch per batch) and launches alternate over two streams; 32 distinct
batches are cycled so that no pass finds the previous pass's index lines in
cache.  Inputs (text, blob, derived index structures, patterns) are resident
in HBM before the timed region.

Multi-GPU: one process per GPU (torchrun); each rank builds its own replica of
the blob on its GPU (deterministic), runs its own pattern batch (weak scaling,
or a shard of --total-patterns), no collective in the timed region; the
results are concatenated over RCCL afterwards (timed separately).

Also reported: the dominant kernel's roofline (HIP events on the engine's
stream), a CPU baseline (the oracle restatement on this host, rank 0), and a
bit-exact check of the GPU results against it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
RANDOM_LINE_CEILING = 47.0  # G random 64-B line requests/s, 1-128 GB buffers, >=1M lanes (profiles/r01_randline.jsonl)
METRIC = "patterns/sec (count+locate), 1 Gbp text / 20 bp patterns, 1/2/4/8 MI355X"

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
               patterns=0, m=20, total=10_000_000,
               desc="C3: 1 Gbp ACGT, 10,000,000 x 20 bp sharded over the GPUs, u32/Block3<u64>, sr 2, k 3"),
    # configs[3]: large-alphabet occ path
    "c4": dict(text_len=1_000_000_000, alphabet=AMINO, symbols=[bytes([c, c + 32]) for c in AMINO] + [b"Xx"],
               pos=4, planes=5, vec=64, k=3, sr=2, patterns=100_000, m=12, total=0,
               desc="C4: 1 G-residue protein text (20 aa + X wildcard), 100,000 x 12 aa, u32/Block5<u64>, sr 2, k 3"),
    # configs[4]: long patterns, wide blocks, u64 positions
    "c5": dict(text_len=3_000_000_000, alphabet=b"ACGT", symbols=ACGTN, pos=8, planes=3, vec=128, k=3, sr=2,
               patterns=0, m=150, total=1_000_000,
               desc="C5: 3 Gbp ACGT, 1,000,000 x 150 bp sharded over the GPUs, u64/Block3<u128>, sr 2, k 3"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=800)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--text-len", type=int, default=0, help="override the config's text length")
    ap.add_argument("--patterns", type=int, default=0, help="patterns per GPU per step (weak scaling)")
    ap.add_argument("--total-patterns", type=int, default=-1,
                    help="> 0: one global batch sharded over the GPUs (strong scaling)")
    ap.add_argument("--pattern-len", type=int, default=0)
    ap.add_argument("--occ", default="interleaved", choices=["interleaved", "blob"])
    ap.add_argument("--no-deep-lut", action="store_true", help="do not build the device K-mer interval table")
    ap.add_argument("--options", type=int, default=-1,
                    help="fmx_load options bit field (FMX_OCC_INTERLEAVED=1|DEEP_LUT=2|FULL_SA=4|TEXT=8|"
                         "ROW_CONTEXT=16); "
                         "default: everything (minus --no-deep-lut)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="diagnostic: no HIP events around the launches in the timed region (no roofline)")
    ap.add_argument("--count-only", action="store_true", help="diagnostic: time fmx_count_batch_async (k_count)")
    ap.add_argument("--event-every", type=int, default=5,
                    help="bracket every k-th launch of the timed region with HIP events (an event pair costs the "
                         "stream several us; 1 = every launch)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (1 thread)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline / parity leg")
    ap.add_argument("--no-fixed-len", action="store_true",
                    help="A/B: do not pass FMX_HINT_FIXED_LEN (the kernels read each tile's offsets first)")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--streams", type=int, default=2,
                    help="launches in flight: launch q runs on HIP stream q %% S (each stream its own batches: "
                         "patterns, outputs and look-back workspaces), as a serving loop pipelines batches")
    ap.add_argument("--batches", type=int, default=32,
                    help="distinct pattern batches cycled over the steps (at least --streams)")
    ap.add_argument("--group", type=int, default=8,
                    help="batches per kernel launch in the timed region (fmx_locate_group_async, at most 8; "
                         "1 = one launch per batch)")
    ap.add_argument("--submit", default="native", choices=["native", "python"],
                    help="native: the timed steps are issued as one fmx_locate_jobs_async queue; "
                         "python: one fmx_locate_batch_async call per step")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_fetch_size.json"))
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


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
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    n = args.text_len or cfg["text_len"]
    m = args.pattern_len or cfg["m"]
    total = args.total_patterns if args.total_patterns >= 0 else cfg["total"]
    if args.patterns:
        total = 0
    if total > 0:
        s0, s1 = D.shard(total, world, rank)
        B = s1 - s0
    else:
        B = args.patterns or cfg["patterns"]
    P = cfg["pos"]
    BLK = cfg["planes"] * cfg["vec"] // 8
    pdt_t, pdt_np = (torch.int32, np.uint32) if P == 4 else (torch.int64, np.uint64)
    position = pkg.u32 if P == 4 else pkg.u64
    block = getattr(pkg.blocks, f"Block{cfg['planes']}")(pkg.Vector(cfg["vec"]))

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
    t2 = time.time()
    ix = pkg.FmIndex.load_device(d_blob.data_ptr(), blob_len, position, block, pkg.text_encoders.EncodingTable,
                                 device=local, occ=args.occ, deep_lut=not args.no_deep_lut,
                                 options=None if args.options < 0 else args.options)
    load_s = time.time() - t2
    info = ix.info()
    log(f"[rank {rank}] index loaded in {load_s:.2f}s: options={info['options']} deep_lut_k={info['deep_lut_k']} "
        f"device_bytes={info['device_bytes']:,}")

    # ---- patterns: substrings at uniform starts (per-rank, per-batch seed) ---
    # NB distinct batches (each its own patterns, outputs and look-back
    # workspace).  Steps run in groups of GR batches per kernel launch
    # (fmx_locate_group_async): batches form chunks of GR, chunk c always on
    # stream c % S, launch q on stream q % S takes that stream's chunks in
    # turn, so consecutive passes over one batch are NB steps apart (their
    # index lines are not still cached).  Batch 0 is the one checked against
    # the CPU oracle.
    S = max(1, args.streams)
    GR = max(1, min(args.group, 8))
    NB = -(-max(S * GR, args.batches) // (S * GR)) * (S * GR)  # whole chunks on every stream
    cap = 4 * B + 4096
    ws = ix.locate_workspace_size(B)
    streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    batches = []
    for bi in range(NB):
        pg = torch.Generator(device=dev)
        pg.manual_seed(args.seed * 1000 + 7 + rank + 100003 * bi)
        starts = torch.randint(0, n - m + 1, (B,), device=dev, dtype=torch.int64, generator=pg)
        batches.append(dict(
            stream=streams[(bi // GR) % S],
            starts=starts,
            pat=d_text[(starts[:, None] + torch.arange(m, device=dev)[None, :]).reshape(-1)].contiguous(),
            off=(torch.arange(B + 1, device=dev, dtype=torch.int64) * m).contiguous(),
            loff=torch.zeros(B + 1, dtype=torch.int64, device=dev),
            locs=torch.zeros(cap, dtype=pdt_t, device=dev),
            need=torch.zeros(1, dtype=torch.int64, device=dev),
            ws=torch.zeros(ws, dtype=torch.uint8, device=dev)))
    torch.cuda.synchronize()
    b0 = batches[0]
    starts, d_pat, d_loff, d_locs, d_need = b0["starts"], b0["pat"], b0["loff"], b0["locs"], b0["need"]
    state = {"i": 0}

    d_cnt = torch.zeros(B, dtype=pdt_t, device=dev)

    stage_kb = min(56, -(-256 * m // 1024))  # FMX_HINT_STAGE_KB: every tile spans 256 * m bytes
    fixed = 0 if args.no_fixed_len else m    # FMX_HINT_FIXED_LEN: every pattern is m bytes (checked on device)

    def job(bt):
        return ix.locate_job(bt["pat"].data_ptr(), bt["off"].data_ptr(), B, bt["loff"].data_ptr(),
                             bt["locs"].data_ptr(), cap, bt["need"].data_ptr(), bt["ws"].data_ptr(), ws,
                             stream=bt["stream"].cuda_stream, stage_kb=stage_kb, fixed_len=fixed)

    def step():
        bt = batches[state["i"] % NB]
        state["i"] += 1
        if args.count_only:  # diagnostic: the search alone (k_count)
            ix.count_batch_async(bt["pat"].data_ptr(), bt["off"].data_ptr(), B, d_cnt.data_ptr(),
                                 stream=bt["stream"].cuda_stream, stage_kb=stage_kb, fixed_len=fixed)
            return
        ix.locate_batch_async(bt["pat"].data_ptr(), bt["off"].data_ptr(), B, bt["loff"].data_ptr(),
                              bt["locs"].data_ptr(), cap, bt["need"].data_ptr(), bt["ws"].data_ptr(), ws,
                              stream=bt["stream"].cuda_stream, stage_kb=stage_kb, fixed_len=fixed)

    # native submission: the K steps of the timed region as ceil(K / GR)
    # grouped launches (GR = 1: one queue of K single-batch jobs)
    native = args.submit == "native" and not args.count_only
    queue, groups = None, []
    if native and GR == 1:
        queue = ix.job_queue([job(batches[i % NB]) for i in range(args.steps)])
    NC = NB // GR  # chunks of GR batches; chunk c runs on stream c % S

    def group_of(q, count=GR):
        # launch q: stream q % S, that stream's chunks in turn
        c = q % S + S * ((q // S) % (NC // S))
        sel = batches[c * GR:c * GR + count]
        return ix.job_queue([job(bt) for bt in sel]), sel[0]["stream"].cuda_stream

    if native and GR > 1:
        for q, i0 in enumerate(range(0, args.steps, GR)):
            groups.append(group_of(q, min(GR, args.steps - i0)))

    # warmup: the timed region's own launches (every batch at least once)
    if native and GR > 1:
        for q in range(max(-(-args.warmup // GR), NC)):
            gq, gs = group_of(q)
            ix.locate_group_async(gq, stream=gs)
    else:
        for _ in range(max(args.warmup, NB)):
            step()
    torch.cuda.synchronize()
    for bt in batches:
        ix.sync(bt["stream"].cuda_stream)
        need = int(bt["need"].item())
        if need > cap:
            raise SystemExit(f"location buffer too small: {need} > {cap}")
    state["i"] = 0

    # ---- timed region ------------------------------------------------------
    ix.timing_read()          # drain warmup events
    ix.timing_enable(not args.no_kernel_timing, every=args.event_every)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    if native and GR == 1:
        ix.locate_jobs_async(queue)
    elif native:
        for gq, gs in groups:
            ix.locate_group_async(gq, stream=gs)
    else:
        for _ in range(args.steps):
            step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        dist.barrier()
    ix.timing_enable(False)
    ix.sync()
    timing = ix.timing_read()
    if world > 1:
        elapsed = D.max_over_ranks(elapsed, device=dev)

    for bt in batches:
        ix.sync(bt["stream"].cuda_stream)

    # ---- result concatenation across ranks (RCCL all-gathers, untimed) -----
    gather_ms = None
    if world > 1:
        torch.cuda.synchronize()
        tg = time.perf_counter()
        g_off, g_locs = D.concat_results(d_loff, d_locs[:int(d_need.item())].to(torch.int64))
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3
        log(f"[rank {rank}] gathered {g_off.numel() - 1:,} patterns / {g_locs.numel():,} locations in {gather_ms:.2f} ms")

    # ---- roofline of the dominant kernel ------------------------------------
    # Algorithmic bytes: per pattern m + 2P (k-mer seed) +
    # L*2*(P+|B|) (two rank queries per LF step) + P (count), per occurrence
    # w*(P+|B|) (walk, E[w] = sr-1) + P (sampled SA) + P (location out).
    k, sr = info["kmer_size"], info["sampling_ratio"]
    offs_h = d_loff.cpu().numpy().view(np.uint64)
    total_occ = int(offs_h[-1])
    # every pattern is cut from the text, so its interval never empties and the
    # LF loop of the reference runs exactly m - k steps (with_slice.rs:27-31)
    L = m - k
    per_pattern = m + 2 * P + L * 2 * (P + BLK) + P
    per_occ = (sr - 1) * (P + BLK) + 2 * P
    kern = {name: t["total_ms"] / max(t["launches"], 1) for name, t in timing.items()}
    if "locate" not in kern:  # --no-kernel-timing
        kern["locate"] = float("nan")
    dominant = "locate"   # one grouped launch: k_search + k_emit (+ k_scan), or the fused k_locate
    if args.count_only:
        dominant = "count"
        kern.pop("locate", None)
    # a launch covers GR batches when grouped: patterns per timed launch
    # from the engine's own counters
    t_dom = timing.get(dominant, {})
    pats_per_launch = t_dom["units"] / t_dom["launches"] if t_dom.get("launches") else B
    alg_bytes = (per_pattern + per_occ * total_occ / B) * pats_per_launch
    achieved = alg_bytes / (kern[dominant] * 1e-3) / 1e9
    traffic, traffic_src = None, None
    key = f"{args.config}:{n}:{B}:{m}:{info['options']}:{info['deep_lut_k']}" + (f":g{GR}" if native and GR > 1 else "")
    if os.path.exists(args.traffic_json):
        try:
            pm = json.load(open(args.traffic_json))
            run = pm.get("runs", {}).get(key)
            if run and "hbm_bytes_per_launch" in run:
                traffic = run["hbm_bytes_per_launch"]
                traffic_src = f"{os.path.relpath(args.traffic_json, ROOT)} [{key}] (rocprofv3 FETCH_SIZE, " \
                              f"tag {run.get('tag')}, avg {run.get('avg_duration_ns', 0) / 1e3:.1f} us/launch)"
        except Exception:
            pass

    # size-independent property at full size, every batch: pattern i was cut
    # at starts[i], so starts[i] must be one of its locations
    self_found = True
    for bt in batches:
        bo = bt["loff"].cpu().numpy().view(np.uint64)
        bl = bt["locs"][:int(bo[-1])].cpu().numpy().view(pdt_np)
        st_h = bt["starts"].cpu().numpy()
        cnt_h = np.diff(bo).astype(np.int64)
        owner = np.repeat(np.arange(B), cnt_h)
        hit = np.zeros(B, dtype=bool)
        hit[owner[bl.astype(np.int64) == st_h[owner]]] = True
        self_found = self_found and bool(hit.all() and (cnt_h >= 1).all())
    locs_h = d_locs[:total_occ].cpu().numpy().view(pdt_np)

    b_all = torch.tensor([B], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(b_all)
    value = int(b_all.item()) * args.steps / elapsed
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "patterns/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if total > 0 else "weak",
        "vs_baseline": None,
        "dtype": "u32" if P == 4 else "u64",
        "data": f"synthetic: seeded uniform {cfg['alphabet'].decode()} text; patterns cut from it at uniform "
                f"random starts",
        "config": {
            "workload": cfg["desc"] if (n == cfg["text_len"] and m == cfg["m"]) else
            f"{args.config} variant: {n:,}-symbol text, {B:,} x {m} patterns per GPU",
            "config": args.config, "text_len": n, "patterns_per_gpu": B, "pattern_len": m,
            "global_batch": int(b_all.item()),
            "layout": f"u{P * 8}/Block{cfg['planes']}<u{cfg['vec']}>/EncodingTable(sigma={table.symbol_count()})",
            "load_options": info["options"], "deep_lut_k": info["deep_lut_k"],
            "index_hbm_bytes": info["device_bytes"],
            "parallelism": f"dp{world} (patterns sharded, blob replicated)",
            "streams": S, "fixed_len_hint": fixed, "batches_per_launch": GR if native else 1, "distinct_batches": NB, "submit": "native" if native else "python",
        },
        "roofline": {
            "bound": "hbm", "kernel": dominant, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
            "achieved_basis": "reference algorithm's bytes per pattern (SURVEY.md 8(d)) x patterns per launch / "
                              "launch time; the derived index structures skip most of those bytes, so frac can "
                              "exceed 1 - traffic_frac is this kernel's own measured HBM traffic over peak",
            "alg_bytes_per_launch": alg_bytes, "alg_bytes_per_pattern": alg_bytes / pats_per_launch,
            "patterns_per_launch": pats_per_launch,
            "avg_launch_ms": kern.get(dominant),
            # the binding resource of a dependent-gather kernel: 64-B HBM line
            # requests per second vs the measured random-line ceiling
            # (scripts/micro/randline.hip, profiles/r01_randline.jsonl)
            "hbm_lines_per_pattern": None if traffic is None else traffic / 64 / pats_per_launch,
            "hbm_glines_per_s": None if traffic is None else traffic / 64 / (kern[dominant] * 1e-3) / 1e9,
            "random_line_ceiling_glines_per_s": RANDOM_LINE_CEILING,
            # what the kernel itself moves (PMC FETCH_SIZE) against the peak:
            # `achieved` credits the reference algorithm's bytes,
            # most of which the derived index structures never read
            "traffic_gbs": None if traffic is None else traffic / (kern[dominant] * 1e-3) / 1e9,
            "traffic_frac": None if traffic is None else traffic / (kern[dominant] * 1e-3) / 1e9 / HBM_PEAK_GBS,
        },
        "kernels_ms_per_launch": kern,
        "occurrences_per_step": total_occ,
        "self_location_check": self_found,
        "build_s": build_s,
        "load_s": load_s,
        "gather_ms": gather_ms,
        "profile_key": key,
    }

    # ---- CPU baseline + bit-exact check (rank 0, N=1 only) -------------------
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import oracle as O
        host_blob = O.aligned_zeros(blob_len, 16)
        host_blob[:] = d_blob.cpu().numpy()
        orc = O.OracleIndex(host_blob, O.layout(P, cfg["planes"], cfg["vec"], 0))
        pats_h = d_pat.cpu().numpy()
        offs_in = np.arange(B + 1, dtype=np.uint64) * m
        # 1 thread, whole passes over the batch until the budget is spent
        done, tc = 0, time.perf_counter()
        ooff = olocs = None
        while True:
            ooff, olocs = orc.locate_batch(pats_h, offs_in, threads=1, cap=cap)
            done += B
            if time.perf_counter() - tc >= args.cpu_seconds:
                break
        cpu1 = done / (time.perf_counter() - tc)
        tc = time.perf_counter()
        orc.locate_batch(pats_h, offs_in, threads=args.cpu_threads, cap=cap)
        cpun = B / (time.perf_counter() - tc)
        exact = bool(np.array_equal(ooff, offs_h) and np.array_equal(olocs, locs_h))
        try:
            model = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
        except Exception:
            model = "unknown"
        result["cpu_baseline"] = {
            "value": cpu1, "unit": "patterns/s", "cores": 1, "kind": "port",
            "sample": f"{done:,} patterns = {done // B} passes over the same {B:,}-pattern batch, "
                      f"oracle/fmx_oracle.c (C restatement of the reference query path), blob in RAM",
            f"value_{args.cpu_threads}_threads": cpun, "cpu_model": model, "host_cpus_visible": os.cpu_count(),
        }
        result["parity"] = {"bit_exact_vs_cpu": exact, "patterns": B, "occurrences": total_occ}
        result["speedup_vs_cpu_1thread"] = value / cpu1
        result[f"speedup_vs_cpu_{args.cpu_threads}_threads"] = value / cpun
        if not exact:
            log("PARITY FAILURE: GPU results differ from the CPU oracle")

    if rank == 0:
        print(json.dumps(result), flush=True)
    ix.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
