"""World-size-2 tests of the multi-GPU plumbing on CPU (gloo): patterns are
sharded across ranks, each rank answers its slab against its own replica of
the index, and the concatenated result must equal the single-process answer.
The per-rank compute here is the CPU oracle (this tests the sharding and the
collectives, not the kernels — those are covered by tests/test_gpu.py)."""
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, result_path):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["FMX_NO_TORCH_RUNTIME"] = "1"
    import torch
    import torch.distributed as dist
    import __graft_entry__ as g
    from oracle import oracle as O
    from _util import table_from_symbols
    pkg = g.load_package()
    D = pkg.distributed
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    rng = np.random.default_rng(123)  # same text / patterns on every rank (replicated blob)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=20000).astype(np.uint8).tobytes()
    table = table_from_symbols([b"A", b"C", b"G", b"T", b"N"])
    L = O.layout(4, 3, 64, 0)
    ix = O.OracleIndex(O.build(text, 5, L, 3, 2, table), L)
    pats = [text[s:s + int(rng.integers(2, 14))] for s in rng.integers(0, len(text) - 14, size=1001)]
    data, offsets = pkg.pack_patterns(pats)
    s, e = D.shard(len(pats), world, rank)
    sd, so = D.slab_patterns(data, offsets, s, e)
    loff, locs = ix.locate_batch(sd, so)
    goff, glocs = D.concat_results(torch.from_numpy(loff.astype(np.int64)),
                                   torch.from_numpy(locs.astype(np.int64)))
    t = D.max_over_ranks(float(rank + 1))
    if rank == 0:
        ref_off, ref_locs = ix.locate_batch(data, offsets)
        ok = (np.array_equal(goff.numpy().astype(np.uint64), ref_off)
              and np.array_equal(glocs.numpy().astype(np.uint32), ref_locs) and t == float(world))
        with open(result_path, "w") as f:
            f.write("ok" if ok else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


def test_shard_partition(pkg):
    for n in (0, 1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            spans = [pkg.distributed.shard(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(e - s for s, e in spans) - min(e - s for s, e in spans) <= 1


def test_two_rank_gloo_concat_matches_single(tmp_path):
    import torch.multiprocessing as mp
    out = tmp_path / "res.txt"
    mp.spawn(_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    assert out.read_text() == "ok"
