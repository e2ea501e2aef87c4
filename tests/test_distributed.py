"""World-size-2 tests of the multi-GPU plumbing on CPU (gloo): patterns are
sharded across ranks, each rank answers its slab against its own replica of
the index, and the concatenated result must equal the single-process answer.
The per-rank compute here is the CPU oracle (this tests the sharding and the
gather bench.py uses — sharding.ShardGather's fixed-size all-gathers and
device-side assembly — not the kernels, which tests/test_gpu.py covers)."""
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
    # the gather bench.py runs: fixed-size slots the results are written into,
    # two all-gathers, no size exchange
    cap = torch.tensor([locs.size], dtype=torch.int64)
    dist.all_reduce(cap, op=dist.ReduceOp.MAX)  # a bound every rank's total stays under
    sizes = D.shard_sizes(len(pats), world)
    g = D.SlabGather(world, slots=2, batch=max(sizes), loc_cap=int(cap.item()), count_dtype=torch.int32,
                     loc_dtype=torch.int32, device="cpu")
    g.counts_slot(1)[:e - s] = torch.from_numpy(np.diff(loff).astype(np.int32))
    g.locs_slot(1)[:locs.size] = torch.from_numpy(locs.astype(np.int32))
    g.gather()
    goff, glocs = D.concat([g.result(r, 1, sizes[r]) for r in range(world)])
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


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_matches_single(tmp_path, world):
    """world 2 and 3 (ragged shards: 1001 patterns)."""
    import torch.multiprocessing as mp
    out = tmp_path / "res.txt"
    mp.spawn(_worker, args=(world, _free_port(), str(out)), nprocs=world, join=True)
    assert out.read_text() == "ok"
