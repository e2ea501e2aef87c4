"""distributed.ShardedLocate on the GPU: one global batch answered by every
rank's shard on its own index, one packed all-gather, the batch's
(offsets, locations) assembled on the device — compared with one index's
answer (which the other GPU tests pin to the oracle).  One rank without a
process group, and two gloo ranks sharing cuda:0."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _case(pkg):
    rng = np.random.default_rng(77)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=2_000_000).astype(np.uint8)
    table = pkg.text_encoders.EncodingTable.from_symbols([b"Aa", b"Cc", b"Gg", b"Tt", b"Nn"])
    block = pkg.blocks.Block3(pkg.Vector.U64)
    b = (pkg.FmIndexBuilder(text.size, 5, table, pkg.u32, block)
         .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(3))
         .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(2)))
    blob = pkg.aligned_buffer(b.blob_size())
    b.build(text, blob)
    # ragged lengths; 2-4 bp patterns have tens of thousands of occurrences
    pats = [text[s:s + int(rng.integers(2, 25))].tobytes() for s in rng.integers(0, text.size - 25, 30001)]
    return blob, block, table, pats


def _run(pkg, dev):
    import torch
    blob, block, table, pats = _case(pkg)
    ix = pkg.FmIndex.load(blob, pkg.u32, block, table, device=dev.index or 0)
    want = ix.locate_batch(pats)
    data, offs = pkg.pack_patterns(pats)
    d_bytes = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64).copy()).to(dev)
    sl = pkg.distributed.ShardedLocate(ix, device=dev)
    got_off, got_locs = sl.locate(d_bytes, d_offs)
    ok = (np.array_equal(got_off.cpu().numpy().view(np.uint64), want[0]) and
          np.array_equal(got_locs.cpu().numpy().view(np.uint32), want[1]))
    ix.close()
    return ok, sl.last


def test_sharded_locate_one_rank(pkg):
    import torch
    ok, last = _run(pkg, torch.device("cuda:0"))
    assert ok and last["shard"] == (0, 30001)


def _worker(rank, world, port, result_path):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import __graft_entry__ as g
    pkg = g.load_package()
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    ok, last = _run(pkg, torch.device("cuda:0"))
    flags = torch.tensor([1 if ok else 0])
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    if rank == 0:
        with open(result_path, "w") as f:
            f.write("ok" if int(flags) == 1 else "mismatch")
    dist.destroy_process_group()


def test_sharded_locate_two_gloo_ranks(tmp_path):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tmp_path / "res.txt"
    mp.spawn(_worker, args=(2, port, str(out)), nprocs=2, join=True)
    assert out.read_text() == "ok"
