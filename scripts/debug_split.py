"""Diagnostic: split vs fused locate on the smoke workload; prints the first differences."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g
from oracle import oracle as O
pkg = g.load_package()
rng = np.random.default_rng(7)
table = pkg.text_encoders.EncodingTable.from_symbols([b"Aa", b"Cc", b"Gg", b"Tt", b"Nn"])
text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=20000).astype(np.uint8)
block = pkg.blocks.Block3(pkg.Vector.U64)
builder = (pkg.FmIndexBuilder(text.size, 5, table, pkg.u32, block)
           .set_lookup_table_config(pkg.build_config.LookupTableConfig.KmerSize(3))
           .set_suffix_array_config(pkg.build_config.SuffixArrayConfig.Compressed(2)))
blob = pkg.aligned_buffer(builder.blob_size())
builder.build(text, blob)
starts = rng.integers(0, text.size - 20, size=512)
pats = [text[s:s + int(rng.integers(1, 21))].tobytes() for s in starts]
orc = O.OracleIndex(blob, O.layout(4, 3, 64, 0))
data, offsets = pkg.pack_patterns(pats)
ooff, olocs = orc.locate_batch(data, offsets)
for opt in (0, 1, 4, 4 | 8, 16, 2 | 8 | 32, 63):
    ix = pkg.FmIndex.load(blob, pkg.u32, block, table, device=0, options=opt)
    off, locs = ix.locate_batch(pats)
    cnt = ix.count_batch(pats)
    print("options", opt, "offsets equal", np.array_equal(off, ooff), "locs equal", np.array_equal(locs, olocs),
          "counts equal", np.array_equal(cnt, np.diff(ooff).astype(cnt.dtype)), "total", off[-1], ooff[-1])
    d = np.nonzero(off != ooff)[0]
    if d.size:
        print("  first offset diffs at", d[:10], off[d[:10]], ooff[d[:10]])
    if locs.size == olocs.size:
        d = np.nonzero(locs != olocs)[0]
        if d.size:
            print("  first loc diffs at", d[:10], locs[d[:10]], olocs[d[:10]])
            owner = np.searchsorted(ooff, d[:10], side="right") - 1
            for t, o in zip(d[:6], owner[:6]):
                sl = slice(int(ooff[o]), int(ooff[o + 1]))
                print("   slot", t, "pattern", o, "len", len(pats[o]), "count", int(ooff[o + 1] - ooff[o]),
                      "gpu", list(locs[sl])[:8], "orc", list(olocs[sl])[:8])
    ix.close()

# records of the split path, via the async API on torch buffers
import torch
dev = torch.device("cuda:0")
ix = pkg.FmIndex.load(blob, pkg.u32, block, table, device=0, options=16)
n = len(pats)
d_data = torch.from_numpy(data.copy()).to(dev)
d_off = torch.from_numpy(offsets.view(np.int64).copy()).to(dev)
d_loff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
cap = int(ooff[-1]) + 16
d_locs = torch.zeros(cap, dtype=torch.int32, device=dev)
d_need = torch.zeros(1, dtype=torch.int64, device=dev)
ws = ix.locate_workspace_size(n)
d_ws = torch.zeros(ws, dtype=torch.uint8, device=dev)
ix.locate_batch_async(d_data.data_ptr(), d_off.data_ptr(), n, d_loff.data_ptr(), d_locs.data_ptr(), cap,
                      d_need.data_ptr(), d_ws.data_ptr(), ws)
ix.sync()
torch.cuda.synchronize()
w = d_ws.cpu().numpy()
T = (n + 255) // 256
rec = w[256 + 16 * T: 256 + 16 * T + 16 * n].view(np.uint32).reshape(n, 4)
print("ws", ws, "tiles", T, "tile_cnt", w[256:256 + 8 * T].view(np.uint64), "tile_off", w[256 + 8 * T:256 + 16 * T].view(np.uint64))
for o in (0, 7):
    print("pattern", o, "rec a,b,x_lo,x_hi", rec[o], "orc", list(olocs[int(ooff[o]):int(ooff[o + 1])]),
          "gpu", list(d_locs.cpu().numpy()[int(ooff[o]):int(ooff[o + 1])]))
