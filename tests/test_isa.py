"""The fused launch's hand-off as the compiler emitted it (ADVICE r5 low:
its correctness across the XCDs' L2s rests on the codegen, so the shipped
code object is checked, not the source).  From sview-fmindex_amd/lib/
libfmx.so's gfx950 code objects (the clang offload bundles in .hip_fatbin),
k_locate<u32, Block3<u64>, 64-B symbol-mask records> (C2's fused kernel) and
k_emit_chain are disassembled and must show, per MI355X_MICROARCH.md's
hand-off table, first row:
  * publish: the tile count stored write-through (global_store_dwordx2 sc1),
    then s_waitcnt vmcnt(0), then the tag stored write-through — in that
    order, with no other store between;
  * poll: the tag loaded with sc1 (past the CU's L1) in a loop with s_sleep,
    and the counts loaded with sc1;
  * the ticket: a returning global_atomic_add (take_ticket), and the
    counter's reset a write-through global_store_dword sc1 (claim_tile).
CPU only: needs llvm-objdump from /opt/rocm and the built library."""
import os
import re
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "sview-fmindex_amd", "lib", "libfmx.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
KERNELS = {
    "k_locate": "_ZN3fmx8k_locateIjLi3ELi64ELi66ELi0EEEvNS_9QueryArgsENS_11LocateGroupEjmm",
    "k_emit_chain": "_ZN3fmx12k_emit_chainIjLi3ELi64ELi66EEEvNS_9QueryArgsENS_11LocateGroupEmm",
}


def gfx950_objects(fatbin: bytes):
    """Every gfx950 code object in a .hip_fatbin section (bundle format: magic,
    u64 entry count, then per entry u64 offset, u64 size, u64 triple length,
    triple; offsets relative to the bundle)."""
    for m in re.finditer(re.escape(MAGIC), fatbin):
        b = m.start()
        p = b + len(MAGIC)
        (n,) = struct.unpack_from("<Q", fatbin, p)
        p += 8
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", fatbin, p)
            p += 24
            triple = fatbin[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and size:
                yield fatbin[b + off:b + off + size]


@pytest.fixture(scope="module")
def disasm(tmp_path_factory):
    if not (os.path.exists(LIB) and os.path.exists(os.path.join(LLVM, "llvm-objdump"))):
        pytest.skip("needs the built library and /opt/rocm's llvm-objdump")
    d = tmp_path_factory.mktemp("isa")
    fb = d / "fatbin.bin"
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", LIB, str(d / "x.so")],
                   check=True, capture_output=True)
    out = {}
    for i, co in enumerate(gfx950_objects(fb.read_bytes())):
        f = d / f"co{i}.o"
        f.write_bytes(co)
        for name, sym in KERNELS.items():
            if name in out:
                continue
            r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", f"--disassemble-symbols={sym}", str(f)],
                               capture_output=True, text=True)
            ins = [ln.split("//")[0].strip() for ln in r.stdout.splitlines() if ln.startswith("\t") or
                   ln.startswith(" ")]
            ins = [x for x in ins if x]
            if len(ins) > 50:
                out[name] = ins
    missing = set(KERNELS) - set(out)
    assert not missing, f"kernels not found in {LIB}: {missing}"
    return out


def publish_sequences(ins):
    """Indices i where an sc1 8-B store is followed by s_waitcnt vmcnt(0) and
    then another sc1 8-B store, with no other memory store in between."""
    hits = []
    for i, x in enumerate(ins):
        if not (x.startswith("global_store_dwordx2") and x.endswith("sc1")):
            continue
        j = i + 1
        waited = False
        while j < len(ins) and j < i + 12:
            y = ins[j]
            if y.startswith("s_waitcnt") and "vmcnt(0)" in y:
                waited = True
            elif y.startswith("global_store") or y.startswith("global_atomic") or y.startswith("buffer_store"):
                if waited and y.startswith("global_store_dwordx2") and y.endswith("sc1"):
                    hits.append(i)
                break
            j += 1
    return hits


@pytest.mark.parametrize("name", sorted(KERNELS))
def test_handoff_codegen(disasm, name):
    ins = disasm[name]
    assert publish_sequences(ins), f"{name}: no count store sc1 -> vmcnt(0) -> tag store sc1 sequence"
    polls = [i for i, x in enumerate(ins) if x.startswith("global_load_dwordx2") and x.endswith("sc1")]
    assert len(polls) >= 2, f"{name}: tag poll / count loads not sc1"
    sleeps = [i for i, x in enumerate(ins) if x.startswith("s_sleep")]
    assert sleeps and any(abs(s - p) < 8 for s in sleeps for p in polls), f"{name}: no s_sleep beside the poll"
    # no plain (L1-served) 8-B load anywhere near the poll loop: every load of a handed-off word is sc1
    lo, hi = min(polls), max(polls)
    plain = [x for x in ins[lo:hi + 1] if x.startswith("global_load_dwordx2") and not x.endswith("sc1")]
    assert not plain, f"{name}: plain 8-B loads inside the poll loop: {plain}"


@pytest.mark.parametrize("name", sorted(KERNELS))
def test_ticket_codegen(disasm, name):
    ins = disasm[name]
    # a returning atomic add (the ticket; GLC/sc0 = return the old value)
    adds = [x for x in ins if x.startswith("global_atomic_add ") and "sc0" in x]
    assert adds, f"{name}: no returning global_atomic_add (take_ticket)"
    resets = [x for x in ins if x.startswith("global_store_dword ") and x.endswith("sc1")]
    assert resets, f"{name}: no write-through reset of the ticket counter (claim_tile)"
