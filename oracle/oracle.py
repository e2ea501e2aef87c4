"""ORACLE — test infrastructure only.

ctypes binding of ``oracle/liboracle.so`` (the plain-C restatement of
baku4/sview-fmindex in ``oracle/fmx_oracle.c``).  Imported only by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg — as the
checker / CPU baseline, never as the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

ORC_OK = 0
ERRORS = {1: "InvalidFormat", 2: "MismatchedBlobSize", 3: "NotAligned", 4: "Layout",
          5: "EmptyPattern", 6: "Symbol", 7: "Capacity", 10: "Config"}


class OracleError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__(f"oracle error {code} ({ERRORS.get(code, '?')}) {msg}")
        self.code = code


class Layout(C.Structure):
    _fields_ = [("pos_bytes", C.c_uint32), ("planes", C.c_uint32),
                ("vec_bits", C.c_uint32), ("encoder", C.c_uint32)]


class Index(C.Structure):
    _fields_ = [("L", Layout), ("blob", C.c_void_p), ("blob_len", C.c_uint64),
                ("enc", C.c_uint8 * 256), ("sigma", C.c_uint32), ("k", C.c_uint32),
                ("sr", C.c_uint32), ("bl", C.c_uint32), ("align", C.c_uint32),
                ("block_bytes", C.c_uint32), ("n", C.c_uint64),
                ("count_array", C.c_uint64 * 65), ("mult", C.c_uint64 * 64),
                ("kmer_table", C.c_void_p), ("kmer_len", C.c_uint64),
                ("sa", C.c_void_p), ("sa_len", C.c_uint64), ("sentinel", C.c_uint64),
                ("ckpt", C.c_void_p), ("ckpt_len", C.c_uint64),
                ("blocks", C.c_void_p), ("blocks_len", C.c_uint64),
                ("off_count_array", C.c_uint64), ("off_mult", C.c_uint64),
                ("off_kmer", C.c_uint64), ("off_sa", C.c_uint64),
                ("off_sentinel", C.c_uint64), ("off_ckpt", C.c_uint64),
                ("off_blocks", C.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = C.CDLL(_LIB_PATH)
        u64, p = C.c_uint64, C.c_void_p
        L.orc_load.argtypes = [p, u64, Layout, C.POINTER(Index), C.POINTER(u64), C.POINTER(u64)]
        L.orc_count.argtypes = [C.POINTER(Index), p, u64, C.POINTER(u64)]
        L.orc_count_rev.argtypes = [C.POINTER(Index), p, u64, C.POINTER(u64)]
        L.orc_locate.argtypes = [C.POINTER(Index), p, u64, p, u64, C.POINTER(u64)]
        L.orc_count_batch.argtypes = [C.POINTER(Index), p, p, u64, p, C.c_int]
        L.orc_locate_batch.argtypes = [C.POINTER(Index), p, p, u64, p, p, u64, C.POINTER(u64), C.c_int]
        L.orc_blob_size.argtypes = [u64, C.c_uint32, Layout, C.c_uint32, C.c_uint32, C.POINTER(u64)]
        L.orc_build.argtypes = [p, u64, p, C.c_uint32, Layout, C.c_uint32, C.c_uint32, p, u64]
        L.orc_suffix_array.argtypes = [p, u64, C.c_uint32, p]
        for f in ("orc_load", "orc_count", "orc_count_rev", "orc_locate", "orc_count_batch",
                  "orc_locate_batch", "orc_blob_size", "orc_build", "orc_suffix_array"):
            getattr(L, f).restype = C.c_int
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data if a is not None and a.size else None


def aligned_zeros(nbytes, align=16):
    """A uint8 array whose data pointer is `align`-aligned (the blob must be)."""
    raw = np.zeros(nbytes + align, dtype=np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


def layout(pos_bytes=4, planes=2, vec_bits=64, encoder=0):
    return Layout(pos_bytes, planes, vec_bits, encoder)


def blob_size(n, sigma, L, k=1, sr=1):
    out = C.c_uint64()
    st = lib().orc_blob_size(n, sigma, L, k, sr, C.byref(out))
    if st:
        raise OracleError(st)
    return out.value


def build(text, sigma, L, k=1, sr=1, table=None):
    """FmIndexBuilder::build restated (builder/mod.rs:187-264).  `table` is the
    256-byte EncodingTable (None = PassThrough)."""
    text = np.frombuffer(bytes(text), dtype=np.uint8) if not isinstance(text, np.ndarray) else text
    enc = 0 if table is not None else 1
    L = Layout(L.pos_bytes, L.planes, L.vec_bits, enc)
    size = blob_size(len(text), sigma, L, k, sr)
    blob = aligned_zeros(size, 16)
    tab = np.frombuffer(bytes(table), dtype=np.uint8) if table is not None else None
    st = lib().orc_build(_ptr(text), len(text), _ptr(tab), sigma, L, k, sr, _ptr(blob), size)
    if st:
        raise OracleError(st)
    return blob


class OracleIndex:
    """FmIndex::load + count/locate restated on the CPU."""

    def __init__(self, blob, L):
        if not isinstance(blob, np.ndarray):
            b = aligned_zeros(len(blob), 16)
            b[:] = np.frombuffer(bytes(blob), dtype=np.uint8)
            blob = b
        self.blob = blob
        self.ix = Index()
        self.expected = C.c_uint64()
        self.actual = C.c_uint64()
        st = lib().orc_load(_ptr(blob), blob.size, L, C.byref(self.ix),
                            C.byref(self.expected), C.byref(self.actual))
        if st:
            raise OracleError(st, f"expected={self.expected.value} actual={self.actual.value}")
        self.L = L
        self.pdt = np.uint32 if L.pos_bytes == 4 else np.uint64

    @property
    def text_len(self):
        return self.ix.n

    def count(self, pattern: bytes) -> int:
        out = C.c_uint64()
        buf = C.create_string_buffer(bytes(pattern), len(pattern) + 1)
        st = lib().orc_count(C.byref(self.ix), buf, len(pattern), C.byref(out))
        if st:
            raise OracleError(st)
        return out.value

    def count_rev(self, rev_pattern: bytes) -> int:
        out = C.c_uint64()
        buf = C.create_string_buffer(bytes(rev_pattern), len(rev_pattern) + 1)
        st = lib().orc_count_rev(C.byref(self.ix), buf, len(rev_pattern), C.byref(out))
        if st:
            raise OracleError(st)
        return out.value

    def locate(self, pattern: bytes):
        """Locations in suffix-array-row order (unsorted, as the reference)."""
        cnt = self.count(pattern)
        out = np.zeros(max(cnt, 1), dtype=np.uint64)
        got = C.c_uint64()
        buf = C.create_string_buffer(bytes(pattern), len(pattern) + 1)
        st = lib().orc_locate(C.byref(self.ix), buf, len(pattern), _ptr(out), cnt, C.byref(got))
        if st:
            raise OracleError(st)
        return [int(x) for x in out[:cnt]]

    def count_batch(self, data: np.ndarray, offsets: np.ndarray, threads=1):
        n = offsets.size - 1
        out = np.zeros(max(n, 1), dtype=self.pdt)
        st = lib().orc_count_batch(C.byref(self.ix), _ptr(data), _ptr(offsets), n, _ptr(out), threads)
        if st:
            raise OracleError(st)
        return out[:n]

    def locate_batch(self, data: np.ndarray, offsets: np.ndarray, threads=1, cap=None):
        n = offsets.size - 1
        loc_off = np.zeros(n + 1, dtype=np.uint64)
        needed = C.c_uint64()
        if cap is None:
            cap = int(self.count_batch(data, offsets, threads).astype(np.uint64).sum())
        locs = np.zeros(max(cap, 1), dtype=self.pdt)
        st = lib().orc_locate_batch(C.byref(self.ix), _ptr(data), _ptr(offsets), n, _ptr(loc_off),
                                    _ptr(locs), cap, C.byref(needed), threads)
        if st:
            raise OracleError(st, f"needed={needed.value}")
        return loc_off, locs[:needed.value]


def suffix_array(t: np.ndarray, alphabet: int) -> np.ndarray:
    sa = np.zeros(max(t.size, 1), dtype=np.uint64)
    lib().orc_suffix_array(_ptr(t), t.size, alphabet, _ptr(sa))
    return sa[:t.size]
