"""sview-fmindex_amd — MI355X-native batched FM-index count/locate.

Host-side mirror of baku4/sview-fmindex's public surface for its query hot
path, over the engine's C ABI (``include/fmx.h``, ``lib/libfmx.so``):

=============================  ===========================================================
this module                    reference (sview-fmindex/src/...)
=============================  ===========================================================
``FmIndex.load``               ``FmIndex::load``                 load_from_blob.rs:28-85
``FmIndex.count``              ``FmIndex::count``                locate/with_slice.rs:5-8
``FmIndex.locate``             ``FmIndex::locate``               locate/with_slice.rs:10-13
``FmIndex.locate_to_buffer``   ``FmIndex::locate_to_buffer``     locate/with_slice.rs:15-18
``FmIndex.*_rev_iter``         ``FmIndex::*_rev_iter``           locate/with_rev_iter.rs:5-19
``FmIndex.blob``               ``FmIndex::blob``                 reference_to_source_blob.rs:9-11
``FmIndex.count_batch`` /      (new) one kernel launch for a whole pattern batch
``FmIndex.locate_batch``
``FmIndexBuilder``             ``FmIndexBuilder``                builder/mod.rs:59-264 (built on the GPU)
``blocks.Block2..Block6``      ``blocks::Block2..Block6<V>``     components/bwm/blocks/
``text_encoders.*``            ``EncodingTable`` / ``PassThrough`` components/text_encoder/
``build_config.*``             ``LookupTableConfig`` / ``SuffixArrayConfig`` builder/build_config/
``LoadError`` / ``BuildError``  the reference's error enums       load_from_blob.rs:16-24, builder/mod.rs:37-57
=============================  ===========================================================

Generic parameters the reference carries in the type (``P``, ``B``, ``E``) are
passed as arguments here.  Every query runs the gfx950 kernels; there is no
CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _native as _n
from . import distributed  # noqa: F401  (multi-GPU helpers)

__all__ = ["FmIndex", "FmIndexBuilder", "Position", "u32", "u64", "Vector", "blocks",
           "text_encoders", "build_config", "LoadError", "BuildError", "FmxError",
           "aligned_buffer", "pack_patterns"]


# ------------------------------------------------------------------ errors

class FmxError(RuntimeError):
    """A failure of the engine that the reference would report as a panic or
    that has no reference counterpart (device errors)."""

    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{_n.status_str(code)} (fmx status {code}){': ' + what if what else ''}")


class LoadError(Exception):
    """``LoadError`` (load_from_blob.rs:16-24)."""


class InvalidFormat(LoadError):
    def __init__(self):
        super().__init__("Invalid FM-index format. The data does not appear to be a valid FM-index blob.")


class MismatchedBlobSize(LoadError):
    def __init__(self, expected: int, actual: int):
        self.expected, self.actual = expected, actual
        super().__init__(f"Mismatched blob size: headers indicate a total size of {expected} bytes, "
                         f"but the provided blob is {actual} bytes.")


LoadError.InvalidFormat = InvalidFormat
LoadError.MismatchedBlobSize = MismatchedBlobSize


class BuildError(Exception):
    """``BuildError`` (builder/mod.rs:37-57)."""


class SymbolCountOver(BuildError):
    def __init__(self, maximum: int, got: int):
        super().__init__(f"The symbol count ({got}) exceeds the maximum for the chosen block type ({maximum}).")


class UnmatchedTextLength(BuildError):
    def __init__(self, expected: int, got: int):
        super().__init__(f"Mismatched text length: expected {expected} bytes, but got {got} bytes.")


class InvalidBlobSize(BuildError):
    def __init__(self, expected: int, got: int):
        super().__init__(f"Incorrect blob size: expected {expected} bytes, but got {got} bytes.")


class NotAlignedBlob(BuildError):
    def __init__(self, required: int, offset: int):
        super().__init__(f"Improper blob alignment: required alignment is {required} bytes, "
                         f"but the blob has an offset of {offset} bytes.")


class InvalidConfig(BuildError):
    pass


for _c in (SymbolCountOver, UnmatchedTextLength, InvalidBlobSize, NotAlignedBlob, InvalidConfig):
    setattr(BuildError, _c.__name__, _c)


def _check(code: int, what: str = ""):
    if code != _n.FMX_OK:
        raise FmxError(code, what)


# ------------------------------------------------------------ type params

class Position:
    """``Position`` (text_length.rs:10-129): u32 or u64."""

    def __init__(self, nbytes: int):
        self.nbytes = nbytes
        self.dtype = np.dtype(np.uint32 if nbytes == 4 else np.uint64)

    def __repr__(self):
        return f"u{self.nbytes * 8}"


u32 = Position(4)
u64 = Position(8)


class Vector:
    """``Vector`` (blocks/vector.rs:11-79): u32 / u64 / u128."""

    def __init__(self, bits: int):
        self.bits = bits
        self.BLOCK_LEN = bits
        self.ALIGN_SIZE = 16 if bits == 128 else 8

    def __repr__(self):
        return f"u{self.bits}"


Vector.U32, Vector.U64, Vector.U128 = Vector(32), Vector(64), Vector(128)


class _Block:
    PLANES = 0

    def __init__(self, vector: Vector = Vector.U64):
        if isinstance(vector, int):
            vector = Vector(vector)
        self.vector = vector

    @property
    def planes(self):
        return self.PLANES

    @property
    def BLOCK_LEN(self):
        return self.vector.bits

    @property
    def MAX_SYMBOL(self):
        return 1 << self.PLANES

    @property
    def ALIGN_SIZE(self):
        return self.vector.ALIGN_SIZE

    def __repr__(self):
        return f"Block{self.PLANES}<{self.vector!r}>"


class blocks:
    """``blocks::Block2..Block6<V>`` (components/bwm/blocks/)."""

    class Block2(_Block):
        PLANES = 2

    class Block3(_Block):
        PLANES = 3

    class Block4(_Block):
        PLANES = 4

    class Block5(_Block):
        PLANES = 5

    class Block6(_Block):
        PLANES = 6


class text_encoders:
    """``text_encoders`` (components/text_encoder/text_encoders/)."""

    class EncodingTable:
        """``EncodingTable([u8; 256])`` (encoding_table.rs:7-39)."""
        ENCODER = _n.FMX_ENC_TABLE

        def __init__(self, table: bytes):
            if len(table) != 256:
                raise ValueError("EncodingTable needs 256 bytes")
            self.table = bytes(table)

        @classmethod
        def from_symbols(cls, symbols: Sequence[bytes]):
            """Last symbol is the wildcard (encoding_table.rs:15-26)."""
            count = len(symbols)
            t = bytearray([count - 1] * 256)
            for idx, sym in enumerate(symbols):
                for x in bytes(sym):
                    t[x] = idx
            return cls(bytes(t))

        @classmethod
        def from_symbols_with_wildcard(cls, symbols: Sequence[bytes]):
            """One extra wildcard symbol (encoding_table.rs:27-35)."""
            count = len(symbols) + 1
            t = bytearray([count - 1] * 256)
            for idx, sym in enumerate(symbols):
                for x in bytes(sym):
                    t[x] = idx
            return cls(bytes(t))

        def symbol_count(self) -> int:
            return max(self.table) + 1

        def idx_of(self, sym: int) -> int:
            return self.table[sym]

    class PassThrough:
        """``PassThrough`` (pass_through.rs:6-12): bytes are already symbol indices."""
        ENCODER = _n.FMX_ENC_PASS
        table = None

        def idx_of(self, sym: int) -> int:
            return sym


class build_config:
    """``build_config`` (builder/build_config/)."""

    class LookupTableConfig:
        def __init__(self, kind: str, value: int = 0):
            self.kind, self.value = kind, value

        @classmethod
        def None_(cls):
            return cls("None")

        @classmethod
        def KmerSize(cls, k: int):
            return cls("KmerSize", k)

        @classmethod
        def MaxMemory(cls, nbytes: int):
            return cls("MaxMemory", nbytes)

        def kmer_size(self, position: Position, symbol_count: int) -> int:
            """lookup_table_config.rs:22-51."""
            if self.kind == "None":
                return 1
            if self.kind == "KmerSize":
                if self.value < 2:
                    raise InvalidConfig("K-mer size must be at least 2")
                return self.value
            k = 2
            while (symbol_count + 1) ** k * position.nbytes <= self.value:
                k += 1
            return k - 1

    class SuffixArrayConfig:
        def __init__(self, kind: str, value: int = 1):
            self.kind, self.value = kind, value

        @classmethod
        def Uncompressed(cls):
            return cls("Uncompressed", 1)

        @classmethod
        def Compressed(cls, ratio: int):
            return cls("Compressed", ratio)

        def sampling_ratio(self) -> int:
            """suffix_array_config.rs:17-32."""
            if self.kind == "Uncompressed":
                return 1
            if self.value < 2:
                raise InvalidConfig("Sampling ratio for compressed suffix array must be at least 2")
            return self.value


build_config.LookupTableConfig.default = staticmethod(build_config.LookupTableConfig.None_)
build_config.SuffixArrayConfig.default = staticmethod(build_config.SuffixArrayConfig.Uncompressed)


# ----------------------------------------------------------------- helpers

def aligned_buffer(nbytes: int, align: int = 16) -> np.ndarray:
    """A zeroed uint8 host buffer whose data pointer is `align`-aligned."""
    raw = np.zeros(nbytes + align, dtype=np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


def pack_patterns(patterns: Iterable[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    """Ragged patterns -> (bytes uint8[total], offsets uint64[n+1])."""
    pats = [bytes(p) for p in patterns]
    lens = np.fromiter((len(p) for p in pats), dtype=np.uint64, count=len(pats))
    offsets = np.zeros(len(pats) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    data = np.frombuffer(b"".join(pats), dtype=np.uint8) if pats else np.zeros(0, np.uint8)
    return data, offsets


def _layout(position: Position, block: _Block, encoder) -> _n.fmx_layout:
    return _n.fmx_layout(position.nbytes, block.planes, block.vector.bits, encoder.ENCODER)


def _options(occ: str, deep_lut: bool, full_sa: bool = True, text: bool = True, context: bool = True,
             lut_rows: bool = True) -> int:
    mode = _n.FMX_OCC_INTERLEAVED if occ == "interleaved" else _n.FMX_OCC_BLOB
    return (mode | (_n.FMX_OPT_DEEP_LUT if deep_lut else 0) | (_n.FMX_OPT_FULL_SA if full_sa else 0)
            | (_n.FMX_OPT_TEXT if text else 0) | (_n.FMX_OPT_ROW_CONTEXT if context else 0)
            | (_n.FMX_OPT_LUT_ROWS if lut_rows else 0))


def _flags(reversed: bool, long_patterns: bool, stage_kb: int = 0, fixed_len: int = 0) -> int:
    """Query flags: FMX_PATTERN_REVERSED, FMX_HINT_LONG_PATTERNS,
    FMX_HINT_STAGE_KB(stage_kb) (LDS KB per 256-pattern tile; 0 = no hint) and
    FMX_HINT_FIXED_LEN(fixed_len) (every pattern fixed_len bytes, offsets[i] ==
    i * fixed_len; 0 = no hint)."""
    if not 0 <= int(fixed_len) <= 0xFFFF:
        raise ValueError("fixed_len must be in 0..65535")
    return ((_n.FMX_PATTERN_REVERSED if reversed else 0) | (_n.FMX_HINT_LONG_PATTERNS if long_patterns else 0)
            | ((int(stage_kb) & 0xFF) << 8) | (int(fixed_len) << 16))


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else C.c_void_p(a.ctypes.data)


# ----------------------------------------------------------------- FmIndex

class FmIndex:
    """``FmIndex<'a, P, B, E>`` (lib.rs:14-28), resident in HBM of one GPU."""

    def __init__(self, handle, position: Position, block: _Block, encoder, blob):
        self._h = handle
        self.position = position
        self.block = block
        self.text_encoder = encoder
        self._blob = blob  # keeps the borrowed host blob alive (fmx_blob)
        self._dt = position.dtype

    # -- load ---------------------------------------------------------
    @classmethod
    def load(cls, blob, position: Position = u32, block: Optional[_Block] = None,
             text_encoder=text_encoders.EncodingTable, device: int = 0,
             occ: str = "interleaved", deep_lut: bool = False, full_sa: bool = False, text: bool = False,
             context: bool = False, lut_rows: bool = False, options: Optional[int] = None) -> "FmIndex":
        """``FmIndex::load`` (load_from_blob.rs:28-85): validate, then copy the
        blob to HBM once.  By default the index is the reference's own: the
        blob, its occ planes and checkpoints re-laid out as one record per
        block (FMX_OPT_DEFAULT).  The flags add derived device structures
        (results are identical with any of them; they cost HBM — ~55x the
        blob at C2 with all of them — and load time; bench.py "derived"):
        `occ` — "blob" reads the blob's arrays as they are, "interleaved"
        re-lays checkpoint + planes into one HBM line per block; `deep_lut` —
        the device K-mer interval table (FMX_OPT_DEEP_LUT); `full_sa` — the
        full suffix array (FMX_OPT_FULL_SA); `text` — the recovered text for
        single-row tail verification (FMX_OPT_TEXT); `context` — row records
        {SA, preceding symbols} so that small intervals finish with one scan
        (FMX_OPT_ROW_CONTEXT); `lut_rows` — single-row deep-table entries
        that hold the row's location (FMX_OPT_LUT_ROWS).  `options` overrides all
        (FMX_OPT_DERIVED: every derived structure)."""
        block = block or blocks.Block2(Vector.U64)
        if isinstance(text_encoder, type):
            text_encoder = text_encoder.__new__(text_encoder)
        arr = blob if isinstance(blob, np.ndarray) else np.frombuffer(bytes(blob), dtype=np.uint8)
        if arr.ctypes.data % block.ALIGN_SIZE:
            a2 = aligned_buffer(arr.size, 16)
            a2[:] = arr
            arr = a2
        h = C.c_void_p()
        exp, act = C.c_uint64(), C.c_uint64()
        mode = options if options is not None else _options(occ, deep_lut, full_sa, text, context, lut_rows)
        st = _n.lib().fmx_load(_ptr(arr), arr.size, _layout(position, block, text_encoder), device, mode,
                               C.byref(h), C.byref(exp), C.byref(act))
        if st == _n.FMX_E_FORMAT:
            raise InvalidFormat()
        if st == _n.FMX_E_SIZE:
            raise MismatchedBlobSize(exp.value, act.value)
        _check(st, "fmx_load")
        if isinstance(text_encoder, text_encoders.EncodingTable) and not hasattr(text_encoder, "table"):
            text_encoder.table = bytes(arr[8 if block.ALIGN_SIZE == 8 else 16:][:256])
        return cls(h, position, block, text_encoder, arr)

    @classmethod
    def load_device(cls, d_blob: int, blob_len: int, position: Position = u32,
                    block: Optional[_Block] = None, text_encoder=text_encoders.EncodingTable,
                    device: int = 0, occ: str = "interleaved", deep_lut: bool = False, full_sa: bool = False,
                    text: bool = False, context: bool = False, lut_rows: bool = False,
                    options: Optional[int] = None) -> "FmIndex":
        """Load a blob already resident in HBM (borrowed, must outlive the index)."""
        block = block or blocks.Block2(Vector.U64)
        if isinstance(text_encoder, type):
            text_encoder = text_encoder.__new__(text_encoder)
        h = C.c_void_p()
        exp, act = C.c_uint64(), C.c_uint64()
        mode = options if options is not None else _options(occ, deep_lut, full_sa, text, context, lut_rows)
        st = _n.lib().fmx_load_device(C.c_void_p(d_blob), blob_len, _layout(position, block, text_encoder),
                                      device, mode, C.byref(h), C.byref(exp), C.byref(act))
        if st == _n.FMX_E_FORMAT:
            raise InvalidFormat()
        if st == _n.FMX_E_SIZE:
            raise MismatchedBlobSize(exp.value, act.value)
        _check(st, "fmx_load_device")
        return cls(h, position, block, text_encoder, None)

    @classmethod
    def load_file(cls, path, position: Position = u32, block: Optional[_Block] = None,
                  text_encoder=text_encoders.EncodingTable, device: int = 0, occ: str = "interleaved",
                  deep_lut: bool = False, full_sa: bool = False, text: bool = False, context: bool = False,
                  lut_rows: bool = False, options: Optional[int] = None, chunk_bytes: int = 0,
                  direct: bool = False) -> "FmIndex":
        """Blob file -> HBM (fmx_load_file): what the bench's mmap loader
        (bench/src/locate/sview_mmap.rs:17-45) followed by ``FmIndex::load``
        does, as a streamed ingest — the header is validated from the file,
        then the body is read in pinned chunks overlapped with their DMA.
        `direct`: the body is read with O_DIRECT (FMX_LOAD_DIRECT), bypassing
        the page cache — a cold load (raises if the file system refuses it)."""
        block = block or blocks.Block2(Vector.U64)
        if isinstance(text_encoder, type):
            text_encoder = text_encoder.__new__(text_encoder)
        h = C.c_void_p()
        exp, act = C.c_uint64(), C.c_uint64()
        mode = options if options is not None else _options(occ, deep_lut, full_sa, text, context, lut_rows)
        if direct:
            mode |= _n.FMX_LOAD_DIRECT
        st = _n.lib().fmx_load_file(os.fsencode(path), _layout(position, block, text_encoder), device, mode,
                                    int(chunk_bytes), C.byref(h), C.byref(exp), C.byref(act))
        if st == _n.FMX_E_FORMAT:
            raise InvalidFormat()
        if st == _n.FMX_E_SIZE:
            raise MismatchedBlobSize(exp.value, act.value)
        _check(st, f"fmx_load_file({path})")
        if isinstance(text_encoder, text_encoders.EncodingTable) and not hasattr(text_encoder, "table"):
            with open(path, "rb") as f:
                f.seek(8 if block.ALIGN_SIZE == 8 else 16)
                text_encoder.table = f.read(256)
        return cls(h, position, block, text_encoder, None)

    def close(self):
        if self._h:
            _n.lib().fmx_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    def blob(self) -> Optional[memoryview]:
        """``FmIndex::blob`` (reference_to_source_blob.rs:9-11)."""
        return None if self._blob is None else memoryview(self._blob)

    def info(self) -> dict:
        i = _n.fmx_index_info()
        _check(_n.lib().fmx_info(self._h, C.byref(i)))
        return {f: getattr(i, f) for f, _ in i._fields_}

    # -- single-pattern API (the reference's own) -----------------------
    def count(self, pattern: bytes) -> int:
        """``FmIndex::count`` (with_slice.rs:5-8)."""
        return int(self.count_batch([pattern])[0])

    def locate(self, pattern: bytes) -> List[int]:
        """``FmIndex::locate`` (with_slice.rs:10-13): suffix-array-row order."""
        _, locs = self.locate_batch([pattern])
        return [int(x) for x in locs]

    def locate_to_buffer(self, pattern: bytes, buffer: list) -> None:
        """``FmIndex::locate_to_buffer`` (with_slice.rs:15-18): appends."""
        buffer.extend(self.locate(pattern))

    def count_rev_iter(self, pattern_rev_iter: Iterable[int]) -> int:
        """``FmIndex::count_rev_iter`` (with_rev_iter.rs:5-9)."""
        rev = bytes(pattern_rev_iter)
        return int(self.count_batch([rev], reversed=True)[0])

    def locate_rev_iter(self, pattern_rev_iter: Iterable[int]) -> List[int]:
        """``FmIndex::locate_rev_iter`` (with_rev_iter.rs:10-14)."""
        rev = bytes(pattern_rev_iter)
        _, locs = self.locate_batch([rev], reversed=True)
        return [int(x) for x in locs]

    def locate_rev_iter_to_buffer(self, pattern_rev_iter: Iterable[int], buffer: list) -> None:
        buffer.extend(self.locate_rev_iter(pattern_rev_iter))

    # -- batched API -----------------------------------------------------
    def count_batch(self, patterns, reversed: bool = False) -> np.ndarray:
        """Counts of many patterns in one launch (P-typed numpy array)."""
        data, offsets = patterns if isinstance(patterns, tuple) else pack_patterns(patterns)
        n = offsets.size - 1
        out = np.zeros(max(n, 1), dtype=self._dt)
        flags = _n.FMX_PATTERN_REVERSED if reversed else 0
        _check(_n.lib().fmx_count_batch(self._h, _ptr(data) if data.size else None, _ptr(offsets), n,
                                        flags, _ptr(out)), "fmx_count_batch")
        return out[:n]

    def locate_batch(self, patterns, reversed: bool = False,
                     cap: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
        """Locations of many patterns: (offsets uint64[n+1], locations P[total]);
        pattern i's locations are locations[offsets[i]:offsets[i+1]] in
        suffix-array-row order."""
        data, offsets = patterns if isinstance(patterns, tuple) else pack_patterns(patterns)
        n = offsets.size - 1
        loc_off = np.zeros(n + 1, dtype=np.uint64)
        flags = _n.FMX_PATTERN_REVERSED if reversed else 0
        needed = C.c_uint64()
        if cap is None:
            # size the output from the counts (second call only if they do not fit)
            cap = 1 << 16
        locs = np.zeros(max(cap, 1), dtype=self._dt)
        st = _n.lib().fmx_locate_batch(self._h, _ptr(data) if data.size else None, _ptr(offsets), n, flags,
                                       _ptr(loc_off), _ptr(locs), cap, C.byref(needed))
        if st == _n.FMX_E_CAPACITY:
            cap = needed.value
            locs = np.zeros(max(cap, 1), dtype=self._dt)
            st = _n.lib().fmx_locate_batch(self._h, _ptr(data) if data.size else None, _ptr(offsets), n, flags,
                                           _ptr(loc_off), _ptr(locs), cap, C.byref(needed))
        _check(st, "fmx_locate_batch")
        return loc_off, locs[:needed.value]

    # -- device-resident API (pointers are ints; stream is a hipStream_t) --
    def count_batch_async(self, d_bytes: int, d_offsets: int, n: int, d_counts: int,
                          stream: int = 0, reversed: bool = False, long_patterns: bool = False, stage_kb: int = 0,
                          fixed_len: int = 0) -> None:
        flags = _flags(reversed, long_patterns, stage_kb, fixed_len)
        _check(_n.lib().fmx_count_batch_async(self._h, C.c_void_p(d_bytes), C.c_void_p(d_offsets), n, flags,
                                              C.c_void_p(d_counts), C.c_void_p(stream) if stream else None))

    def locate_workspace_size(self, n: int) -> int:
        b = C.c_uint64()
        _check(_n.lib().fmx_locate_workspace_size(self._h, n, C.byref(b)))
        return b.value

    def locate_batch_async(self, d_bytes: int, d_offsets: int, n: int, d_loc_offsets: int,
                           d_locs: int, cap: int, d_needed: int, d_ws: int, ws_bytes: int,
                           d_counts: int = 0, stream: int = 0, reversed: bool = False,
                           long_patterns: bool = False, stage_kb: int = 0, fixed_len: int = 0) -> None:
        """`long_patterns`: FMX_HINT_LONG_PATTERNS (patterns average > 64 bytes);
        `fixed_len`: FMX_HINT_FIXED_LEN (checked on the device: FMX_E_ARG at sync)."""
        flags = _flags(reversed, long_patterns, stage_kb, fixed_len)
        _check(_n.lib().fmx_locate_batch_async(
            self._h, C.c_void_p(d_bytes), C.c_void_p(d_offsets), n, flags,
            C.c_void_p(d_counts) if d_counts else None, C.c_void_p(d_loc_offsets), C.c_void_p(d_locs), cap,
            C.c_void_p(d_needed) if d_needed else None, C.c_void_p(d_ws), ws_bytes,
            C.c_void_p(stream) if stream else None))

    @staticmethod
    def locate_job(d_bytes: int, d_offsets: int, n: int, d_loc_offsets: int, d_locs: int, cap: int,
                   d_needed: int, d_ws: int, ws_bytes: int, d_counts: int = 0, stream: int = 0,
                   reversed: bool = False, long_patterns: bool = False, stage_kb: int = 0,
                   fixed_len: int = 0) -> "_n.fmx_locate_job":
        """One entry of a locate queue (fmx_locate_job): the arguments of
        locate_batch_async."""
        flags = _flags(reversed, long_patterns, stage_kb, fixed_len)
        return _n.fmx_locate_job(d_bytes, d_offsets, n, flags, 0, d_counts or None, d_loc_offsets, d_locs, cap,
                                 d_needed, d_ws, ws_bytes, stream or None)

    @staticmethod
    def job_queue(jobs) -> "C.Array":
        """A ctypes array of jobs, built once and submitted many times."""
        return (_n.fmx_locate_job * len(jobs))(*jobs)

    def locate_jobs_async(self, queue) -> None:
        """Issue a queue of locate batches in one native call
        (fmx_locate_jobs_async): no per-batch Python overhead."""
        _check(_n.lib().fmx_locate_jobs_async(self._h, queue, len(queue)))

    def locate_group_async(self, queue, stream: int = 0) -> None:
        """Run a queue of locate batches together, up to 256 per kernel launch,
        on `stream` (fmx_locate_group_async); distinct workspaces and outputs."""
        _check(_n.lib().fmx_locate_group_async(self._h, queue, len(queue), C.c_void_p(stream) if stream else None))

    def sync(self, stream: int = 0) -> None:
        _check(_n.lib().fmx_sync(self._h, C.c_void_p(stream) if stream else None))

    def release_stream(self, stream: int) -> None:
        """Done with `stream`: wait for it, raise what it latched (as sync),
        free its status word (fmx_stream_release)."""
        _check(_n.lib().fmx_stream_release(self._h, C.c_void_p(stream) if stream else None))

    def timing_enable(self, on: bool = True, every: int = 1) -> None:
        """Bracket every `every`-th launch with HIP events (fmx_timing_enable)."""
        _check(_n.lib().fmx_timing_enable(self._h, max(1, int(every)) if on else 0))

    def timing_read(self) -> dict:
        arr = (_n.fmx_kernel_timing * 16)()
        cnt = C.c_int()
        _check(_n.lib().fmx_timing_read(self._h, arr, 16, C.byref(cnt)))
        return {arr[i].name.decode(): {"launches": arr[i].launches, "total_ms": arr[i].total_ms,
                                       "units": arr[i].units} for i in range(min(cnt.value, 16))}


# ------------------------------------------------------- MultiDeviceIndex

class MultiDeviceIndex:
    """One index over several GPUs of this process (fmx_multi_*): a replica
    per entry of `devices` (the blob copied host -> devices[0] once, then
    device to device), batches cut into contiguous shards answered
    concurrently and concatenated — the same answers as `FmIndex` on one
    device, for a single-process caller with no process group."""

    def __init__(self, blob, devices: Sequence[int], position: Position = u32, block: Optional[_Block] = None,
                 text_encoder=text_encoders.EncodingTable, options: int = _n.FMX_OPT_DEFAULT):
        block = block or blocks.Block2(Vector.U64)
        if isinstance(text_encoder, type):
            text_encoder = text_encoder.__new__(text_encoder)
        arr = blob if isinstance(blob, np.ndarray) else np.frombuffer(bytes(blob), dtype=np.uint8)
        if arr.ctypes.data % block.ALIGN_SIZE:
            a2 = aligned_buffer(arr.size, 16)
            a2[:] = arr
            arr = a2
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        exp, act = C.c_uint64(), C.c_uint64()
        st = _n.lib().fmx_multi_load(_ptr(arr), arr.size, _layout(position, block, text_encoder), devs, len(devices),
                                     options, C.byref(h), C.byref(exp), C.byref(act))
        if st == _n.FMX_E_FORMAT:
            raise InvalidFormat()
        if st == _n.FMX_E_SIZE:
            raise MismatchedBlobSize(exp.value, act.value)
        _check(st, "fmx_multi_load")
        self._h = h
        self._dt = position.dtype
        self.devices = list(devices)

    @property
    def replicas(self) -> int:
        return _n.lib().fmx_multi_replicas(self._h)

    def close(self):
        if self._h:
            _n.lib().fmx_multi_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def count_batch(self, patterns, reversed: bool = False) -> np.ndarray:
        data, offsets = patterns if isinstance(patterns, tuple) else pack_patterns(patterns)
        n = offsets.size - 1
        out = np.zeros(max(n, 1), dtype=self._dt)
        flags = _n.FMX_PATTERN_REVERSED if reversed else 0
        _check(_n.lib().fmx_multi_count_batch(self._h, _ptr(data) if data.size else None, _ptr(offsets), n, flags,
                                              _ptr(out)), "fmx_multi_count_batch")
        return out[:n]

    def locate_batch(self, patterns, reversed: bool = False,
                     cap: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
        data, offsets = patterns if isinstance(patterns, tuple) else pack_patterns(patterns)
        n = offsets.size - 1
        loc_off = np.zeros(n + 1, dtype=np.uint64)
        flags = _n.FMX_PATTERN_REVERSED if reversed else 0
        needed = C.c_uint64()
        cap = (1 << 16) if cap is None else cap
        locs = np.zeros(max(cap, 1), dtype=self._dt)
        args = lambda: (self._h, _ptr(data) if data.size else None, _ptr(offsets), n, flags, _ptr(loc_off),  # noqa
                        _ptr(locs), cap, C.byref(needed))
        st = _n.lib().fmx_multi_locate_batch(*args())
        if st == _n.FMX_E_CAPACITY:
            cap = needed.value
            locs = np.zeros(max(cap, 1), dtype=self._dt)
            st = _n.lib().fmx_multi_locate_batch(*args())
        _check(st, "fmx_multi_locate_batch")
        return loc_off, locs[:needed.value]


# ---------------------------------------------------------- FmIndexBuilder

class FmIndexBuilder:
    """``FmIndexBuilder<P, B, E>`` (builder/mod.rs:17-264); ``build`` runs on the GPU."""

    def __init__(self, text_len: int, symbol_count: int, text_encoder, position: Position = u32,
                 block: Optional[_Block] = None, lookup_table_config=None, suffix_array_config=None):
        self.block = block or blocks.Block2(Vector.U64)
        if symbol_count > self.block.MAX_SYMBOL:
            raise SymbolCountOver(self.block.MAX_SYMBOL, symbol_count)
        self.text_len = text_len
        self.symbol_count = symbol_count
        self.text_encoder = text_encoder
        self.position = position
        self.lookup_table_config = lookup_table_config or build_config.LookupTableConfig.None_()
        self.suffix_array_config = suffix_array_config or build_config.SuffixArrayConfig.Uncompressed()
        self.kmer_size = self.lookup_table_config.kmer_size(position, symbol_count)
        self.sampling_ratio = self.suffix_array_config.sampling_ratio()

    @classmethod
    def new(cls, text_len, symbol_count, text_encoder, position=u32, block=None):
        return cls(text_len, symbol_count, text_encoder, position, block)

    def set_lookup_table_config(self, config) -> "FmIndexBuilder":
        return FmIndexBuilder(self.text_len, self.symbol_count, self.text_encoder, self.position, self.block,
                              config, self.suffix_array_config)

    def set_suffix_array_config(self, config) -> "FmIndexBuilder":
        return FmIndexBuilder(self.text_len, self.symbol_count, self.text_encoder, self.position, self.block,
                              self.lookup_table_config, config)

    def _layout(self):
        return _layout(self.position, self.block, self.text_encoder)

    def blob_size(self) -> int:
        out = C.c_uint64()
        st = _n.lib().fmx_build_blob_size(self.text_len, self.symbol_count, self._layout(), self.kmer_size,
                                          self.sampling_ratio, C.byref(out))
        if st == _n.FMX_E_CONFIG:
            raise InvalidConfig("unsupported configuration")
        _check(st)
        return out.value

    def build(self, text, blob: np.ndarray, device: int = 0) -> None:
        """``FmIndexBuilder::build`` (builder/mod.rs:187-264) on `device`."""
        t = np.frombuffer(bytes(text), dtype=np.uint8) if not isinstance(text, np.ndarray) else text
        if t.size != self.text_len:
            raise UnmatchedTextLength(self.text_len, t.size)
        if blob.ctypes.data % self.block.ALIGN_SIZE:
            raise NotAlignedBlob(self.block.ALIGN_SIZE, blob.ctypes.data % self.block.ALIGN_SIZE)
        size = self.blob_size()
        if blob.size != size:
            raise InvalidBlobSize(size, blob.size)
        table = self.text_encoder.table
        tb = None if table is None else C.create_string_buffer(table, 256)
        st = _n.lib().fmx_build(_ptr(t) if t.size else None, t.size, tb, self.symbol_count, self._layout(),
                                self.kmer_size, self.sampling_ratio, _ptr(blob), blob.size, device)
        if st == _n.FMX_E_SYMBOL:
            raise FmxError(st, "text symbol index >= symbol_count")
        _check(st, "fmx_build")

    def build_device(self, d_text: int, d_blob: int, blob_len: int, device: int = 0) -> None:
        """Build from a text already in HBM into a device blob."""
        table = self.text_encoder.table
        tb = None if table is None else C.create_string_buffer(table, 256)
        _check(_n.lib().fmx_build_device(C.c_void_p(d_text), self.text_len, tb, self.symbol_count,
                                         self._layout(), self.kmer_size, self.sampling_ratio,
                                         C.c_void_p(d_blob), blob_len, device), "fmx_build_device")
