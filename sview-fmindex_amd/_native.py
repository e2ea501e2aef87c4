"""ctypes binding of the engine's C ABI (``include/fmx.h``) in ``lib/libfmx.so``.

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C sview-fmindex_amd/csrc``).  There is no fallback: if the library is
missing, importing this module raises, and every query runs the gfx950 kernels.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libfmx.so")

FMX_OK = 0
FMX_E_FORMAT = 1
FMX_E_SIZE = 2
FMX_E_ALIGN = 3
FMX_E_LAYOUT = 4
FMX_E_EMPTY_PATTERN = 5
FMX_E_SYMBOL = 6
FMX_E_CAPACITY = 7
FMX_E_DEVICE = 8
FMX_E_ARG = 9
FMX_E_CONFIG = 10

FMX_ENC_TABLE = 0
FMX_ENC_PASS = 1
FMX_PATTERN_REVERSED = 1
FMX_HINT_LONG_PATTERNS = 2
FMX_OCC_BLOB = 0
FMX_OCC_INTERLEAVED = 1
FMX_OPT_DEEP_LUT = 2
FMX_OPT_FULL_SA = 4
FMX_OPT_TEXT = 8
FMX_OPT_ROW_CONTEXT = 16
FMX_OPT_LUT_ROWS = 32
FMX_OPT_DEFAULT = FMX_OCC_INTERLEAVED
FMX_OPT_DERIVED = (FMX_OCC_INTERLEAVED | FMX_OPT_DEEP_LUT | FMX_OPT_FULL_SA | FMX_OPT_TEXT | FMX_OPT_ROW_CONTEXT
                   | FMX_OPT_LUT_ROWS)
FMX_LOAD_DIRECT = 1 << 16


class fmx_layout(C.Structure):
    _fields_ = [("pos_bytes", C.c_uint32), ("planes", C.c_uint32),
                ("vec_bits", C.c_uint32), ("encoder", C.c_uint32)]


class fmx_index_info(C.Structure):
    _fields_ = [("text_len", C.c_uint64), ("sentinel_index", C.c_uint64),
                ("blob_len", C.c_uint64), ("device_bytes", C.c_uint64),
                ("symbol_count", C.c_uint32), ("kmer_size", C.c_uint32),
                ("sampling_ratio", C.c_uint32), ("block_len", C.c_uint32),
                ("options", C.c_uint32), ("deep_lut_k", C.c_uint32), ("device", C.c_int32),
                ("context_len", C.c_uint32), ("scan_rows", C.c_uint32),
                ("occ_record", C.c_uint32), ("group_key_len", C.c_uint32),
                ("group_key_base", C.c_uint32), ("grouped_min", C.c_uint64),
                ("launches_grouped", C.c_uint64), ("launches_grouped_raw", C.c_uint64),
                ("launches_ordered", C.c_uint64), ("launches_fused", C.c_uint64),
                ("launches_chained", C.c_uint64)]


class fmx_locate_job(C.Structure):
    _fields_ = [("d_bytes", C.c_void_p), ("d_offsets", C.c_void_p), ("n_patterns", C.c_uint64),
                ("flags", C.c_uint32), ("reserved", C.c_uint32), ("d_counts", C.c_void_p),
                ("d_loc_offsets", C.c_void_p), ("d_locs", C.c_void_p), ("cap", C.c_uint64),
                ("d_needed", C.c_void_p), ("d_workspace", C.c_void_p), ("workspace_bytes", C.c_uint64),
                ("stream", C.c_void_p)]


class fmx_kernel_timing(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_uint64),
                ("total_ms", C.c_double), ("units", C.c_uint64)]


_u64, _u32, _p, _i = C.c_uint64, C.c_uint32, C.c_void_p, C.c_int
_PU64 = C.POINTER(C.c_uint64)

# name -> (restype, argtypes); every function declared in include/fmx.h
SIGNATURES = {
    "fmx_abi_version": (_u32, []),
    "fmx_status_str": (C.c_char_p, [_i]),
    "fmx_device_count": (_i, []),
    "fmx_load": (_i, [_p, _u64, fmx_layout, _i, _u32, C.POINTER(_p), _PU64, _PU64]),
    "fmx_load_device": (_i, [_p, _u64, fmx_layout, _i, _u32, C.POINTER(_p), _PU64, _PU64]),
    "fmx_load_file": (_i, [C.c_char_p, fmx_layout, _i, _u32, _u64, C.POINTER(_p), _PU64, _PU64]),
    "fmx_free": (None, [_p]),
    "fmx_blob": (_p, [_p, _PU64]),
    "fmx_info": (_i, [_p, C.POINTER(fmx_index_info)]),
    "fmx_count_batch": (_i, [_p, _p, _p, _u64, _u32, _p]),
    "fmx_locate_batch": (_i, [_p, _p, _p, _u64, _u32, _p, _p, _u64, _PU64]),
    "fmx_count_batch_async": (_i, [_p, _p, _p, _u64, _u32, _p, _p]),
    "fmx_locate_workspace_size": (_i, [_p, _u64, _PU64]),
    "fmx_workspace_bytes": (_i, [_u64, _u32, _PU64]),
    "fmx_locate_batch_async": (_i, [_p, _p, _p, _u64, _u32, _p, _p, _p, _u64, _p, _p, _u64, _p]),
    "fmx_locate_jobs_async": (_i, [_p, C.POINTER(fmx_locate_job), _u64]),
    "fmx_locate_group_async": (_i, [_p, C.POINTER(fmx_locate_job), _u64, _p]),
    "fmx_sync": (_i, [_p, _p]),
    "fmx_stream_release": (_i, [_p, _p]),
    "fmx_multi_load": (_i, [_p, _u64, fmx_layout, C.POINTER(_i), _i, _u32, C.POINTER(_p), _PU64, _PU64]),
    "fmx_multi_free": (None, [_p]),
    "fmx_multi_replicas": (_i, [_p]),
    "fmx_multi_replica": (_p, [_p, _i]),
    "fmx_multi_count_batch": (_i, [_p, _p, _p, _u64, _u32, _p]),
    "fmx_multi_locate_batch": (_i, [_p, _p, _p, _u64, _u32, _p, _p, _u64, _PU64]),
    "fmx_timing_enable": (_i, [_p, _i]),
    "fmx_timing_read": (_i, [_p, C.POINTER(fmx_kernel_timing), _i, C.POINTER(_i)]),
    "fmx_build_blob_size": (_i, [_u64, _u32, fmx_layout, _u32, _u32, _PU64]),
    "fmx_build_device": (_i, [_p, _u64, _p, _u32, fmx_layout, _u32, _u32, _p, _u64, _i]),
    "fmx_build": (_i, [_p, _u64, _p, _u32, fmx_layout, _u32, _u32, _p, _u64, _i]),
}

_lib = None


def lib():
    """Load libfmx.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build the HIP engine first "
                "(python -c 'import __graft_entry__ as g; g.build()')")
        # One HIP runtime per process: when torch is installed, load its HIP
        # runtime first (SONAME libamdhip64.so.7, as the system one), so that
        # libfmx.so's DT_NEEDED binds to it and torch tensors / RCCL / our kernels
        # share one device context.  Loaded the other way round, two HSA runtimes
        # would compete for the device.
        if os.environ.get("FMX_NO_TORCH_RUNTIME") != "1":
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        L = C.CDLL(os.environ.get("FMX_LIB", LIB_PATH))  # FMX_LIB: another build of the engine
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def status_str(code: int) -> str:
    return lib().fmx_status_str(code).decode()
