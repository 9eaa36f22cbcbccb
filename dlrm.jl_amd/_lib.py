"""ctypes binding of libdlrm_hip.so — the C ABI declared in include/dlrm_hip.h.

This is the Python equivalent of the Julia `ccall` shim in INTEGRATION.md: plain pointers,
sizes and status codes; torch only supplies device memory and the stream.  The library is
REQUIRED: if it is missing the import fails loudly (there is no CPU fallback).
"""
import ctypes
import os
import re
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("DLRM_HIP_LIB") or os.path.join(_HERE, "lib", "libdlrm_hip.so")  # override: A/B runs
HEADER = os.path.join(REPO, "include", "dlrm_hip.h")

# dlrm_status
OK, E_ARG, E_HIP, E_INDEX, E_UNSUPPORTED, E_NOMEM, E_STATE = 0, -1, -2, -3, -4, -5, -6
# dlrm_dtype / dlrm_itype
F32, BF16 = 0, 1
I32, I64 = 0, 1
UPDATE_ATOMIC, UPDATE_PREBUILT = 1, 2
STEP_BWD_ONLY, STEP_APPLY_ONLY = 1, 2
IX_BUILT, IX_SPLIT, IX_PREPARED, IX_SINGLES_DONE = 1, 2, 4, 8
COMM_ID_BYTES = 128


class DLRMError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[dlrm_hip status {code}] {msg}")
        self.code = code


class BoundsError(IndexError):
    """Out-of-range embedding index (the reference raises Julia's BoundsError)."""


class LibraryMissing(ImportError):
    pass


_vp, _i32, _i64, _f32, _u32, _sz = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float,
                                    ctypes.c_uint, ctypes.c_size_t)
_pp = ctypes.POINTER(ctypes.c_void_p)
_pi64 = ctypes.POINTER(ctypes.c_int64)

# name -> (restype, argtypes); must match include/dlrm_hip.h (checked by tests/test_abi.py)
SIGNATURES = {
    "dlrm_abi_version": (_i32, []),
    "dlrm_ctx_create": (_i32, [_i32, _vp, _pp]),
    "dlrm_ctx_destroy": (_i32, [_vp]),
    "dlrm_ctx_set_stream": (_i32, [_vp, _vp]),
    "dlrm_last_error": (ctypes.c_char_p, [_vp]),
    "dlrm_debug_fatal_trace": (_i32, [_i32]),
    "dlrm_sync": (_i32, [_vp]),
    "dlrm_check_bounds": (_i32, [_vp]),
    "dlrm_error_snapshot": (_i32, [_vp]),
    "dlrm_error_peek": (_i32, [_vp, _vp]),
    "dlrm_malloc": (_i32, [_vp, _sz, _pp]),
    "dlrm_free": (_i32, [_vp, _vp]),
    "dlrm_memcpy_h2d": (_i32, [_vp, _vp, _vp, _sz]),
    "dlrm_memcpy_d2h": (_i32, [_vp, _vp, _vp, _sz]),
    "dlrm_memcpy_h2d_async": (_i32, [_vp, _vp, _vp, _sz]),
    "dlrm_host_register": (_i32, [_vp, _sz]),
    "dlrm_host_unregister": (_i32, [_vp]),
    "dlrm_tables_create": (_i32, [_vp, _i32, _i32, _i32, _pp, _pi64, _pp]),
    "dlrm_tables_destroy": (_i32, [_vp]),
    "dlrm_maplookup": (_i32, [_vp, _vp, _vp, _i32, _i64, _i32, _i32, _i32, _vp, _i64, _i64]),
    "dlrm_maplookup_blocked": (_i32, [_vp, _vp, _vp, _i32, _i64, _i32, _i32, _i32, _vp, _i64, _i64, _i64, _i64,
                                      _i64]),
    "dlrm_indexer_build_split": (_i32, [_vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32]),
    "dlrm_scatter_rows": (_i32, [_vp, _i32, _i32, _i32, _i32, _vp, _i64, _i64, _vp, _vp, _vp]),
    "dlrm_interact_fwd": (_i32, [_vp, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _i64, _i32]),
    "dlrm_lookup_interact_fwd": (_i32, [_vp, _vp, _vp, _i32, _i64, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _i64,
                                         _i32]),
    "dlrm_interact_bwd": (_i32, [_vp, _i32, _i32, _i32, _i32, _vp, _i64, _i32, _vp, _i64, _vp, _i64, _vp, _i64]),
    "dlrm_interact_bwd_gather": (_i32, [_vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _i32,
                                        _vp, _i64, _vp, _i64]),
    "dlrm_triangular_slice": (_i32, [_vp, _i32, _i32, _i32, _vp, _i64, _vp, _i64]),
    "dlrm_triangular_slice_back": (_i32, [_vp, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _i32]),
    "dlrm_self_batched_mul": (_i32, [_vp, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _i64]),
    "dlrm_self_batched_mul_back": (_i32, [_vp, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _i64]),
    "dlrm_indexer_create": (_i32, [_vp, _i32, _i64, _pp]),
    "dlrm_indexer_destroy": (_i32, [_vp]),
    "dlrm_indexer_build": (_i32, [_vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32, _i32]),
    "dlrm_indexer_read": (_i32, [_vp, _vp, _i32, _pi64, _pi64, _pi64, _pi64, _i64]),
    "dlrm_indexer_state": (_i32, [_vp, ctypes.POINTER(ctypes.c_uint)]),
    "dlrm_indexer_prepare": (_i32, [_vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32]),
    "dlrm_indexer_bytes": (_i32, [_vp, _vp]),
    "dlrm_indexer_reserve": (_i32, [_vp, _vp, _i32]),
    "dlrm_indexer_set_chunk": (_i32, [_vp, _vp, _i32]),
    "dlrm_indexer_set_parts": (_i32, [_vp, _vp, _i32]),
    "dlrm_sgd_update": (_i32, [_vp, _vp, _vp, _u32, _vp, _i32, _i64, _i32, _i32, _i32, _vp, _i32, _i64, _i64, _f32]),
    "dlrm_bce_head": (_i32, [_vp, _i32, _vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    "dlrm_relu_bwd_bias_workspace": (_i32, [_i32, _i32, _pi64, _pi64]),
    "dlrm_relu_bwd_bias": (_i32, [_vp, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _vp, _vp]),
    "dlrm_dac_parse_tsv": (_i32, [_vp, _i64, _vp, _i64, _pi64]),
    "dlrm_dac_maps_create": (_i32, [_pp]),
    "dlrm_dac_maps_destroy": (_i32, [_vp]),
    "dlrm_dac_maps_add": (_i32, [_vp, _vp, _i64]),
    "dlrm_dac_maps_sizes": (_i32, [_vp, _pi64]),
    "dlrm_dac_maps_lookup": (_i32, [_vp, _i32, _u32, ctypes.POINTER(ctypes.c_uint32)]),
    "dlrm_dac_reindex": (_i32, [_vp, _vp, _i64]),
    "dlrm_dac_decode": (_i32, [_vp, _vp, _i32, _vp, _vp, _i64, _vp, _i32, _i64]),
    "dlrm_dac_loader_create": (_i32, [_i32, _vp, _i64, _i32, _i32, _pp, _pp, _pp, _pp]),
    "dlrm_dac_loader_start": (_i32, [_vp, _pi64]),
    "dlrm_dac_loader_next": (_i32, [_vp, _vp, ctypes.POINTER(ctypes.c_int)]),
    "dlrm_dac_loader_release": (_i32, [_vp, _i32, _vp]),
    "dlrm_dac_loader_stop": (_i32, [_vp]),
    "dlrm_dac_loader_destroy": (_i32, [_vp]),
    "dlrm_comm_unique_id": (_i32, [_vp]),
    "dlrm_comm_init": (_i32, [_vp, _vp, _i32, _i32, _pp]),
    "dlrm_comm_destroy": (_i32, [_vp]),
    "dlrm_comm_count": (_i32, [_vp, _vp]),
    "dlrm_alltoall_fwd": (_i32, [_vp, _vp, _i32, _i32, _i32, ctypes.POINTER(ctypes.c_int), _vp, _vp]),
    "dlrm_alltoall_bwd": (_i32, [_vp, _vp, _i32, _i32, ctypes.POINTER(ctypes.c_int), _vp, _vp]),
    "dlrm_interact_bwd_blocked": (_i32, [_vp, _vp, _vp, _i32, _i64, _i32, _i32, _vp, _i64, _vp, _i64, _i32, _vp,
                                         _i64, _vp, _vp, _vp]),
    "dlrm_step_fwd": (_i32, [_vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32, _vp, _i64, _vp, _i64, _i32]),
    "dlrm_step_bwd": (_i32, [_vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32, _vp, _i64, _vp, _i64, _i32, _vp, _i64, _vp,
                             _i64, _f32, _u32]),
    "dlrm_step_bwd_prepare": (_i32, [_vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32, _vp, _i64, _vp, _i64, _i32, _vp, _i64,
                                     _vp, _i64, _f32, _vp, _vp, _u32]),
}

_lib = None
_lock = threading.Lock()


def header_functions(path=HEADER):
    """Names of every function the C header declares (used by the ABI export test)."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dlrm_[a-z0-9_]+)\s*\(", text)))


def load(path=LIB_PATH):
    """Loads the HIP library once.  Raises LibraryMissing if it was not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise LibraryMissing(
                f"{path} not found: build it with `make -C dlrm.jl_amd/csrc` or __graft_entry__.build(); "
                "the DLRM hot path has no CPU fallback")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(rc, ctx=None):
    if rc == OK:
        return
    msg = ""
    if ctx is not None and _lib is not None:
        raw = _lib.dlrm_last_error(ctx)
        msg = raw.decode() if raw else ""
    if rc == E_INDEX:
        raise BoundsError(msg or "embedding index out of range")
    raise DLRMError(rc, msg)
