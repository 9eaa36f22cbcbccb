"""ctypes binding of the C oracle (oracle/dlrm_oracle.c) + tiny pure-Python restatements.

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() (as the checker)
and bench.py's cpu_baseline leg.  Never imported by the product package (dlrm.jl_amd),
which fails loudly when its HIP library is missing instead of falling back to this.

All arrays are numpy, C row-major (a Julia (D, N) matrix is [N][D] here).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libdlrm_oracle.so")
_lib = None

F32, BF16 = 0, 1


class OracleBoundsError(IndexError):
    """The reference raises BoundsError on an out-of-range lookup index."""


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def use_native():
    """Selects the -march=native build of the oracle, compiled by gcc on the host that calls this
    (bench.py's cpu_baseline leg only).  Returns the path, or None (portable build kept)."""
    global _LIB_PATH, _lib
    path = os.path.join(_HERE, "build", "libdlrm_oracle_native.so")
    if _lib is not None and _LIB_PATH == path:
        return path
    try:
        if os.path.exists(path):
            os.unlink(path)  # never reuse one built for another host's CPU
        subprocess.check_call(["make", "-s", "-C", _HERE, "native"], timeout=120)
    except Exception:
        return None
    _LIB_PATH, _lib = path, None
    return path


def host_cpu():
    """(model name, logical CPUs of the machine, CPUs this process may run on)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count() or 1, len(os.sched_getaffinity(0))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i64, i32, f32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
        L.oracle_maplookup.argtypes = [i32, i32, i32, ctypes.POINTER(vp), vp, vp, i64, i32, i32, i32, vp, i64, i64, i32]
        L.oracle_interact_fwd.argtypes = [i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, i32, i32]
        L.oracle_interact_bwd.argtypes = [i32, i32, i32, i32, vp, i64, i32, vp, i64, vp, i64, vp, i64, i32]
        L.oracle_sgd_update.argtypes = [i32, i32, i32, ctypes.POINTER(vp), vp, vp, i64, i32, i32, i32, vp, i32, i64, i64, f32, vp, i32]
        L.oracle_triangular_slice.argtypes = [i32, vp, vp]
        L.oracle_triangular_slice_back_sym.argtypes = [i32, vp, vp]
        L.oracle_max_threads.restype = i32
        L.oracle_fill_uniform.argtypes = [vp, i64, f32, f32, ctypes.c_uint64, i32]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _check(rc):
    if rc == -3:
        raise OracleBoundsError("index out of range")
    if rc != 0:
        raise ValueError(f"oracle error {rc}")


def _dt(a):
    if a.dtype == np.float32:
        return F32
    if a.dtype == np.uint16:  # bf16 bit pattern
        return BF16
    raise TypeError(a.dtype)


def max_threads():
    return lib().oracle_max_threads()


def maplookup(tables, idx, base, B, L, out, out_offset, nthreads=0):
    """tables: list of [N_t][D] arrays (f32 or uint16-bf16); idx: int64 [T][B*L]; out [B][ld]."""
    T = len(tables)
    D = tables[0].shape[1]
    ptrs = (ctypes.c_void_p * T)(*[t.ctypes.data for t in tables])
    nrows = np.array([t.shape[0] for t in tables], dtype=np.int64)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    _check(lib().oracle_maplookup(T, D, _dt(tables[0]), ptrs, _p(nrows), _p(idx), idx.shape[1] if T else 0,
                                  base, B, L, _p(out), out.shape[1], out_offset, nthreads))
    return out


def interact_fwd(x, ys, F, padding=0, nthreads=0):
    B, d = x.shape
    out = np.zeros((B, d + F * (F - 1) // 2 + padding), dtype=x.dtype)
    _check(lib().oracle_interact_fwd(_dt(x), d, F, B, _p(x), x.shape[1], _p(ys), ys.shape[1], _p(out),
                                     out.shape[1], padding, nthreads))
    return out


def interact_bwd(dout, t, d, F, padding=0, nthreads=0):
    B = dout.shape[0]
    dx = np.zeros((B, d), dtype=np.float32)
    dt = np.zeros((B, F * d), dtype=np.float32)
    _check(lib().oracle_interact_bwd(_dt(dout), d, F, B, _p(dout), dout.shape[1], padding, _p(t), t.shape[1],
                                     _p(dx), d, _p(dt), F * d, nthreads))
    return dx, dt


def sgd_update(tables, idx, base, B, L, grad, grad_offset, lr, nthreads=0):
    """In place on `tables`; returns per-table unique-row counts."""
    T = len(tables)
    D = tables[0].shape[1]
    ptrs = (ctypes.c_void_p * T)(*[t.ctypes.data for t in tables])
    nrows = np.array([t.shape[0] for t in tables], dtype=np.int64)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    uniq = np.zeros(T, dtype=np.int64)
    _check(lib().oracle_sgd_update(T, D, _dt(tables[0]), ptrs, _p(nrows), _p(idx), idx.shape[1] if T else 0,
                                   base, B, L, _p(grad), _dt(grad), grad.shape[1], grad_offset, lr, _p(uniq),
                                   nthreads))
    return uniq


def fill_uniform(a, lo, hi, seed, nthreads=0):
    """In-place U(lo, hi) fill of a float32 array (multithreaded; CPU-baseline setup)."""
    assert a.dtype == np.float32 and a.flags.c_contiguous
    lib().oracle_fill_uniform(_p(a), a.size, lo, hi, seed, nthreads)
    return a


def triangular_slice(z):
    F = z.shape[0]
    z = np.ascontiguousarray(z, dtype=np.float32)
    y = np.zeros(F * (F - 1) // 2, dtype=np.float32)
    lib().oracle_triangular_slice(F, _p(z), _p(y))
    return y


def triangular_slice_back_sym(y, F):
    y = np.ascontiguousarray(y, dtype=np.float32)
    z = np.zeros((F, F), dtype=np.float32)
    lib().oracle_triangular_slice_back_sym(F, _p(y), _p(z))
    return z


# ---- bf16 helpers (bit patterns in uint16) -------------------------------------------
def f32_to_bf16(a):
    """Round-to-nearest-even float32 -> bf16 bit pattern (uint16); NaN stays NaN."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = (u & 0x7F800000) == 0x7F800000
    nan &= (u & 0x007FFFFF) != 0
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def bf16_to_f32(h):
    return (np.ascontiguousarray(h, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


# ---- float64 numpy restatement (reference-of-record, interact.jl:7-31) -----------------
def dot_interaction_reference(x, ys_list):
    """dot_interaction_reference(X, Ys): vcat -> batched T'T -> strict triangle -> vcat(X, Zflat).
    x: [B][d]; ys_list: list of [B][d]; returns [B][d + P] float64."""
    Tm = np.stack([x] + list(ys_list), axis=1).astype(np.float64)  # [B][F][d]
    F = Tm.shape[1]
    Z = Tm @ Tm.transpose(0, 2, 1)
    li, lj = np.tril_indices(F, -1)
    order = np.lexsort((lj, li))  # row-major lower triangle == interact.jl:64-75 order
    return np.concatenate([x.astype(np.float64), Z[:, li[order], lj[order]]], axis=1)
