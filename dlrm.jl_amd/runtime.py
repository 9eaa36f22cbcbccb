"""Device context: one dlrm_ctx per GPU, bound to torch's current stream at each call.

Mirrors the ABI's threading rule (one ctx = one device + one stream, not re-entrant):
every call re-binds the ctx to `torch.cuda.current_stream()`, so kernels are ordered with
the surrounding torch work and can be captured by torch.cuda graphs.
"""
import ctypes
import threading

import torch

from . import _lib

_contexts = {}
_lock = threading.Lock()


class Context:
    def __init__(self, device_index):
        self.lib = _lib.load()
        self.device = device_index
        h = ctypes.c_void_p()
        with torch.cuda.device(device_index):
            _lib.check(self.lib.dlrm_ctx_create(device_index, None, ctypes.byref(h)))
        self.handle = h

    def bind(self):
        """Returns the ctx handle bound to torch's current stream on this device."""
        stream = torch.cuda.current_stream(self.device).cuda_stream
        self.lib.dlrm_ctx_set_stream(self.handle, ctypes.c_void_p(stream))
        return self.handle

    def check(self, rc):
        _lib.check(rc, self.handle)

    def check_bounds(self):
        """Synchronises and raises BoundsError if a kernel skipped an out-of-range index."""
        self.check(self.lib.dlrm_check_bounds(self.bind()))

    def error_snapshot(self):
        """Queues a copy of the device error flag into host memory (no synchronisation; capturable)."""
        self.check(self.lib.dlrm_error_snapshot(self.bind()))

    def error_peek(self):
        """The last snapshot of the error flag that has landed (no GPU call; 0 = none seen)."""
        w = ctypes.c_uint()
        self.check(self.lib.dlrm_error_peek(self.handle, ctypes.byref(w)))
        return w.value

    def __del__(self):
        try:
            if self.handle:
                self.lib.dlrm_ctx_destroy(self.handle)
        except Exception:
            pass


def context(device=None):
    if not torch.cuda.is_available():
        raise RuntimeError("dlrm.jl_amd needs a ROCm GPU (torch.cuda.is_available() is False); "
                           "there is no CPU fallback for the hot path")
    if device is None:
        idx = torch.cuda.current_device()
    elif isinstance(device, torch.device):
        idx = device.index if device.index is not None else torch.cuda.current_device()
    else:
        idx = int(device)
    with _lock:
        ctx = _contexts.get(idx)
        if ctx is None:
            ctx = _contexts[idx] = Context(idx)
        return ctx


def require_device(t, device, name):
    """Every buffer handed to a kernel must be a CUDA tensor on the ctx's device: a host
    pointer would fault the GPU.  Raises ValueError before anything is launched."""
    if t is None:
        return
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch tensor, got {type(t).__name__}")
    if not t.is_cuda or (device is not None and t.device != torch.device(device)):
        raise ValueError(f"{name} lives on {t.device}, the kernel runs on {device}")


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def dtype_code(dt):
    if dt == torch.float32:
        return _lib.F32
    if dt == torch.bfloat16:
        return _lib.BF16
    raise TypeError(f"unsupported dtype {dt}: the hot path computes in float32 or bfloat16")


def itype_code(dt):
    if dt == torch.int32:
        return _lib.I32
    if dt == torch.int64:
        return _lib.I64
    raise TypeError(f"unsupported index dtype {dt}: int32 or int64")
