"""The Criteo DAC data path (SURVEY §8 rows f2 + f4): TSV -> binary DACRecords -> reindexed
categorical ids -> device batches for the hot path.

Reference: src/data/criteo.jl.
    DACRecord (:91-95)              DAC_DTYPE, 160 B, the on-disk binary format (mmap-able)
    parseline / binarize (:137-176) parse_tsv / binarize           (C: dlrm_dac_parse_tsv)
    categorical_values + reindex    DACMaps.add / reindex          (C: dlrm_dac_maps_*)
      (:182-249)
    reindex!(data, maps) (:251-259) DACMaps.reindex_               (C: dlrm_dac_reindex)
    process (:265-273)              process
    load (:114-118)                 load (numpy memmap)
    DACLoader + load! (:284-340)    DACLoader: each batch's raw records are staged into pinned
                                    host memory, copied to HBM on a copy stream and split by the
                                    dlrm_dac_decode kernel into labels [B] f32, dense [B][13] f32
                                    and sparse [26][B] int32 (index_base 1) -- the hot path's index
                                    layout -- while the previous batch computes (double-buffered).

Parsing and reindexing are host C++ in the library (no GPU needed); decoding needs the GPU.
"""
import collections
import ctypes
import gzip
import os

import numpy as np
import torch

from . import _lib
from .runtime import context, itype_code, ptr

NUM_CONTINUOUS = 13  # num_continuous_features(DAC()), criteo.jl:88
NUM_CATEGORICAL = 26  # num_categorical_features(DAC()), criteo.jl:89
DAC_DTYPE = np.dtype([("label", "<i4"), ("continuous", "<f4", (NUM_CONTINUOUS,)),
                      ("categorical", "<u4", (NUM_CATEGORICAL,))])
assert DAC_DTYPE.itemsize == 160


def _read_text(src):
    if isinstance(src, (bytes, bytearray)):
        return bytes(src)
    with (gzip.open(src, "rb") if str(src).endswith(".gz") else open(src, "rb")) as f:  # gunzip_open
        return f.read()


def parse_tsv(src):
    """parseline over every line of a TSV file (.gz allowed) or bytes -> records (DAC_DTYPE)."""
    text = _read_text(src)
    lib = _lib.load()
    cap = text.count(b"\n") + 1
    out = np.empty(cap, dtype=DAC_DTYPE)
    n = ctypes.c_int64()
    buf = ctypes.create_string_buffer(text, len(text))
    _lib.check(lib.dlrm_dac_parse_tsv(buf, len(text), out.ctypes.data, cap, ctypes.byref(n)))
    return out[: n.value].copy()


def binarize(src, dst=None):
    """binarize(src, dst) (criteo.jl:137-162): parsed records, written to `dst` when given and
    returned as a writable memmap of it; in memory otherwise."""
    recs = parse_tsv(src)
    if dst is None:
        return recs
    recs.tofile(dst)
    return load(dst, writable=True)


def load(path, *, writable=False):
    """load(DAC(), path; writable) (criteo.jl:114-118): the binary file as a record array (mmap)."""
    return np.memmap(path, dtype=DAC_DTYPE, mode="r+" if writable else "r")


class DACMaps:
    """Per-feature `Dict{UInt32,UInt32}` value -> id maps (criteo.jl:180-249), ids 1, 2, ... in
    first-appearance order over the records added, shard after shard."""

    def __init__(self):
        self.lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(self.lib.dlrm_dac_maps_create(ctypes.byref(h)))
        self.handle = h

    def add(self, records):
        """categorical_values(records) merged in with reindex! (get!(dict, v, length(dict)+1))."""
        r = np.ascontiguousarray(records, dtype=DAC_DTYPE)
        _lib.check(self.lib.dlrm_dac_maps_add(self.handle, r.ctypes.data, len(r)))
        return self

    def sizes(self):
        """Unique values per feature = the embedding table sizes of the dataset."""
        s = (ctypes.c_int64 * NUM_CATEGORICAL)()
        _lib.check(self.lib.dlrm_dac_maps_sizes(self.handle, s))
        return list(s)

    def lookup(self, feature, value):
        out = ctypes.c_uint32()
        rc = self.lib.dlrm_dac_maps_lookup(self.handle, int(feature), int(value), ctypes.byref(out))
        if rc == _lib.E_INDEX:
            raise KeyError((feature, value))
        _lib.check(rc)
        return out.value

    def reindex_(self, records):
        """reindex!(data, maps) (criteo.jl:251-259) in place (`records` must be writable and
        C-contiguous: an array or a writable memmap)."""
        if records.dtype != DAC_DTYPE or not records.flags.c_contiguous or not records.flags.writeable:
            raise ValueError("reindex_ needs a writable, contiguous DAC_DTYPE array")
        rc = self.lib.dlrm_dac_reindex(self.handle, records.ctypes.data, len(records))
        if rc == _lib.E_INDEX:  # the reference's KeyError from maps[j][value]
            raise KeyError("a categorical value is missing from the maps")
        _lib.check(rc)
        return records

    def __del__(self):
        try:
            if self.handle:
                self.lib.dlrm_dac_maps_destroy(self.handle)
        except Exception:
            pass


def reindex(shards):
    """reindex(sets) / reindex(setsvector) (criteo.jl:222-241): maps over one record array or
    over several shards in order."""
    if isinstance(shards, np.ndarray):
        shards = [shards]
    maps = DACMaps()
    for s in shards:
        maps.add(s)
    return maps


def process(path, binpath=None):
    """process(path, binpath) (criteo.jl:265-273): binarize, build the maps, reindex! in place."""
    if binpath is not None and os.path.exists(binpath):
        os.remove(binpath)
    data = binarize(path, binpath)
    maps = reindex(data)
    maps.reindex_(data)
    return data, maps


DIRECT_MAX_BYTES = 32 << 30  # page-lock datasets up to 32 GB; larger ones stream via pinned staging

Batch = collections.namedtuple("Batch", ["labels", "dense", "sparse"])


class DACLoader:
    """DACLoader(dataset, batchsize) (criteo.jl:309-340) on the GPU.  Iterating yields `Batch`
    tuples of device tensors: labels [B] f32, dense [B][13] f32 and sparse [26][B] (int32 by
    default; 1-based ids = DACLoader's Matrix{UInt32}(B, 26), i.e. the [T][B] index layout
    `PackedIndices` takes with index_base=1).  Only whole batches are produced:
    len = div(length(dataset), batchsize), as in the reference.

    Default (`native`): a C++ prefetch thread (dlrm_dac_loader_*) copies each batch's records into
    one of two pinned (hipHostMalloc) staging buffers, uploads and decodes them on its own stream
    while the caller computes (34.6 M samples/s beside the eager hot-path step, against 30.7 M
    with `native=False`, where the same staging is driven from the caller's thread).  With `direct=True` the dataset's memory is page-locked once
    (dlrm_host_register) and each batch is one async DMA straight out of it (falls back to staging
    when registration is refused, e.g. a read-only file mapping or a dataset over
    DIRECT_MAX_BYTES).  Measured on MI355X (tools/bench_dac_loader.py, B = 2048): staging 53 M
    records/s, direct 20 M records/s, because copies out of registered memory are slower than out
    of hipHostMalloc buffers, so staging is the default.

    The two batch buffers alternate: a yielded batch stays valid until the next batch is
    requested; work queued on the current stream before that request is ordered before the
    buffer is reused.  (A Python prefetch thread staging the next batch was measured slower on
    MI355X, 20.6 M records/s alone and 14.3 M samples/s beside the step, against 53 M and
    27.8-30.7 M for this single-threaded form, so staging runs in the caller's thread.)"""

    def __init__(self, dataset, batchsize, device=None, *, index_dtype=torch.int32, direct=False, native=True):
        if dataset.dtype != DAC_DTYPE:
            raise ValueError("dataset must be a DAC_DTYPE record array (load / binarize)")
        self.dataset = dataset
        self.B = int(batchsize)
        if self.B <= 0:
            raise ValueError("batchsize must be positive")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.ctx = context(self.device)
        self.itype = itype_code(index_dtype)
        self._raw = np.frombuffer(dataset, dtype=np.uint8) if len(dataset) else np.empty(0, np.uint8)
        nbytes = self.B * DAC_DTYPE.itemsize
        self._pinned = [torch.empty(nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        self._dev = [torch.empty(nbytes, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self._out = [Batch(torch.empty(self.B, dtype=torch.float32, device=self.device),
                           torch.empty((self.B, NUM_CONTINUOUS), dtype=torch.float32, device=self.device),
                           torch.empty((NUM_CATEGORICAL, self.B), dtype=index_dtype, device=self.device))
                     for _ in range(2)]
        self._copy = torch.cuda.Stream(device=self.device)
        self._ready = [torch.cuda.Event() for _ in range(2)]
        self._h2d = [None, None]  # event after the H2D out of each pinned buffer
        self._consumed = [torch.cuda.Event() for _ in range(2)]
        # direct DMA: the dataset itself page-locked (hipHostRegister), each batch one async copy
        # straight out of it (no host memcpy, no host wait); else the pinned staging buffers
        self._registered = None
        self._nl = None
        self._iterating = False
        nb = self._raw.nbytes
        if direct and 0 < nb <= DIRECT_MAX_BYTES and self._raw.flags.c_contiguous:
            addr = self._raw.ctypes.data
            if self.ctx.lib.dlrm_host_register(ctypes.c_void_p(addr), nb) == _lib.OK:
                self._registered = addr
        self.direct = self._registered is not None
        # native (default): a C++ prefetch thread stages / uploads / decodes the next batch
        # (dlrm_dac_loader_*) while the caller computes; the Python-driven forms below remain for
        # `direct` and for comparison
        self._nl = None
        if native and not self.direct and len(self) > 0:
            dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
            arr = lambda ts: (ctypes.c_void_p * 2)(*[t.data_ptr() for t in ts])  # noqa: E731
            h = ctypes.c_void_p()
            _lib.check(self.ctx.lib.dlrm_dac_loader_create(
                dev_index, ctypes.c_void_p(self._raw.ctypes.data), len(dataset), self.B, self.itype,
                arr([o.labels for o in self._out]), arr([o.dense for o in self._out]),
                arr([o.sparse for o in self._out]), ctypes.byref(h)))
            self._nl = h
        self.native = self._nl is not None

    def __len__(self):
        return len(self.dataset) // self.B

    def _stage(self, i, slot, wait_consumer):
        nbytes = self.B * DAC_DTYPE.itemsize
        if not self.direct:
            if self._h2d[slot] is not None:
                self._h2d[slot].synchronize()  # the pinned buffer's previous upload has left
            np.copyto(self._pinned[slot].numpy(), self._raw[i * nbytes:(i + 1) * nbytes])
        with torch.cuda.stream(self._copy):
            if wait_consumer:
                self._copy.wait_event(self._consumed[slot])
            if self.direct:
                h = self.ctx.bind()
                self.ctx.check(self.ctx.lib.dlrm_memcpy_h2d_async(h, ptr(self._dev[slot]),
                                                                  ctypes.c_void_p(self._registered + i * nbytes),
                                                                  nbytes))
            else:
                self._dev[slot].copy_(self._pinned[slot], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._copy)
                self._h2d[slot] = ev
            out = self._out[slot]
            h = self.ctx.bind()
            self.ctx.check(self.ctx.lib.dlrm_dac_decode(h, ptr(self._dev[slot]), self.B, ptr(out.labels),
                                                        ptr(out.dense), out.dense.stride(0), ptr(out.sparse),
                                                        self.itype, out.sparse.stride(0)))
            self._ready[slot].record(self._copy)

    def _iter_native(self, cur):
        lib = self.ctx.lib
        if self._iterating:
            raise RuntimeError("DACLoader: another iteration over this loader is still live (its batch "
                               "buffers would be overwritten); finish or close it first")
        _lib.check(lib.dlrm_dac_loader_start(self._nl, None))
        self._iterating = True
        st = ctypes.c_void_p(cur.cuda_stream)
        held = -1
        try:
            while True:
                slot = ctypes.c_int()
                _lib.check(lib.dlrm_dac_loader_next(self._nl, st, ctypes.byref(slot)))
                if slot.value < 0:
                    return
                held = slot.value
                yield self._out[held]
                _lib.check(lib.dlrm_dac_loader_release(self._nl, held, st))  # the caller's work is queued
                held = -1
        finally:
            if held >= 0:
                lib.dlrm_dac_loader_release(self._nl, held, st)
            lib.dlrm_dac_loader_stop(self._nl)
            self._iterating = False

    def close(self):
        """Releases the page-locked dataset (after the queued copies have run) and the native loader."""
        if self._nl is not None:
            self.ctx.lib.dlrm_dac_loader_destroy(self._nl)
            self._nl = None
        if self._registered is not None:
            self._copy.synchronize()
            self.ctx.lib.dlrm_host_unregister(ctypes.c_void_p(self._registered))
            self._registered = None
            self.direct = False

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __iter__(self):
        n = len(self)
        if n == 0:
            return
        cur = torch.cuda.current_stream(self.device)
        if self._nl is not None:
            yield from self._iter_native(cur)
            return
        self._stage(0, 0, wait_consumer=False)
        for i in range(n):
            slot = i & 1
            if i + 1 < n:
                # everything queued so far for batch i-1 (slot ^ 1) precedes its buffers' reuse
                self._consumed[slot ^ 1].record(cur)
                self._stage(i + 1, slot ^ 1, wait_consumer=i >= 1)
            cur.wait_event(self._ready[slot])
            yield self._out[slot]
