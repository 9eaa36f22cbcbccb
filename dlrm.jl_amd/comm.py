"""The table-sharded exchange through the library's own RCCL entry points (dlrm_comm_*,
dlrm_alltoall_fwd / _bwd in include/dlrm_hip.h).

This is the path a host process per GPU without torch.distributed takes (the Julia shim binds
the same functions).  `ShardedHotPath(..., exchange="abi")` (or
DLRM_EXCHANGE=abi) uses it instead of torch.distributed's all_to_all_single; the layouts are
the same, so the two are interchangeable bit for bit.
"""
import ctypes

import torch

from . import _lib
from .runtime import context, dtype_code, ptr


class CommExchange:
    """One RCCL communicator over `world` ranks (this process = `rank`, on `device`).

    uid: the DLRM_COMM_ID_BYTES bytes from dlrm_comm_unique_id on one rank.  None: rank 0 makes
    them and, for world > 1, torch.distributed (already initialised) broadcasts them."""

    def __init__(self, rank, world, device, uid=None, group=None):
        self.ctx = context(device)
        self.lib = self.ctx.lib
        self.rank, self.world = int(rank), int(world)
        if uid is None:
            buf = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
            if self.rank == 0:
                _lib.check(self.lib.dlrm_comm_unique_id(buf))
            if self.world > 1:
                import torch.distributed as dist
                obj = [bytes(buf.raw) if self.rank == 0 else None]
                dist.broadcast_object_list(obj, src=0, group=group)
                buf = ctypes.create_string_buffer(obj[0], _lib.COMM_ID_BYTES)
            uid = buf.raw
        if len(uid) != _lib.COMM_ID_BYTES:
            raise ValueError(f"a communicator id has {_lib.COMM_ID_BYTES} bytes")
        self._uid = ctypes.create_string_buffer(bytes(uid), _lib.COMM_ID_BYTES)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.ctx.device):
            self.ctx.check(self.lib.dlrm_comm_init(self.ctx.bind(), self._uid, self.rank, self.world, ctypes.byref(h)))
        self.handle = h
        # hipGraphs that captured this communicator's exchanges.  RCCL keeps a reference on the
        # communicator for every live graph holding its work, and ncclCommDestroy waits for those
        # references to go: destroying the communicator while such a graph is alive never returns
        # (the round-4 "capture hang" of test_sharded_whole_step_graph_world1 was exactly that, at
        # the test's end, when Python freed the communicator before the engine's graphs).  So the
        # graphs are registered here and reset before the communicator is destroyed.
        self._graphs = []

    def retain_graphs(self, graphs):
        """Registers captured graphs that hold this communicator's work (reset by close())."""
        self._graphs.extend(graphs)

    @staticmethod
    def _counts(counts):
        return (ctypes.c_int * len(counts))(*[int(c) for c in counts])

    def nranks(self):
        """The rank count RCCL reports for this communicator (dlrm_comm_count = ncclCommCount)."""
        n = ctypes.c_int(0)
        _lib.check(self.lib.dlrm_comm_count(self.handle, ctypes.byref(n)))
        return n.value

    def alltoall_fwd(self, send, recv, dim, batch_local, counts):
        """send [world][T_me][B][dim] -> recv [src][T_src][B][dim] (dtype of send)."""
        self.ctx.check(self.lib.dlrm_alltoall_fwd(self.ctx.bind(), self.handle, dtype_code(send.dtype), dim,
                                                  batch_local, self._counts(counts), ptr(send), ptr(recv)))

    def alltoall_bwd(self, gsend, grecv, dim, batch_local, counts):
        """gsend [owner][B][T_owner][dim] fp32 -> grecv [src][B][T_me][dim] fp32."""
        if gsend.dtype != torch.float32 or grecv.dtype != torch.float32:
            raise TypeError("the gradient exchange is fp32")
        self.ctx.check(self.lib.dlrm_alltoall_bwd(self.ctx.bind(), self.handle, dim, batch_local,
                                                  self._counts(counts), ptr(gsend), ptr(grecv)))

    def close(self):
        for g in getattr(self, "_graphs", ()):
            g.reset()  # (first: see __init__)
        self._graphs = []
        if getattr(self, "handle", None):
            torch.cuda.synchronize(self.ctx.device)
            self.lib.dlrm_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
