"""The dense half of a DLRM training step around the hot path.

The reference's model (src/model/model.jl:124-163) is

    y   = maplookup(strategy, embeddings, sparse)        -> the hot path (HIP)
    x   = bottom_mlp(dense)                              -> Dense layers, relu   (model.jl:72-93)
    z   = interaction(x, y)                              -> the hot path (HIP)
    out = top_mlp(z)                                     -> Dense layers, relu, last: sigmoid
    l   = bce_loss(out, labels)                          (train.jl:33-41)

and one `train!` iteration (train.jl:215-227) takes the Zygote gradient of all of it and
applies `custom_update!(Descent(η))` (train.jl:232-292): every dense weight and bias gets
`p .-= η·g`, the tables get `EmbeddingTables.update!` (here: inside `HotPath.backward`).

The MLP GEMMs run on rocBLAS/hipBLASLt through torch (plain library GEMMs, the guide's rule);
the loss, its pullback and the SGD are a handful of elementwise launches.  No autograd: every
activation the backward needs is kept from the forward, so a whole step is a fixed launch
sequence on the current stream and can be captured in a torch.cuda graph.  Layouts follow the
hot path's: C row-major [B][features] (Julia's (features, B) column-major), weights W[out][in]
(Flux's Dense orientation).
"""
import ctypes
import math

import torch
import torch.distributed as dist

from . import _lib

from .embedding import EmbeddingTableSet
from .hotpath import HotPath
from .interact import interaction_sizes
from .runtime import context, ptr, require_device


def glorot_normal(out_f, in_f, generator=None, device=None):
    """GlorotNormal (model.jl:58-59): N(0, sqrt(2 / (out + in)))."""
    w = torch.empty((out_f, in_f), dtype=torch.float32, device=device)
    return w.normal_(0.0, math.sqrt(2.0 / (out_f + in_f)), generator=generator)


class DenseMLP:
    """`create_mlp(sizes, sigmoid_index)` (model.jl:72-93): Dense(in, out, relu) layers; with
    `sigmoid_last` the last layer is identity followed by a float32 sigmoid."""

    def __init__(self, weights, biases, *, sigmoid_last=False):
        if len(weights) != len(biases) or not weights:
            raise ValueError("one bias per weight, at least one layer")
        for i, (w, b) in enumerate(zip(weights, biases)):
            if w.dim() != 2 or b.shape != (w.shape[0],):
                raise ValueError(f"layer {i}: weight must be [out][in], bias [out]")
            if i and w.shape[1] != weights[i - 1].shape[0]:
                raise ValueError(f"layer {i}: input size {w.shape[1]} != previous output {weights[i - 1].shape[0]}")
        self.W = [w.detach().float().clone().contiguous() for w in weights]  # owned (updated in place)
        self.b = [b.detach().float().clone().contiguous() for b in biases]
        self.sigmoid_last = sigmoid_last
        self.gW = [torch.zeros_like(w) for w in self.W]
        self.gb = [torch.zeros_like(b) for b in self.b]
        self._acts = None  # [input, a_1, ..., a_n] of the last forward
        self._logits = False
        self.flat_param = self.flat_grad = None
        self._ws = {}  # (layer, batch) -> dlrm_relu_bwd_bias scratch
        self._context = None

    def flatten(self):
        """Re-homes every weight/bias AND its gradient as views of two flat fp32 buffers with the
        same piece offsets (every piece 16-B aligned: dlrm_relu_bwd_bias writes gb in float4s).
        The Descent step is then one axpy launch over the whole MLP, and a data-parallel step
        all-reduces the gradients as one bucket (the returned flat gradient)."""
        if self.flat_grad is not None:
            return self.flat_grad

        def padded(k):
            return (k + 3) // 4 * 4

        n = sum(padded(g.numel()) for g in self.gW + self.gb)
        dev = self.W[0].device
        fp = torch.zeros(n, dtype=torch.float32, device=dev)
        fg = torch.zeros(n, dtype=torch.float32, device=dev)
        o = 0
        for plist, glist in ((self.W, self.gW), (self.b, self.gb)):
            for i in range(len(plist)):
                k = plist[i].numel()
                fp[o:o + k].copy_(plist[i].reshape(-1))
                plist[i] = fp[o:o + k].view(plist[i].shape)
                glist[i] = fg[o:o + k].view(glist[i].shape)
                o += padded(k)
        self.flat_param, self.flat_grad = fp, fg
        return fg

    @property
    def sizes(self):
        return [self.W[0].shape[1]] + [w.shape[0] for w in self.W]

    def params(self):
        return self.W + self.b

    def grads(self):
        return self.gW + self.gb

    def forward(self, x, *, logits=False):
        """The activations of every layer; with `logits` (a sigmoid-last MLP) the last layer's
        sigmoid is left to `dlrm_bce_head` and the logits are returned."""
        acts = [x]
        n = len(self.W)
        for i in range(n):
            if i == n - 1 and self.sigmoid_last:
                y = torch.addmm(self.b[i], acts[-1], self.W[i].t())
                if not logits:
                    y = torch.sigmoid(y)  # Base.Fix1(OneDNN.eltwise, Flux.sigmoid), float32
            else:
                # relu(x W^T + b) with the bias + relu in the GEMM's epilogue (hipBLASLt)
                y = torch._addmm_activation(self.b[i], acts[-1], self.W[i].t())
            acts.append(y)
        self._acts = acts
        self._logits = logits and self.sigmoid_last
        return acts[-1]

    def _relu_seam(self, i, g):
        """relu pullback + bias gradient of layer i: one HIP launch on the GPU (dlrm_relu_bwd_bias),
        the torch formulation on CPU tensors (test-side reference of the same math)."""
        y = self._acts[i + 1]
        if not g.is_cuda:
            g = torch.ops.aten.threshold_backward(g, y, 0.0)  # relu': y > 0
            torch.sum(g, dim=0, out=self.gb[i])
            return g
        B, N = g.shape
        ws = self._ws.get((i, B))
        if ws is None:
            nw, nc = ctypes.c_int64(), ctypes.c_int64()
            _lib.check(self._ctx().lib.dlrm_relu_bwd_bias_workspace(B, N, ctypes.byref(nw), ctypes.byref(nc)))
            ws = self._ws[(i, B)] = (torch.empty(max(nw.value, 4), dtype=torch.float32, device=g.device),
                                      torch.zeros(max(nc.value, 1), dtype=torch.int32, device=g.device))
        g = g.contiguous()
        ctx = self._ctx()
        ctx.check(ctx.lib.dlrm_relu_bwd_bias(ctx.bind(), B, N, ptr(y), y.stride(0), ptr(g), g.stride(0),
                                             ptr(self.gb[i]), ptr(ws[0]), ptr(ws[1])))
        return g

    def _ctx(self):
        if self._context is None:
            self._context = context(self.W[0].device)
        return self._context

    def backward(self, dy, *, need_dx=True):
        """dy = dLoss/d(the last activation's output) -> dLoss/d(input); fills gW, gb.  After a
        `forward(..., logits=True)`, dy is dLoss/dlogit and the last bias gradient is the caller's
        (dlrm_bce_head writes it)."""
        acts = self._acts
        n = len(self.W)
        g = dy
        for i in reversed(range(n)):
            if i == n - 1 and self.sigmoid_last:
                if not self._logits:
                    y = acts[i + 1]
                    g = g * y * (1.0 - y)  # sigmoid' = s(1 - s)
                    torch.sum(g, dim=0, out=self.gb[i])
            else:
                g = self._relu_seam(i, g)
            torch.mm(g.t(), acts[i], out=self.gW[i])
            if i > 0 or need_dx:
                g = torch.mm(g, self.W[i])
        return g if need_dx else None

    def sgd_(self, lr):
        """Flux.update!(Descent(η), p, g) for every weight and bias (train.jl:251-271): one launch
        over the flat buffers after `flatten`, else one multi-tensor launch.  (The padding between
        pieces holds zero gradients, so it stays zero.)"""
        if self.flat_param is not None:
            self.flat_param.add_(self.flat_grad, alpha=-float(lr))
        else:
            torch._foreach_add_(self.params(), self.grads(), alpha=-float(lr))


def bce_loss(p, labels):
    """train.jl:33-41: mean(-y·max(log p, -100) + (y - 1)·max(log(1 - p), -100))."""
    lp = torch.clamp_min(torch.log(p), -100.0)
    lq = torch.clamp_min(torch.log(1.0 - p), -100.0)
    return torch.mean(-labels * lp + (labels - 1.0) * lq)


def bce_loss_back(p, labels, dl=1.0):
    """rrule(bce_loss) (train.jl:43-64): dp = (Δ/n)·((1 - y)/(1 - p + ε) - y/(p + ε))."""
    eps = torch.finfo(p.dtype).eps
    d = dl / p.numel()
    return d * ((1.0 - labels) / (1.0 - p + eps) - labels / (p + eps))


class DLRMModel:
    """`DLRMModel(bottom_mlp, embeddings, interaction, top_mlp)` (model.jl:110-163) with the hot
    path (maplookup + DotInteraction + dot_back + update!) behind `HotPath`.

    `step(dense, sparse, labels)` is one `train!` iteration with `Descent(lr)`: returns the loss
    (a device scalar, no host sync).  `forward(dense, sparse)` is the model call (probabilities).
    """

    def __init__(self, bottom, tables, top, batch, lookups=1, *, lr=0.1, index_base=0, **hot_kw):
        self.bottom, self.top = bottom, top
        ts = tables if isinstance(tables, EmbeddingTableSet) else EmbeddingTableSet(tables)
        self.hot = HotPath(ts, batch, lookups, lr=lr, index_base=index_base, **hot_kw)
        self.lr = float(lr)
        d, F = bottom.sizes[-1], len(ts) + 1
        if d != ts.D:
            raise ValueError(f"bottom MLP output {d} != embedding feature size {ts.D} (model.jl:220)")
        width = self.hot.width
        if top.sizes[0] != width:
            raise ValueError(f"top MLP input {top.sizes[0]} != interaction output {width} (model.jl:225-231)")
        if not top.sigmoid_last:
            raise ValueError("the top MLP ends in the sigmoid (model.jl:232)")
        self.tdtype = ts.dtype
        self.loss = None
        self.prob = None
        bottom.flatten()  # one Descent launch per MLP
        top.flatten()

    @property
    def tables(self):
        return self.hot.ts

    def forward(self, dense, sparse):
        x = self.bottom.forward(dense)
        out = self.hot.forward(x.to(self.tdtype), sparse)
        self.prob = self.top.forward(out.float()).reshape(-1)
        return self.prob

    def head(self, z, labels):
        """dlrm_bce_head on the top MLP's logits: prob, loss, dLoss/dlogit (self._dz) and the last
        layer's bias gradient, one launch."""
        B = z.shape[0]
        check_labels(labels, z)
        if self.prob is None or self.prob.shape[0] != B:
            self.prob = torch.empty(B, dtype=torch.float32, device=z.device)
            self.loss = torch.empty((), dtype=torch.float32, device=z.device)
            self._dz = torch.empty((B, 1), dtype=torch.float32, device=z.device)
        ctx = self.top._ctx()
        ctx.check(ctx.lib.dlrm_bce_head(ctx.bind(), B, ptr(z), z.stride(0), ptr(labels), ptr(self.prob),
                                        ptr(self._dz), ptr(self.loss), ptr(self.top.gb[-1])))
        return self.loss

    def step(self, dense, sparse, labels):
        """train.jl:215-227 + custom_update! (train.jl:232-292)."""
        if not dense.is_cuda:
            raise ValueError("DLRMModel.step runs on the GPU (the hot path has no CPU fallback)")
        x = self.bottom.forward(dense)
        out = self.hot.forward(x.to(self.tdtype), sparse)
        z = self.top.forward(out.float(), logits=True)  # [B][1]
        self.head(z, labels)
        dout = self.top.backward(self._dz)
        dx = self.hot.backward(sparse, dout.to(self.tdtype).contiguous())  # tables updated here
        self.bottom.backward(dx, need_dx=False)
        self.top.sgd_(self.lr)
        self.bottom.sgd_(self.lr)
        return self.loss


def check_labels(labels, z):
    """dlrm_bce_head reads labels as a packed fp32 vector of the logits' batch on their device."""
    B = z.shape[0]
    if labels.shape != (B,) or labels.dtype != torch.float32 or not labels.is_contiguous():
        raise ValueError(f"labels must be a contiguous float32 vector of {B}")
    require_device(labels, z.device, "labels")


def kaggle_mlp_sizes(feature_size, num_tables):
    """kaggle_dlrm (criteo.jl:408-433): bottom [13, 512, 256, D], top [D + P, 1024, 1024, 512, 256, 1]
    with P = F(F-1)/2 pairs of the F = T + 1 interacting vectors (model.jl:218-231)."""
    F = num_tables + 1
    _, width, _ = interaction_sizes(feature_size, F)
    return [13, 512, 256, feature_size], [width, 1024, 1024, 512, 256, 1]


def random_mlp(sizes, *, sigmoid_last, generator=None, device=None):
    """Dense layers of `sizes`: GlorotNormal weights (model.jl:187-192), zero biases (Flux.Dense's
    default bias)."""
    Ws = [glorot_normal(o, i, generator, device) for i, o in zip(sizes[:-1], sizes[1:])]
    bs = [torch.zeros(o, dtype=torch.float32, device=device) for o in sizes[1:]]
    return DenseMLP(Ws, bs, sigmoid_last=sigmoid_last)


class ShardedDLRMModel:
    """The full training step on one rank of a table-sharded, data-parallel job (SURVEY §8 rows
    f1 + f3): the MLPs are replicated (data parallel, B samples per rank), the tables are sharded
    by table (`sharded.ShardedHotPath`: one all-to-all each way), and the MLP gradients are summed
    over ranks with all-reduce (RCCL over xGMI for backend "nccl").

    The loss is the global-batch mean, as one process on the world*B batch would compute it
    (train.jl:33-41): dLoss/dlogit carries 1/(world*B), so the summed dense gradients and the
    tables' updates equal the single-process step.  Two gradient buckets: the top MLP's is
    all-reduced asynchronously while the sparse backward (exchange + table update) runs, the
    bottom MLP's after its backward.  Descent(lr) then runs on every rank's replica.
    """

    def __init__(self, bottom, top, engine, lr, group=None):
        self.bottom, self.top, self.engine = bottom, top, engine
        self.lr = float(lr)
        self.group = group
        self.world = engine.world
        self.tdtype = engine.out.dtype
        self._top_flat = top.flatten()
        self._bot_flat = bottom.flatten()
        self.loss = None
        self.prob = None

    def _head(self, z, labels):
        scale = 1.0 / self.world
        if z.is_cuda:
            B = z.shape[0]
            check_labels(labels, z)
            if self.prob is None or self.prob.shape[0] != B:
                self.prob = torch.empty(B, dtype=torch.float32, device=z.device)
                self.loss = torch.empty((), dtype=torch.float32, device=z.device)
                self._dz = torch.empty((B, 1), dtype=torch.float32, device=z.device)
            ctx = self.top._ctx()
            ctx.check(ctx.lib.dlrm_bce_head(ctx.bind(), B, ptr(z), z.stride(0), ptr(labels), ptr(self.prob),
                                            ptr(self._dz), ptr(self.loss), ptr(self.top.gb[-1])))
            if self.world > 1:
                self._dz.mul_(scale)
                self.top.gb[-1].mul_(scale)
            return self._dz
        # CPU tensors (the gloo tests): the same formulas in torch
        p = torch.sigmoid(z).reshape(-1)
        self.prob = p
        self.loss = bce_loss(p, labels)
        dz = (bce_loss_back(p, labels) * p * (1.0 - p) * scale).reshape(-1, 1)
        self.top.gb[-1].copy_(dz.sum(0))
        return dz

    def step(self, dense, idx, labels):
        """dense [B][13] and labels [B] of this rank's samples; idx: PackedIndices of this rank's
        tables for the GLOBAL batch (ShardedHotPath's convention).  Returns the global-batch loss
        (a device scalar; the all-reduce is queued, not waited on by the host)."""
        x = self.bottom.forward(dense)
        xt = x.to(self.tdtype)  # the hot path reads x in the tables' dtype, forward and backward
        out = self.engine.forward(xt, idx)
        z = self.top.forward(out.float(), logits=True)
        dz = self._head(z, labels)
        dout = self.top.backward(dz)
        multi = self.world > 1
        w_top = dist.all_reduce(self._top_flat, group=self.group, async_op=True) if multi else None
        dx = self.engine.backward(idx, dout.to(self.tdtype).contiguous(), xt)
        self.bottom.backward(dx, need_dx=False)
        if multi:
            dist.all_reduce(self._bot_flat, group=self.group)
            w_top.wait()
        self.top.sgd_(self.lr)
        self.bottom.sgd_(self.lr)
        loss = self.loss.detach().clone().reshape(1)
        if multi:
            dist.all_reduce(loss, group=self.group)
            loss /= self.world
        return loss.reshape(())
