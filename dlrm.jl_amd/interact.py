"""DotInteraction — the pairwise-dot feature interaction (src/model/interact.jl:294-489).

`dot = DotInteraction(); out = dot(x, ys)` runs fast_vcat + process_batches on the GPU
(one MFMA kernel); `dot_back(dot, Δ, t, xlen, padding)` runs process_batches_back + sumavx
(one MFMA kernel); `rrule(dot, x, ys)` pairs them like ChainRulesCore.rrule (:438-447).

Shapes (torch, row-major = the transpose of the Julia matrices):
  x   [B][d]                    dense bottom-MLP output
  ys  [B][P + D*T], P == d      maplookup(PreallocationStrategy(d)) output; x is copied in
  out [B][d + F(F-1)/2 + pad]   F = 1 + T, pad from POST_INTERACTION_PAD_TO_MUL (model.jl:32)
  dt  [B][F*d] float32          dt_reshaped, x rows included (:428-435)
"""
import torch

from .runtime import context, dtype_code, ptr, require_device

POST_INTERACTION_PAD_TO_MUL = 1  # model.jl:32


def cdiv(x, y):
    return 1 + (x - 1) // y


def up_to_mul_of(x, y):
    return y * cdiv(x, y)


def interaction_sizes(d, F, pad_to=POST_INTERACTION_PAD_TO_MUL):
    """(unpadded, padded, padding) exactly as process_batches computes them (:449-456)."""
    unpadded = (F * F - F) // 2 + d
    padded = up_to_mul_of(unpadded, pad_to)
    return unpadded, padded, padded - unpadded


class DotInteraction:
    """DotInteraction (interact.jl:369-411).  Holds no per-thread scratchpads: the kernel keeps
    each sample's Gram tile in MFMA accumulators and its packed row in LDS."""

    def __init__(self, pad_to=POST_INTERACTION_PAD_TO_MUL):
        self.pad_to = pad_to

    def __call__(self, x, ys, *, return_t=False, out=None):
        from .lazy import LazyLookup
        if isinstance(ys, LazyLookup):  # HipTables: the fused gather + interaction (dlrm_step_fwd)
            if return_t or out is not None or self.pad_to != POST_INTERACTION_PAD_TO_MUL:
                ys = ys.materialize()
            else:
                return ys.interact(x).out
        if x.dim() != 2 or ys.dim() != 2 or x.shape[0] != ys.shape[0]:
            raise ValueError("DotInteraction: x [B][d] and ys [B][d + D*T] expected")
        if x.dtype != ys.dtype:
            raise TypeError("DotInteraction: x and ys must share a dtype")
        B, d = x.shape
        if ys.shape[1] % d != 0:
            # reshape(combined, (d, :, batchsize)) in the reference requires this (:397)
            raise ValueError(f"ys width {ys.shape[1]} is not a multiple of d={d}")
        if x.stride(1) != 1 or ys.stride(1) != 1:
            raise ValueError("DotInteraction: rows must be contiguous")
        F = ys.shape[1] // d
        _, padded, padding = interaction_sizes(d, F, self.pad_to)
        if out is None:
            out = torch.empty((B, padded), dtype=x.dtype, device=x.device)
        for name, t in (("x", x), ("ys", ys), ("out", out)):
            require_device(t, x.device, name)
        if out.shape[0] != B or out.shape[1] < padded or out.stride(1) != 1:
            raise ValueError("DotInteraction: `out` has the wrong shape/layout")
        ctx = context(x.device)
        ctx.check(ctx.lib.dlrm_interact_fwd(ctx.bind(), dtype_code(x.dtype), d, F, B, ptr(x), x.stride(0), ptr(ys),
                                            ys.stride(0), ptr(out), out.stride(0), padding))
        if return_t:
            return out, ys, padding
        return out


def dot_back(dot, delta, t, xlen, padding, *, dx=None, dt=None):
    """dot_back(dot, Δ, T, xlen, padding) -> (dx, dt_reshaped)   (interact.jl:415-436).
    bf16 Δ is handled like the reference (converted to fp32; dx and dt are fp32)."""
    B = delta.shape[0]
    d = xlen
    F = t.shape[1] // d
    if dx is None:
        dx = torch.empty((B, d), dtype=torch.float32, device=delta.device)
    if dt is None:
        dt = torch.empty((B, F * d), dtype=torch.float32, device=delta.device)
    if delta.dtype != t.dtype:
        raise TypeError("dot_back: Δ and T must share a dtype")
    for name, a in (("Δ", delta), ("T", t), ("dx", dx), ("dt", dt)):
        require_device(a, delta.device, name)
    if (t.shape[0] != B or delta.stride(1) != 1 or t.stride(1) != 1 or dx.shape != (B, d) or
            dt.shape[0] != B or dt.shape[1] < F * d or dx.dtype != torch.float32 or dt.dtype != torch.float32):
        raise ValueError("dot_back: inconsistent shapes/dtypes")
    ctx = context(delta.device)
    ctx.check(ctx.lib.dlrm_interact_bwd(ctx.bind(), dtype_code(delta.dtype), d, F, B, ptr(delta), delta.stride(0),
                                        padding, ptr(t), t.stride(0), ptr(dx), dx.stride(0), ptr(dt), dt.stride(0)))
    return dx, dt


def rrule(dot, x, ys):
    """ChainRulesCore.rrule(dot::DotInteraction, X, Y) (interact.jl:438-447).  With a LazyLookup
    (HipTables): the training step's forward, and a pullback running its backward (lazy.py)."""
    from .lazy import LazyLookup, rrule_lazy
    if isinstance(ys, LazyLookup) and dot.pad_to == POST_INTERACTION_PAD_TO_MUL:
        return rrule_lazy(x, ys)
    if isinstance(ys, LazyLookup):
        ys = ys.materialize()
    forward, t, padding = dot(x, ys, return_t=True)
    xlen = x.shape[1]

    def dot_pullback(delta):
        dx, dy = dot_back(dot, delta, t, xlen, padding)
        return None, dx, dy

    return forward, dot_pullback


# ---- Implementation 2 (interact.jl:176-215, :503-554): the same interaction as separate operators
def _check_3d(name, a, B, n, m):
    if a.dim() != 3 or a.shape != (B, n, m) or a.stride(2) != 1 or a.stride(1) != m:
        raise ValueError(f"{name} must be a [{B}][{n}][{m}] tensor with contiguous matrices")


def triangular_slice(z):
    """triangular_slice(X) (interact.jl:176-191) of a batch of square matrices.  z: [B][sz][sz]
    (row-major view of Julia's (sz, sz, B): z[b][col][row] = X[row, col, b]) -> [B][sz(sz-1)/2],
    entries with row < col in triangular_slice_kernel! order (:64-75).  Bit-exact copy."""
    B, sz = z.shape[0], z.shape[1]
    _check_3d("z", z, B, sz, sz)
    out = torch.empty((B, sz * (sz - 1) // 2), dtype=z.dtype, device=z.device)
    ctx = context(z.device)
    ctx.check(ctx.lib.dlrm_triangular_slice(ctx.bind(), dtype_code(z.dtype), sz, B, ptr(z), z.stride(0), ptr(out),
                                            out.stride(0)))
    return out


def triangular_slice_back(delta, sz, *, symmetric=False):
    """triangular_slice_back(Δ, size) (interact.jl:193-203): [B][ncols] -> [B][sz][sz] with Δ on the
    upper triangle (z[b][col][row], row < col) and zeros elsewhere (triangular_slice_back_kernel!,
    :104-120); symmetric=True is the fused add-transpose form (:150-171)."""
    B = delta.shape[0]
    if delta.dim() != 2 or delta.shape[1] < sz * (sz - 1) // 2 or delta.stride(1) != 1:
        raise ValueError("triangular_slice_back: Δ must be [B][>= sz(sz-1)/2] with contiguous rows")
    a = torch.empty((B, sz, sz), dtype=delta.dtype, device=delta.device)
    ctx = context(delta.device)
    ctx.check(ctx.lib.dlrm_triangular_slice_back(ctx.bind(), dtype_code(delta.dtype), sz, B, ptr(delta),
                                                 delta.stride(0), ptr(a), a.stride(0), 1 if symmetric else 0))
    return a


def rrule_triangular_slice(z):
    """ChainRulesCore.rrule(triangular_slice, x) (interact.jl:205-215)."""
    sz = z.shape[1]

    def triangular_slice_pullback(delta):
        return None, triangular_slice_back(delta, sz)

    return triangular_slice(z), triangular_slice_pullback


def self_batched_mul(t):
    """self_batched_mul(T) (interact.jl:526-537): Z_b = T_bᵀ T_b over the feature dim.
    t: [B][F][d] (Julia's (d, F, B)) -> [B][F][F] in t's dtype (fp32 accumulation)."""
    B, F, d = t.shape
    _check_3d("t", t, B, F, d)
    z = torch.empty((B, F, F), dtype=t.dtype, device=t.device)
    ctx = context(t.device)
    ctx.check(ctx.lib.dlrm_self_batched_mul(ctx.bind(), dtype_code(t.dtype), d, F, B, ptr(t), t.stride(0), ptr(z),
                                            z.stride(0)))
    return z


def rrule_self_batched_mul(t):
    """ChainRulesCore.rrule(self_batched_mul, x) (interact.jl:539-551): dT = T (Δ + Δᵀ), fp32."""
    B, F, d = t.shape
    z = self_batched_mul(t)

    def self_batched_mul_back(delta):
        _check_3d("Δ", delta, B, F, F)
        if delta.dtype != t.dtype:
            raise TypeError("self_batched_mul_back: Δ and T must share a dtype")
        dt = torch.empty((B, F, d), dtype=torch.float32, device=t.device)
        ctx = context(t.device)
        ctx.check(ctx.lib.dlrm_self_batched_mul_back(ctx.bind(), dtype_code(t.dtype), d, F, B, ptr(t), t.stride(0),
                                                     ptr(delta), delta.stride(0), ptr(dt), dt.stride(0)))
        return None, dt

    return z, self_batched_mul_back


def dot_interaction(x, ys):
    """dot_interaction(X, Ys) (interact.jl:503-517), Implementation 2: fast_vcat, the full batched
    Gram, its triangle, concat with X.  x: [B][d]; ys: [B][d + D*T] (rows 0:d reserved for x, as
    maplookup(PreallocationStrategy(d)) leaves them) -> [B][d + F(F-1)/2].  One MFMA launch: the
    composition is DotInteraction's forward with no padding (the same values)."""
    return DotInteraction(pad_to=1)(x, ys)


def rrule_dot_interaction(x, ys):
    """Zygote's pullback of dot_interaction: through concat, triangular_slice's rrule (upper
    triangle), self_batched_mul's (Δ + Δᵀ) and fast_vcat's -- dT = T S with S the symmetric
    zero-diagonal unpack of Δ's pair rows, dx = Δ_x + dT's x rows: dot_back's math, one launch."""
    return rrule(DotInteraction(pad_to=1), x, ys)


def fast_vcat(x, ys):
    """fast_vcat(x, ys) (interact.jl:271-281): copy x into the top rows reserved in ys.
    DotInteraction already fuses this copy into its kernel; this standalone form exists for
    API parity (a plain device copy)."""
    ys[:, : x.shape[1]].copy_(x)
    return ys
