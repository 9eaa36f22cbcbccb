"""Extract golden vectors for the DLRM hot path from the reference's PyTorch HDF5 files.

Test infrastructure only.  Run ONCE in the build container with the conda interpreter that
has h5py (the GPU box has no h5py and no /root/reference):

    /opt/conda/bin/python3.9 tests/golden/make_fixtures.py

Inputs  : /root/reference/ref/pytorch_reference_{single,multi}.hdf5  (read-only, data only)
Outputs : tests/golden/pytorch_reference_{single,multi}.npz + fixtures_meta.json

What is stored (all C row-major, PyTorch orientation; Julia reads the same bytes transposed,
see /root/reference/src/data/criteo.jl:464-560):
  emb            (T, N, D) f32   embedding tables before the step        (`emb_*`)
  idx            (T, B*L)  i64   0-based indices, sample-major            (`input_emb_*`)
  L              lookups per sample (1 = single, 10 = multi, sum pooling)
  mlp_bottom     (B, d)    f32   dense vector x                           (`mlp_bottom`)
  concatenated   (B, F, D) f32   [x | e_1 .. e_T] per sample              (`concatenated_result`)
  zflat          (B, P)    f32   strict lower triangle, PyTorch li/lj     (`zflat`)
  output_interaction (B, d+P) f32                                         (`output_interaction`)
  d_output_interaction (B, d+P) f32  dLoss/d(output_interaction), DERIVED in float64 from
                 the top MLP weights + labels (BCE mean) and validated below by reproducing
                 `update_top_*` and `update_emb_*` of the same file.
  upd_rows_t / upd_vals_t        touched rows of `update_emb_t` (untouched rows are asserted
                 bit-identical to `emb_t` here, so only touched rows are stored)
  lr             10.0  (src/validation.jl:23-24)

Dense half (the full training step), in pytorch_reference_{kind}_dense.npz:
  input_bot (B, 13) f32, labels (B,) f32, loss () f32, mlp_top (B,) f32
  bot_W{i} / bot_b{i}, top_W{i} / top_b{i}     MLP parameters before the step (layer i, Flux
                 orientation W[out][in]; PyTorch `bot_l.{i}` / `top_l.{i}`)
  upd_bot_W{i} / upd_bot_b{i}, upd_top_W{i} / upd_top_b{i}   after one Descent(10) step
                 (PyTorch `update_bot_{2i}` / `update_top_{2i}`, validation.jl:74-123)
"""
import json
import os
import sys

import h5py
import numpy as np

REF = "/root/reference/ref"
OUT = os.path.dirname(os.path.abspath(__file__))


def natural_tables(h, prefix):
    names = [k for k in h.keys() if k.startswith(prefix) and k[len(prefix):].isdigit()]
    return sorted(names, key=lambda k: int(k[len(prefix):]))


def mlp_forward(h, prefix, x, last_sigmoid):
    """Returns list of (pre, post) activations. PyTorch Linear: y = x W^T + b."""
    layers = sorted({k.split(".")[1] for k in h.keys() if k.startswith(prefix + ".")}, key=int)
    acts = [x]
    pres = []
    for li, l in enumerate(layers):
        W = h[f"{prefix}.{l}.weight"][()].astype(np.float64)
        b = h[f"{prefix}.{l}.bias"][()].astype(np.float64)
        z = acts[-1] @ W.T + b
        pres.append(z)
        last = li == len(layers) - 1
        if last and last_sigmoid:
            acts.append(1.0 / (1.0 + np.exp(-z)))
        else:
            acts.append(np.maximum(z, 0.0))
    return layers, pres, acts


def tri_pairs(F):
    # PyTorch DLRM li/lj order == Julia triangular_slice_kernel! order
    # (/root/reference/src/model/interact.jl:64-75): for i = 1..F-1, j = 0..i-1.
    return [(i, j) for i in range(1, F) for j in range(i)]


def process(kind):
    path = os.path.join(REF, f"pytorch_reference_{kind}.hdf5")
    h = h5py.File(path, "r")
    emb_names = natural_tables(h, "emb_")
    T = len(emb_names)
    emb = np.stack([h[n][()] for n in emb_names]).astype(np.float32)  # (T, N, D)
    _, N, D = emb.shape
    idx = np.stack([h[f"input_emb_{t}"][()] for t in range(T)]).astype(np.int64)
    labels = h["labels"][()].reshape(-1).astype(np.float64)
    B = labels.shape[0]
    L = idx.shape[1] // B
    assert idx.shape[1] == B * L
    x = h["mlp_bottom"][()].astype(np.float32)
    d = x.shape[1]
    F = T + 1
    P = F * (F - 1) // 2

    # --- forward restatement (float64) ---
    e = emb.astype(np.float64)[np.arange(T)[:, None], idx]  # (T, B*L, D)
    e = e.reshape(T, B, L, D).sum(axis=2)  # sum pooling, sample-major
    Tm = np.concatenate([x.astype(np.float64)[None], e], axis=0).transpose(1, 0, 2)  # (B,F,D)
    conc = h["concatenated_result"][()]
    err_conc = np.abs(Tm - conc).max()
    Z = Tm @ Tm.transpose(0, 2, 1)
    pairs = tri_pairs(F)
    li = np.array([p[0] for p in pairs])
    lj = np.array([p[1] for p in pairs])
    zflat = Z[:, li, lj]
    out = np.concatenate([x.astype(np.float64), zflat], axis=1)
    err_zflat = np.abs(zflat - h["zflat"][()]).max()
    err_out = np.abs(out - h["output_interaction"][()]).max()
    err_zpre = np.abs(Z - h["zpre"][()]).max()

    # --- top MLP + BCE to derive dLoss/dOut (float64) ---
    oi = h["output_interaction"][()].astype(np.float64)
    layers, pres, acts = mlp_forward(h, "top_l", oi, last_sigmoid=True)
    p = acts[-1].reshape(-1)
    err_top = np.abs(p - h["mlp_top"][()].reshape(-1)).max()
    loss = np.mean(-labels * np.log(p) - (1 - labels) * np.log(1 - p))
    err_loss = abs(loss - float(h["loss"][()]))
    g = ((p - labels) / B).reshape(-1, 1)  # dL/dlogit of last layer
    lr = 10.0
    top_grad_err = 0.0
    for li_, l in reversed(list(enumerate(layers))):
        W = h[f"top_l.{l}.weight"][()].astype(np.float64)
        gW = g.T @ acts[li_]
        gb = g.sum(axis=0)
        # PyTorch names the updated layers by Sequential index (0, 2, 4): li_*2
        upd = h[f"update_top_{2 * li_}.weight"][()].astype(np.float64)
        top_grad_err = max(top_grad_err, np.abs((W - lr * gW) - upd).max())
        updb = h[f"update_top_{2 * li_}.bias"][()].astype(np.float64)
        bb = h[f"top_l.{l}.bias"][()].astype(np.float64)
        top_grad_err = max(top_grad_err, np.abs((bb - lr * gb) - updb).max())
        g = g @ W
        if li_ > 0:
            g = g * (pres[li_ - 1] > 0)
    dout = g  # (B, d+P)

    # --- interaction backward + SGD restatement (interact.jl:415-489) ---
    dz = dout[:, d:]
    S = np.zeros((B, F, F))
    S[:, li, lj] = dz
    S[:, lj, li] = dz
    dT = S @ Tm  # (B, F, D)
    upd_err = 0.0
    upd_rows, upd_vals = [], []
    for t in range(T):
        grad = dT[:, t + 1, :]  # (B, D) pulled back through the sum pooling
        acc = np.zeros((N, D))
        np.add.at(acc, idx[t], np.repeat(grad, L, axis=0))
        new = e_t = emb[t].astype(np.float64) - lr * acc
        ref = h[f"update_emb_{t}"][()]
        upd_err = max(upd_err, np.abs(new - ref).max())
        rows = np.unique(idx[t])
        untouched = np.setdiff1d(np.arange(N), rows)
        assert np.array_equal(ref[untouched], emb[t][untouched]), "untouched rows changed"
        upd_rows.append(rows.astype(np.int64))
        upd_vals.append(ref[rows].astype(np.float32))
        del e_t

    arrays = dict(
        emb=emb, idx=idx, L=np.int64(L), lr=np.float32(lr),
        mlp_bottom=x, concatenated=conc.astype(np.float32),
        zflat=h["zflat"][()].astype(np.float32),
        output_interaction=h["output_interaction"][()].astype(np.float32),
        d_output_interaction=dout.astype(np.float32),
    )
    for t in range(T):
        arrays[f"upd_rows_{t}"] = upd_rows[t]
        arrays[f"upd_vals_{t}"] = upd_vals[t]
    np.savez_compressed(os.path.join(OUT, f"pytorch_reference_{kind}.npz"), **arrays)
    meta = dict(
        T=T, N=N, D=D, B=B, L=L, d=d, F=F, P=P,
        unique_rows=[int(len(r)) for r in upd_rows],
        err_concatenated=float(err_conc), err_zpre=float(err_zpre),
        err_zflat=float(err_zflat), err_output_interaction=float(err_out),
        err_mlp_top=float(err_top), err_loss=float(err_loss),
        err_update_top=float(top_grad_err), err_update_emb=float(upd_err),
    )
    print(kind, json.dumps(meta))
    for k in ("err_concatenated", "err_zflat", "err_output_interaction", "err_update_emb"):
        assert meta[k] < 1e-5, (k, meta[k])
    return meta


def process_dense(kind):
    h = h5py.File(os.path.join(REF, f"pytorch_reference_{kind}.hdf5"), "r")
    arrays = dict(input_bot=h["input_bot"][()].astype(np.float32),
                  labels=h["labels"][()].reshape(-1).astype(np.float32),
                  loss=np.float32(h["loss"][()]), mlp_top=h["mlp_top"][()].reshape(-1).astype(np.float32))
    for short, prefix, upd in (("bot", "bot_l", "update_bot"), ("top", "top_l", "update_top")):
        layers = sorted({k.split(".")[1] for k in h.keys() if k.startswith(prefix + ".")}, key=int)
        for i, l in enumerate(layers):
            for kk, suffix in (("W", "weight"), ("b", "bias")):
                arrays[f"{short}_{kk}{i}"] = h[f"{prefix}.{l}.{suffix}"][()].astype(np.float32)
                arrays[f"upd_{short}_{kk}{i}"] = h[f"{upd}_{2 * i}.{suffix}"][()].astype(np.float32)
    # the bottom MLP restated reproduces the stored mlp_bottom (the hot path's x)
    _, _, acts = mlp_forward(h, "bot_l", arrays["input_bot"].astype(np.float64), last_sigmoid=False)
    err = float(np.abs(acts[-1] - h["mlp_bottom"][()]).max())
    assert err < 1e-5, err
    np.savez_compressed(os.path.join(OUT, f"pytorch_reference_{kind}_dense.npz"), **arrays)
    return err


if __name__ == "__main__":
    meta = {k: process(k) for k in ("single", "multi")}
    for k in ("single", "multi"):
        meta[k]["err_mlp_bottom"] = process_dense(k)
    with open(os.path.join(OUT, "fixtures_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    sys.exit(0)
