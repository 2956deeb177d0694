"""Native codec ops (HIP gfx950 + C++ CPU): Count Sketch, deterministic top-k,
fused server/client state updates, DP clip+noise, download accounting and
on-device augmentation.  See ``csrc/`` for the kernels."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .._ext import ops as _ops
from .sketch import CSVec, make_hashes

__all__ = ["CSVec", "make_hashes", "topk_abs", "topk_dense", "momentum_ef", "sparse_apply",
           "dense_apply", "count_ge", "axpby", "l2norm", "clip_noise", "client_state", "client_tail",
           "zero_at", "scatter_dense", "augment_u8_nhwc", "augment_u8_nhwc_y", "account_round",
           "account_hist"]

ERROR_MODE = {"none": 0, "virtual": 1, "local": 2}


_TOPK_HINTS: dict = {}


def topk_hint(tag, device) -> Optional[torch.Tensor]:
    """Persistent per-site lower-bound hint for ``topk_abs`` (csrc/topk.hip:
    the previous call's threshold / 2 bounds the first histogram pass; the
    result never depends on it).  One per selection site (``tag``)."""
    device = torch.device(device)
    if device.type != "cuda":
        return None
    key = (tag, str(device))
    h = _TOPK_HINTS.get(key)
    if h is None:
        h = _TOPK_HINTS[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return h


def pack_topk(idx: torch.Tensor, vals: torch.Tensor, cmap: Optional[torch.Tensor] = None,
              m: int = 1) -> torch.Tensor:
    """int64 words idx << 32 | bits(vals) (``cmap``: idx are compact shard
    positions, global = cmap[idx // m] * m + idx % m) -- csrc/shard.hip."""
    return _ops().topk_pack(idx.contiguous(), vals.contiguous(), cmap, int(m))


def merge_packed(allp: torch.Tensor, nl: int, k: int):
    """(vals f32, idx int64) of nl packed k-lists (each ascending by index,
    disjoint) in ascending index order."""
    return _ops().merge_packed(allp.contiguous(), int(nl), int(k))


def gather_i64(src: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
    return _ops().gather_i64(src.contiguous(), pos.contiguous())


def zero_(t: torch.Tensor) -> None:
    """``t.zero_()`` as a native memset (recordable by a launch tape,
    parallel/tape.py); t contiguous."""
    _ops().zero_(t)


def topk_abs(x: torch.Tensor, k: int, hint: Optional[torch.Tensor] = None
             ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Deterministic magnitude top-k: (idx ascending int64, vals=x[idx]); ties -> lower index.
    ``hint``: a ``topk_hint`` tensor of the call site (speed only)."""
    return _ops().topk_abs(x.reshape(-1).contiguous(), int(k), hint)


def topk_dense(x: torch.Tensor, k: int) -> torch.Tensor:
    """Dense result of the reference ``_topk`` (utils.py:232-252): zeros except the top-k."""
    if x.dim() == 2:
        return torch.stack([topk_dense(row, k) for row in x])
    idx, vals = topk_abs(x, k)
    return _ops().scatter_dense(idx, vals, x.numel()).view_as(x)


def momentum_ef(V: torch.Tensor, E: Optional[torch.Tensor], G: torch.Tensor, rho: float,
                gscale: float = 1.0, error_type: str = "none") -> None:
    """V = rho*V + gscale*G ; virtual: E += V ; local: E = V."""
    _ops().momentum_ef(V, E, G, float(rho), float(gscale), ERROR_MODE[error_type])


def sparse_apply(w, idx, vals, lr, lr_vec=None, last_mod=None, round_idx: int = 0, step=None,
                 hist=None):
    """w[idx] -= lr * vals; last_mod[idx] = round where w changed.  ``step``
    (int32 [2] = lr bits, round) overrides lr/round from device memory (HIP
    graph replay); ``hist`` (int32, hist[r+1] = #{i: last_mod[i] == r}) is
    kept in step with the stamps."""
    _ops().sparse_apply(w, idx, vals, float(lr), lr_vec, last_mod, int(round_idx), step, hist)


def dense_apply(w, delta, lr, lr_vec=None, last_mod=None, round_idx: int = 0, step=None,
                hist=None):
    _ops().dense_apply(w, delta, float(lr), lr_vec, last_mod, int(round_idx), step, hist)


def account_hist(hist, meta, W: int, client_dl, client_ul, upload_per_client: float):
    """Round accounting from the change histogram: meta = int64 [last_seen (W) |
    clients (W)]; returns per-client download bytes 4 * #{i : last_mod[i] >=
    last_seen} and adds them (and the upload) to the running totals."""
    return _ops().account_hist(hist, meta, int(W), client_dl, client_ul, float(upload_per_client))


def count_ge(last_mod: torch.Tensor, thr: torch.Tensor) -> torch.Tensor:
    return _ops().count_ge(last_mod, thr)


def account_round(last_mod, meta, T: int, W: int, client_dl, client_ul, upload_per_client: float):
    """Fused round accounting (HIP): meta = int64 [thr (T) | inv (W) | clients (W)];
    returns per-client download bytes and adds them (and the upload) to the totals."""
    return _ops().account_round(last_mod, meta, int(T), int(W), client_dl, client_ul,
                                float(upload_per_client))


def axpby(out, a, alpha, b=None, beta=0.0):
    _ops().axpby(out, a, float(alpha), b, float(beta))


def l2norm(x: torch.Tensor) -> torch.Tensor:
    return _ops().l2norm(x.reshape(-1).contiguous())


def clip_noise(x, norm=None, clip=0.0, noise_std=0.0, seed=0, offset=0):
    _ops().clip_noise(x, norm, float(clip), float(noise_std), int(seed), int(offset))


def client_state(g, u=None, e=None, rho=0.0):
    _ops().client_state(g, u, e, float(rho))


def client_tail(g, w=None, wd=0.0, scale=1.0, u=None, e=None, rho=0.0):
    """t = scale (g + wd w); u = rho u + t (t = u); e += t; g = t when there is
    neither u nor e -- one pass (csrc/elementwise.hip client_tail_kernel)."""
    _ops().client_tail(g, w, float(wd), float(scale), u, e, float(rho))


def zero_at(idx, a=None, b=None, c=None):
    _ops().zero_at(a, b, c, idx)


def scatter_dense(idx, vals, n):
    return _ops().scatter_dense(idx, vals, int(n))


def augment_u8_nhwc(data, idx, pad, flip, mean, inv_std, seed, out_bf16=True, keys=None):
    return _ops().augment_u8_nhwc(data, idx, int(pad), bool(flip), mean, inv_std, int(seed),
                                  bool(out_bf16), keys)


def augment_u8_nhwc_y(data, idx, pad, flip, mean, inv_std, seed, out_bf16, keys, targets):
    """augment_u8_nhwc and the labels targets[idx] from one kernel (GPU)."""
    return _ops().augment_u8_nhwc_y(data, idx, int(pad), bool(flip), mean, inv_std, int(seed),
                                    bool(out_bf16), keys, targets)


# ------------------------------------------------------------ conv3x3 (MFMA)
def conv_weight_prep(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 [K, C, 3, 3] -> (bf16 [K, 3, 3, C], bf16 [C, 3, 3, K] spatially flipped)."""
    return _ops().conv_weight_prep(w)


def conv3x3_fwd(x, wf, relu: bool = False, mask=None, addend=None) -> torch.Tensor:
    """act(conv3x3(x, wf)) on NHWC bf16; epilogue: relu, y=0 where mask<=0, y+=addend."""
    return _ops().conv3x3_fwd(x, wf, bool(relu), mask, addend)


def conv3x3_wgrad(dy, x, splits: int = 0) -> torch.Tensor:
    """fp32 [K, C, 3, 3] weight gradient (deterministic split-K)."""
    return _ops().conv3x3_wgrad(dy, x, int(splits))


def relu_mask(gy, y) -> torch.Tensor:
    return _ops().relu_mask(gy, y)


def client_means(out, rows, slot, counts) -> None:
    """out[i, w] = mean of rows[i][e] over examples e with slot[e] == w (slot
    ascending), 0 where a client has no examples here; one native kernel."""
    _ops().client_means(out, list(rows), slot, counts)


__all__ += ["conv_weight_prep", "conv3x3_fwd", "conv3x3_wgrad", "relu_mask", "client_means"]
