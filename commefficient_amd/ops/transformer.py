"""GPT-2 transformer forward/backward on the native block-junction kernels.

The reference trains HF ``GPT2DoubleHeadsModel`` (/root/reference/CommEfficient/
gpt2_train.py:4-6,262-273), whose pre-LN block runs, per sublayer, separate
kernels for the residual add, dropout, LayerNorm (forward and three backward
kernels), GELU and the bias-gradient reductions.  ``gpt2_hidden`` computes the
same function over the same HF parameters with one native kernel per
junction (csrc/transformer.hip):

    y0 = LN1_0(drop(wte[ids] + wpe[pos] + wte[tt]))              _EmbedLN
    per block:
      qkv = y @ W_attn + b_attn                                     _Linear (bias grad native)
      o   = SDPA(q, k, v, causal, attn dropout)                     fused attention kernels
      h, y = h + drop(o @ W_proj + b_proj), LN2(h)                  _ResidLN
      f   = gelu_tanh(y @ W_fc + b_fc)                              _FcGelu
      h, y = h + drop(f @ W_mproj + b_mproj), LN1_next|LN_f(h)      _ResidLN

The forward and input-gradient GEMMs run on the native MFMA kernels of
csrc/gemm.hip (``_mm`` / ``_mm_t``; COMMEFF_GEMM=blas: hipBLASLt), the
weight gradients on csrc/gemm_tn.hip.  Backward of each junction is one
kernel (LN backward + residual gradient + dropout backward + column partials
of dgamma/dbeta/dbias) plus one fixed-order column reduction, so every
gradient is deterministic for a given dropout seed.  Dropout masks are a
32-bit counter hash of (seed, element) recomputed in backward (no mask
tensors).  Seeds come from a host-side counter per model: no device syncs.

On CPU the same Functions run on the PyTorch reference implementations below
(``_ref_*``), which mirror the kernels' bf16 rounding points; they are the
numerics oracle of tests/test_transformer.py.
"""
from __future__ import annotations

import os

from contextlib import contextmanager
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from .._ext import ops as _ops
from . import lanes as _lanes

_M32 = 0xFFFFFFFF


# ------------------------------------------------------------- references
def _mix32(x: torch.Tensor) -> torch.Tensor:
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def drop_keep(numel: int, seed: int, p: float, device=None) -> torch.Tensor:
    """The kernels' dropout keep-mask of ``numel`` consecutive elements."""
    return keep_at(torch.arange(numel, dtype=torch.int64, device=device), seed, p)


def keep_at(idx: torch.Tensor, seed: int, p: float) -> torch.Tensor:
    """The kernels' dropout keep-mask at element indices ``idx`` (int64)."""
    hi = _mix32(((idx >> 32) + (seed & _M32)) & _M32)
    h = _mix32((idx & _M32) ^ hi)
    thresh = min(int(p * 4294967296.0), _M32) if p > 0 else 0
    return h >= thresh


def _bf(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).float()


def _ref_resid_ln_fwd(x, p, bias, gamma, beta, p_drop, seed, eps, want_h):
    M, H = x.shape
    v = x.float()
    scale = 1.0 / (1.0 - p_drop) if p_drop > 0 else 1.0
    keep = drop_keep(M * H, seed, p_drop, x.device).view(M, H) if p_drop > 0 else None
    if p is not None:
        t = _bf(p.float() + (bias.float() if bias is not None else 0.0))
        if keep is not None:
            t = torch.where(keep, _bf(t * scale), torch.zeros_like(t))
        v = _bf(v + t)
    elif keep is not None:
        v = torch.where(keep, _bf(v * scale), torch.zeros_like(v))
    mean = v.mean(1)
    rstd = torch.rsqrt(((v - mean[:, None]) ** 2).mean(1) + eps)
    y = ((v - mean[:, None]) * rstd[:, None] * gamma.float() + beta.float()).to(torch.bfloat16)
    h = v.to(torch.bfloat16) if want_h else x.new_empty(0)
    return h, y, mean, rstd


def _ref_resid_ln_bwd(gy, gh, h, mean, rstd, gamma, p_drop, seed, want_dp, want_dbias,
                      sgamma=None, sbeta=None, sbias=None):
    M, H = h.shape
    xh = (h.float() - mean[:, None]) * rstd[:, None]
    dy = gy.float()
    dx = dy * gamma.float()
    s1 = dx.mean(1, keepdim=True)
    s2 = (dx * xh).mean(1, keepdim=True)
    dh = rstd[:, None] * (dx - s1 - xh * s2)
    if gh is not None:
        dh = dh + gh.float()
    dh = _bf(dh)
    dgamma = (dy * xh).sum(0).to(gamma.dtype)
    dbeta = dy.sum(0).to(gamma.dtype)
    dp = h.new_empty(0)
    dbias = gamma.new_empty(0) if not want_dbias else torch.zeros_like(gamma)
    if want_dp:
        dpf = dh
        if p_drop > 0:
            keep = drop_keep(M * H, seed, p_drop, h.device).view(M, H)
            dpf = torch.where(keep, _bf(dh / (1.0 - p_drop)), torch.zeros_like(dh))
        dp = dpf.to(torch.bfloat16)
        if want_dbias:
            dbias = dpf.sum(0).to(gamma.dtype)
            if sbias is not None:
                sbias.add_(dpf.sum(0))
                dbias = gamma.new_empty(0)
    if sgamma is not None:
        sgamma.add_((dy * xh).sum(0))
        dgamma = gamma.new_empty(0)
    if sbeta is not None:
        sbeta.add_(dy.sum(0))
        dbeta = gamma.new_empty(0)
    return dh.to(torch.bfloat16), dp, dgamma, dbeta, dbias


_GK = 0.7978845608028654
_GC = 0.044715


def _ref_bias_gelu_fwd(u, b):
    x = _bf(u.float() + b.float())
    return (0.5 * x * (1.0 + torch.tanh(_GK * (x + _GC * x ** 3)))).to(torch.bfloat16)


def _ref_bias_act_bwd(gf, u, b, gelu, sbias=None):
    g = gf.float()
    du = gf.new_empty(0)
    if gelu:
        x = _bf(u.float() + b.float())
        t = torch.tanh(_GK * (x + _GC * x ** 3))
        g = _bf(g * (0.5 * (1.0 + t) + 0.5 * x * (1.0 - t * t) * _GK * (1.0 + 3.0 * _GC * x * x)))
        du = g.to(torch.bfloat16)
    if sbias is not None:
        sbias.add_(g.sum(0))
        return du, b.new_empty(0)
    return du, g.sum(0).to(b.dtype)


class _Impl:
    """torch.ops.commeff on HIP tensors, the references on CPU."""

    @staticmethod
    def resid_ln_fwd(x, *a):
        return (_ops().resid_ln_fwd if x.is_cuda else _ref_resid_ln_fwd)(x, *a)

    @staticmethod
    def resid_ln_bwd(gy, *a):
        return (_ops().resid_ln_bwd if gy.is_cuda else _ref_resid_ln_bwd)(gy, *a)

    @staticmethod
    def bias_gelu_fwd(u, b):
        return (_ops().bias_gelu_fwd if u.is_cuda else _ref_bias_gelu_fwd)(u, b)

    @staticmethod
    def bias_act_bwd(gf, u, b, gelu, sbias=None):
        return (_ops().bias_act_bwd if gf.is_cuda else _ref_bias_act_bwd)(gf, u, b, gelu, sbias)


def _c(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    return None if t is None else t.contiguous()


# ------------------------------------------------------- gradient sinks
# With the bf16 model replica (parallel/flat.py make_bf16_shadow) the weight
# gradients would be produced in bf16, concatenated into one bf16 buffer and
# added to the fp32 flat gradient (one 124M-element cat + one add per pass).
# Inside ``grad_sinks({id(param): fp32 view of the flat gradient})`` the
# junctions instead accumulate their weight / bias / LayerNorm gradients
# straight into those fp32 views (GEMM with an fp32 C and beta = 1; the
# column sums add in fp32) and return no gradient for them.
_SINKS: list = [None]


@contextmanager
def grad_sinks(mapping: Optional[Dict[int, torch.Tensor]]):
    prev = _SINKS[0]
    _SINKS[0] = mapping
    try:
        yield
    finally:
        _SINKS[0] = prev


def _sink(p: torch.Tensor) -> Optional[torch.Tensor]:
    m = _SINKS[0]
    return None if m is None else m.get(id(p))


def _sinks(*params):
    return tuple(_sink(p) for p in params)


# forward / input-gradient / weight-gradient GEMMs on the native MFMA kernels
# (csrc/gemm.hip, gemm_tn.hip); COMMEFF_GEMM=blas: hipBLASLt (torch.mm)
_GEMM = {"native": os.environ.get("COMMEFF_GEMM", "native") == "native"}
_WGRAD_GEMM = _GEMM


def _native_mm_ok(a: torch.Tensor, b: torch.Tensor, n: int) -> bool:
    # (bf16 CUDA operands are checked by the op itself; this keeps the shapes
    # it serves: one Python test per call instead of a dozen attribute reads)
    sa, sb = a.stride(), b.stride()
    return (_GEMM["native"] and a.is_cuda and n % 64 == 0 and a.shape[1] % 64 == 0
            and sa[1] == 1 and sb[1] == 1 and sa[0] % 8 == 0 and sb[0] % 8 == 0
            and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0)


def _mm(a: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """a @ W (+ bias): the HF Conv1D forward, W [in, out] (native NN GEMM, the
    bf16 bias added in its epilogue)."""
    if _native_mm_ok(a, W, W.shape[1]):
        return _ops().mm_nn(a, W, bias)
    return torch.addmm(bias, a, W) if bias is not None else torch.mm(a, W)


def _mm_t(dy: torch.Tensor, W: torch.Tensor) -> torch.Tensor:
    """dy @ W^T: the input gradient of a Conv1D, W [in, out] (native NT GEMM)."""
    if _native_mm_ok(dy, W, W.shape[0]):
        return _ops().mm_nt(dy, W)
    return torch.mm(dy, W.t())


def _gemm_tn_ok(sink: torch.Tensor, at: torch.Tensor, b: torch.Tensor) -> bool:
    """csrc/gemm_tn.hip serves sink [M, N] += at^T b: bf16 [T, M] / [T, N]
    operands with unit column stride, M and N multiples of 256 (M also when
    at's rows hold the 8-column chunk past M: the padded LM-head gradient)."""
    M = at.shape[1] if at.dim() == 2 else 0
    return (_WGRAD_GEMM["native"] and sink.dtype == torch.float32 and sink.dim() == 2
            and sink.stride(1) == 1 and at.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
            and at.dim() == 2 and b.dim() == 2 and at.stride(1) == 1 and b.stride(1) == 1
            and (M % 256 == 0 or at.stride(0) >= -(-M // 8) * 8) and b.shape[1] % 256 == 0
            and at.stride(0) % 8 == 0 and b.stride(0) % 8 == 0 and sink.stride(0) % 4 == 0
            and at.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0 and sink.data_ptr() % 16 == 0)


def _acc_mm(sink: torch.Tensor, a: torch.Tensor, b: torch.Tensor, blas: bool = False) -> None:
    """sink (fp32) += a @ b (bf16 operands, fp32 accumulation and output).
    The weight gradients (a = X^T, a view of the token rows) run on the
    native split-K TN GEMM (csrc/gemm_tn.hip) when the shapes fit, else (or
    ``blas``) on hipBLASLt (COMMEFF_GEMM=blas: always)."""
    if sink.is_cuda:
        if not blas and _gemm_tn_ok(sink, a.t(), b):
            _ops().gemm_tn_acc(sink, a.t(), b)
            return
        torch.addmm(sink, a, b, out_dtype=torch.float32, out=sink)
    else:
        sink.add_(a.float() @ b.float())


# Weight-gradient GEMMs into the sinks run on the side lane (ops/lanes.py):
# they have few output tiles (768 x 768 .. 768 x 3072 over K = tokens: 36-144
# tiles of 128 x 128 on 256 CUs) and nothing in the backward waits for them,
# so they overlap the input-gradient GEMMs, attention backward and junction
# kernels of the layers below.  ``join_wgrad_stream()`` orders the main
# stream after them before the flat gradient is read.
_SIDE: dict = {"enabled": True}


def set_wgrad_stream(enabled: bool) -> None:
    _SIDE["enabled"] = bool(enabled)


def join_wgrad_stream() -> None:
    _lanes.join()


_ATTN = {"enabled": True}


def set_fused_attention(enabled: bool) -> None:
    _ATTN["enabled"] = bool(enabled)


# The junction backward's column sums (LayerNorm dgamma / dbeta, the branch
# bias gradients) go to the same side stream when all their outputs are fp32
# sinks: ~40 us each of latency-bound reductions that otherwise sit in the
# input-gradient chain behind the side stream's GEMM blocks (1.9 ms per GPT-2
# round, profiles/r4_gpt2_native_gemm_round_kernels.txt).
_COLSUM_SIDE = True


def _colsum_deferred(t: torch.Tensor, *sinks) -> bool:
    return (_COLSUM_SIDE and _SIDE["enabled"] and t.is_cuda
            and all(x is not None for x in sinks))


def _side_colsum(part: torch.Tensor, q: int, sinks) -> None:
    """sinks[i] += column sums of the block partials ``part`` (quantity i),
    on the weight-gradient side stream after the producing kernel."""
    with _lanes.fork(part):
        _ops().colsum_into(part, q, *sinks)


def _wgrad(sink, a, b, blas: bool = False):
    if sink is None:
        return torch.mm(a, b)
    if sink.is_cuda and _SIDE["enabled"]:
        with _lanes.fork(a, b):  # (the operands stay referenced until the join)
            _acc_mm(sink, a, b, blas)
        return None
    _acc_mm(sink, a, b, blas)
    return None


# ---------------------------------------------------------------- autograd
_EMB_WS: Dict = {}  # (device, V, H) -> the embedding backward's fixed-point workspace


def _emb_ws(device, V: int, H: int):
    key = (str(device), V, H)
    ws = _EMB_WS.get(key)
    if ws is None:
        # zero once; every backward leaves the rows it touched zeroed again
        ws = (torch.zeros(V * H, dtype=torch.int64, device=device),
              torch.zeros(V * H, dtype=torch.float32, device=device),  # out-of-range spill
              torch.zeros(V, dtype=torch.int32, device=device),
              torch.zeros(V + 1, dtype=torch.int32, device=device))
        _EMB_WS[key] = ws
    return ws


class _Embed(torch.autograd.Function):
    """e = wte[ids] + wpe[pos] (+ wte[token types]) on the real token rows
    (csrc/embed.hip): one gather-add kernel forward; backward scatters the row
    gradients into the token and position tables' fp32 gradients with
    fixed-point integer atomics -- order-independent, hence deterministic,
    without PyTorch's sort + sum_and_scatter (HF GPT2Model.forward,
    gpt2_train.py:55-99)."""

    @staticmethod
    def forward(ctx, wte, wpe, ids, tt, tok, L):
        out = _ops().embed_fwd(ids, tt, tok, L, wte, wpe)
        ctx.save_for_backward(ids, tt, tok)
        ctx.L = L
        ctx.params = (wte, wpe)
        ctx.sinks = (_sink(wte), _sink(wpe))
        return out

    @staticmethod
    def backward(ctx, de):
        ids, tt, tok = ctx.saved_tensors
        de = de.to(torch.bfloat16).contiguous()
        grads = []
        for i, (w, sink) in enumerate(zip(ctx.params, ctx.sinks)):
            if not ctx.needs_input_grad[i]:
                grads.append(None)
                continue
            V, H = w.shape
            dst = sink if sink is not None else torch.zeros(V, H, dtype=torch.float32, device=de.device)
            acc, spill, cnt, lst = _emb_ws(de.device, V, H)
            _ops().embed_bwd(de, ids, tt, tok, ctx.L, i == 1, acc, spill, cnt, lst, dst)
            grads.append(None if sink is not None else dst.to(w.dtype))
        return grads[0], grads[1], None, None, None, None


def _embed_native_ok(tr, ids) -> bool:
    wte, wpe = tr.wte.weight, tr.wpe.weight
    return (ids.is_cuda and wte.dtype == torch.bfloat16 and wpe.dtype == torch.bfloat16
            and wte.is_contiguous() and wpe.is_contiguous() and ids.dtype == torch.int64)


class _EmbedLN(torch.autograd.Function):
    """h = drop(x); y = LN(h)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, p_drop, seed, eps):
        h, y, mean, rstd = _Impl.resid_ln_fwd(x, None, None, gamma, beta, p_drop, seed, eps, True)
        ctx.save_for_backward(h, mean, rstd, gamma)
        ctx.cfg = (p_drop, seed)
        ctx.sinks = _sinks(gamma, beta)
        return h, y

    @staticmethod
    def backward(ctx, gh, gy):
        h, mean, rstd, gamma = ctx.saved_tensors
        p_drop, seed = ctx.cfg
        sg, sb = ctx.sinks
        gy = torch.zeros_like(h) if gy is None else gy.contiguous()
        if _colsum_deferred(gy, sg, sb):
            _, dx, part = _ops().resid_ln_bwd_part(gy, _c(gh), h, mean, rstd, gamma, p_drop, seed, True)
            _side_colsum(part, 3, (sg, sb, None))
            return dx, None, None, None, None, None
        _, dx, dgamma, dbeta, _ = _Impl.resid_ln_bwd(gy, _c(gh), h, mean, rstd, gamma, p_drop,
                                                     seed, True, False, sg, sb, None)
        return (dx, None if sg is not None else dgamma, None if sb is not None else dbeta,
                None, None, None)


class _ResidLN(torch.autograd.Function):
    """p = o @ W; h = x + drop(p + b); y = LN(h)."""

    @staticmethod
    def forward(ctx, x, o, W, b, gamma, beta, p_drop, seed, eps):
        p = _mm(o, W)
        h, y, mean, rstd = _Impl.resid_ln_fwd(x, p, b, gamma, beta, p_drop, seed, eps, True)
        ctx.save_for_backward(o, W, h, mean, rstd, gamma)
        ctx.cfg = (p_drop, seed)
        ctx.sinks = _sinks(W, b, gamma, beta)
        return h, y

    @staticmethod
    def backward(ctx, gh, gy):
        o, W, h, mean, rstd, gamma = ctx.saved_tensors
        p_drop, seed = ctx.cfg
        sW, sb, sg, sbe = ctx.sinks
        gy = torch.zeros_like(h) if gy is None else gy.contiguous()
        if _colsum_deferred(gy, sg, sbe, sb):
            dh, dp, part = _ops().resid_ln_bwd_part(gy, _c(gh), h, mean, rstd, gamma, p_drop, seed, True)
            _side_colsum(part, 3, (sg, sbe, sb))
            dgamma = dbeta = dbias = None
        else:
            dh, dp, dgamma, dbeta, dbias = _Impl.resid_ln_bwd(gy, _c(gh), h, mean, rstd, gamma,
                                                              p_drop, seed, True, True, sg, sbe, sb)
        do = _mm_t(dp, W) if ctx.needs_input_grad[1] else None
        dW = _wgrad(sW, o.t(), dp) if ctx.needs_input_grad[2] else None
        return (dh, do, dW, None if sb is not None else dbias,
                None if sg is not None else dgamma, None if sbe is not None else dbeta,
                None, None, None)


class _FcGelu(torch.autograd.Function):
    """f = gelu_tanh(a @ W + b)."""

    @staticmethod
    def forward(ctx, a, W, b):
        u = _mm(a, W)
        f = _Impl.bias_gelu_fwd(u, b)
        ctx.save_for_backward(a, W, u, b)
        ctx.sinks = _sinks(W, b)
        return f

    @staticmethod
    def backward(ctx, gf):
        a, W, u, b = ctx.saved_tensors
        sW, sb = ctx.sinks
        gf = gf.contiguous()
        if _colsum_deferred(gf, sb) and gf.shape[0] > 0:
            du, part = _ops().bias_act_bwd_part(gf, u, b, True)
            _side_colsum(part, 1, (sb, None, None))
            db = None
        else:
            du, db = _Impl.bias_act_bwd(gf, u, b, True, sb)
        da = _mm_t(du, W) if ctx.needs_input_grad[0] else None
        dW = _wgrad(sW, a.t(), du) if ctx.needs_input_grad[1] else None
        return da, dW, None if sb is not None else db


class _Linear(torch.autograd.Function):
    """y = a @ W + b (bias in the GEMM epilogue forward, native column sum backward)."""

    @staticmethod
    def forward(ctx, a, W, b):
        ctx.save_for_backward(a, W, b)
        ctx.sinks = _sinks(W, b)
        return _mm(a, W, b)

    @staticmethod
    def backward(ctx, gy):
        a, W, b = ctx.saved_tensors
        sW, sb = ctx.sinks
        gy = gy.contiguous()
        if _colsum_deferred(gy, sb) and gy.shape[0] > 0:
            _, part = _ops().bias_act_bwd_part(gy, None, b, False)
            _side_colsum(part, 1, (sb, None, None))
            db = None
        else:
            _, db = _Impl.bias_act_bwd(gy, None, b, False, sb)
        da = _mm_t(gy, W) if ctx.needs_input_grad[0] else None
        dW = _wgrad(sW, a.t(), gy) if ctx.needs_input_grad[1] else None
        return da, dW, None if sb is not None else db


class _LMHead(torch.autograd.Function):
    """logits = h W^T of the tied LM head, W [V, H] bf16 (V = 50,257: no tile
    multiple).  Forward: the native NT GEMM with in-kernel N-edge masking (W's
    rows past V load the zero page, chunks past V are not stored) into a bf16
    buffer whose rows are padded to a multiple of 8 columns; the logits are a
    [T, V] view of it, which the native cross-entropy reads and whose gradient
    it writes in the same padded layout (pad columns 0).  Backward: dW from
    that gradient straight into the tied weight's fp32 sink on the
    weight-gradient side lane (the native TN GEMM with its M = V edge tile;
    COMMEFF_LM_DW=blas: hipBLASLt's fp32-output GEMM), dh = g W (K = 50,257, only
    T x H outputs) on the native split-K NN GEMM (``mm_nn_splitk``).  No padded copies of W or of the gradient,
    no bf16 dW + accumulation pass (HF's lm_head on hipBLASLt; reference
    model: gpt2_train.py:262-273)."""

    @staticmethod
    def forward(ctx, h, W):
        V = W.shape[0]
        buf = torch.empty(h.shape[0], -(-V // 8) * 8, dtype=torch.bfloat16, device=h.device)
        out = buf[:, :V]
        _ops().mm_nt(h, W, None, out)
        ctx.save_for_backward(h, W)
        ctx.sink = _sink(W)
        return out

    @staticmethod
    def backward(ctx, g):
        h, W = ctx.saved_tensors
        g = g.to(torch.bfloat16)
        if g.stride(1) != 1:
            g = g.contiguous()
        dh = None
        if ctx.needs_input_grad[0]:
            # split-K native NN GEMM (K = V, only T x H outputs; the K tail in its
            # reduction), COMMEFF_LM_DH=blas: hipBLASLt
            dh = (_ops().mm_nn_splitk(g, W) if _LM_DH_NATIVE and g.stride(0) % 8 == 0 and W.shape[1] % 64 == 0
                  else torch.mm(g, W))
        dW = None
        if ctx.needs_input_grad[1]:
            if ctx.sink is not None:
                # (in isolation hipBLASLt's fp32-output GEMM is faster: 120 vs
                # 150 us for the TN GEMM's 2,358 short-K (T = 640) tiles,
                # scripts/dev/bench_lm_bwd.py; on the side lane the round time
                # is the same: 13.35 / 13.72 vs 13.39 / 13.59 ms)
                _wgrad(ctx.sink, g.t(), h, blas=not _LM_DW_TN)
            else:
                dW = torch.mm(g.t(), h, out_dtype=torch.float32).to(W.dtype)
        return dh, dW


# The native LM head (default; COMMEFF_LM_HEAD=blas: HF's lm_head module on
# hipBLASLt).  Round 5's version copied W and the gradient into tile-padded
# buffers every call and was slower than hipBLASLt (699 vs 377 us isolated).
_LM_NATIVE = os.environ.get("COMMEFF_LM_HEAD", "native") == "native"
_LM_DW_TN = os.environ.get("COMMEFF_LM_DW", "tn") == "tn"
_LM_DH_NATIVE = os.environ.get("COMMEFF_LM_DH", "native") == "native"


def lm_head(m, h: torch.Tensor) -> torch.Tensor:
    """The (tied) LM head of an HF double-heads model on h [..., H]: native
    (``_LMHead``) for bf16 CUDA operands, else the module itself."""
    W = m.lm_head.weight
    H = h.shape[-1]
    h2 = h.reshape(-1, H)
    if (_LM_NATIVE and _GEMM["native"] and h.is_cuda and h.dtype == torch.bfloat16 and W.dtype == torch.bfloat16
            and getattr(m.lm_head, "bias", None) is None and H % 64 == 0 and W.shape[0] >= 64
            and W.is_contiguous() and W.data_ptr() % 16 == 0
            and h2.is_contiguous() and h2.data_ptr() % 16 == 0):
        return _LMHead.apply(h2, W).view(h.shape[:-1] + (W.shape[0],))
    return m.lm_head(h)


# ------------------------------------------------------------------ model
class _Seeds:
    """Host-side dropout seed stream (64-bit LCG), one per model."""

    def __init__(self, base: int):
        self.s = (int(base) * 0x9E3779B97F4A7C15 + 1) & 0xFFFFFFFFFFFFFFFF

    def next(self) -> int:
        self.s = (self.s * 6364136223846793005 + 1442695040888963407) & 0xFFFFFFFFFFFFFFFF
        return self.s >> 32


def native_ok(tr, input_ids: torch.Tensor) -> bool:
    """The native path covers HF GPT2Model blocks as configured for GPT-2
    (pre-LN, tanh GELU, default attention scaling) with bf16 weights."""
    cfg = getattr(tr, "config", None)
    if cfg is None or getattr(cfg, "model_type", "") != "gpt2" or not hasattr(tr, "h"):
        return False
    from .nn import stock_active
    if stock_active():  # torch.func transforms: the HF modules
        return False
    H = cfg.n_embd
    return (tr.wte.weight.dtype == torch.bfloat16
            and (not input_ids.is_cuda or _native_hidden_size(H))
            and cfg.activation_function in ("gelu_new", "gelu_pytorch_tanh")
            and (cfg.n_inner is None or cfg.n_inner == 4 * H)
            and cfg.scale_attn_weights and not cfg.scale_attn_by_inverse_layer_idx
            and not cfg.reorder_and_upcast_attn and not cfg.add_cross_attention
            and H % cfg.n_head == 0)


def _native_hidden_size(H: int) -> bool:
    return H % 256 == 0 and 1 <= H // 256 <= 6


def _ref_pad_rows(src, inv, rows):
    if inv is None:
        return src.clone()
    inv = inv.long()
    out = src.new_zeros(rows, src.shape[1])
    real = inv >= 0
    out[real] = src[inv[real]]
    return out


def _ref_heads_to_rows(srcs, tok, Mr):
    N, nh, L, hd = srcs[0].shape
    rows = torch.cat([s.permute(0, 2, 1, 3).reshape(N * L, nh * hd) for s in srcs], dim=1)
    return rows if tok is None else rows.index_select(0, tok.long())


def _pad_rows(src, inv, rows):
    return (_ops().pad_rows if src.is_cuda else _ref_pad_rows)(src, inv, rows)


def _heads_to_rows(srcs, tok, Mr):
    return (_ops().heads_to_rows if srcs[0].is_cuda else _ref_heads_to_rows)(srcs, tok, Mr)


def _heads(rows: torch.Tensor, N: int, L: int, nh: int):
    """[N*L, H] padded rows -> the [N, nh, L, hd] head view (HF's layout)."""
    H = rows.shape[1]
    return rows.view(N, L, nh, H // nh).transpose(1, 2)


class _RowsToHeads(torch.autograd.Function):
    """qkv token rows [Mr, 3H] -> q, k, v [N, nh, L, hd] views of ONE padded
    [N*L, 3H] buffer (zero at pads); backward gathers dq, dk, dv straight
    into the token rows of dqkv (no concatenation)."""

    @staticmethod
    def forward(ctx, qkv, tok, inv, N, L, nh):
        ctx.save_for_backward(tok)
        ctx.Mr = qkv.shape[0]
        H = qkv.shape[1] // 3
        pad = _pad_rows(qkv, inv, N * L)
        return tuple(_heads(t, N, L, nh) for t in pad.split(H, dim=1))

    @staticmethod
    def backward(ctx, dq, dk, dv):
        (tok,) = ctx.saved_tensors
        like = next(g for g in (dq, dk, dv) if g is not None)
        gs = [g if g is not None else torch.zeros_like(like) for g in (dq, dk, dv)]
        return _heads_to_rows(gs, tok, ctx.Mr), None, None, None, None, None


class _HeadsToRows(torch.autograd.Function):
    """attention output [N, nh, L, hd] (any strides) -> token rows [Mr, H]."""

    @staticmethod
    def forward(ctx, o, tok, inv, Mr):
        ctx.save_for_backward(inv)
        ctx.dims = (o.shape[0], o.shape[1], o.shape[2])
        return _heads_to_rows([o], tok, Mr)

    @staticmethod
    def backward(ctx, g):
        (inv,) = ctx.saved_tensors
        N, nh, L = ctx.dims
        return _heads(_pad_rows(g.contiguous(), inv, N * L), N, L, nh), None, None, None


class _ToPadded(torch.autograd.Function):
    """[Mr, K] token rows -> [rows, K] with the rows at ``tok`` (others 0)."""

    @staticmethod
    def forward(ctx, x, tok, rows):
        ctx.save_for_backward(tok)
        return x.new_zeros(rows, x.shape[1]).index_copy_(0, tok.long(), x)

    @staticmethod
    def backward(ctx, g):
        (tok,) = ctx.saved_tensors
        return g.index_select(0, tok.long()), None, None


def real_token_index(lengths: torch.Tensor, L: int, device):
    """(tok, inv, start, len) for host-side sequence lengths: tok = flat
    positions n*L + t (t < lengths[n]) of the real tokens, inv = token row of
    every padded position or -1, start / len = each sequence's token rows;
    built on the host (their sizes are known without a sync), one int32 H2D
    copy."""
    import numpy as np
    ln = lengths.reshape(-1).numpy().astype(np.int64)
    if ln.size == 0 or int(ln.min()) < 0 or int(ln.max()) > L:
        return None
    Mr = int(ln.sum())
    cs = np.concatenate([[0], np.cumsum(ln)[:-1]])
    starts = np.repeat(np.arange(ln.size, dtype=np.int64) * L - cs, ln)
    tok = starts + np.arange(Mr, dtype=np.int64)
    inv = np.full(ln.size * L, -1, dtype=np.int64)
    inv[tok] = np.arange(Mr)
    both = np.concatenate([tok, inv, cs, ln]).astype(np.int32)
    if torch.device(device).type == "cuda":
        from ..parallel.dist import h2d
        both = h2d(both, device)
    else:
        both = torch.from_numpy(both)
    n = ln.size
    return both[:Mr], both[Mr:Mr + n * L], both[Mr + n * L:Mr + n * L + n], both[Mr + n * L + n:]


# ------------------------------------------------------- fused attention
# csrc/attention.hip: sequences of <= 128 tokens run the all-in-LDS kernels,
# longer ones (up to GPT-2's 1024 positions) the flash-style kernels; both
# draw dropout from the same (sequence, head, i, j) hash
ATTN_MAX_LEN = 1024
ATTN_SHORT_LEN = 128
_DS = 1024  # dropout index stride (csrc/attention.hip DS)


def attn_lse_ld(max_len: int) -> int:
    """LSE row stride (and kernel family) for sequences of <= max_len tokens."""
    return 128 if max_len <= ATTN_SHORT_LEN else (max_len + 127) // 128 * 128


def _ref_attn(qkv, start, lens, nh, p, seed, max_len=ATTN_SHORT_LEN):
    """fp32 reference of csrc/attention.hip over unpadded token rows (same
    dropout hash; P_drop rounded to bf16 as the kernel feeds it to the MFMA)."""
    M, H3 = qkv.shape
    H = H3 // 3
    hd = H // nh
    ld = attn_lse_ld(max_len)
    o = qkv.new_zeros(M, H, dtype=torch.float32)
    lse = torch.zeros(start.numel() * nh * ld, dtype=torch.float32, device=qkv.device)
    for n in range(start.numel()):
        s0, L = int(start[n]), int(lens[n])
        if L == 0:
            continue
        x = qkv[s0:s0 + L].float().view(L, 3, nh, hd).permute(1, 2, 0, 3)  # [3, nh, L, hd]
        q, k, v = x[0], x[1], x[2]
        S = (q @ k.transpose(1, 2)) * (hd ** -0.5)
        mask = torch.ones(L, L, dtype=torch.bool, device=qkv.device).tril()
        S = S.masked_fill(~mask, float("-inf"))
        m = S.amax(-1, keepdim=True)
        e = torch.exp(S - m)
        ssum = e.sum(-1, keepdim=True)
        P = e / ssum
        base = (n * nh + torch.arange(nh, device=qkv.device)) * _DS
        i = torch.arange(L, device=qkv.device)
        idx = ((base[:, None, None] + i[None, :, None]) * _DS + i[None, None, :])
        if p > 0:
            keep = keep_at(idx.long(), seed, p)
            P = torch.where(keep, P / (1.0 - p), torch.zeros_like(P))
        P = _bf(P)
        o[s0:s0 + L] = (P @ v).transpose(0, 1).reshape(L, H)
        lse.view(-1, ld)[n * nh:(n + 1) * nh, :L] = (m + torch.log(ssum)).squeeze(-1)
    return o.to(qkv.dtype), lse


class _Attention(torch.autograd.Function):
    """o [M, H] = causal self-attention of every sequence's token rows of
    qkv [M, 3H] (csrc/attention.hip on HIP tensors); ``max_len`` (host int)
    bounds every sequence's length and selects the kernel family."""

    @staticmethod
    def forward(ctx, qkv, start, lens, nh, p, seed, max_len=ATTN_SHORT_LEN):
        if qkv.is_cuda:
            o, lse = _ops().attn_fwd(qkv, start, lens, nh, p, seed, max_len)
            ctx.save_for_backward(qkv, o, lse, start, lens)
        else:
            o, _ = _ref_attn(qkv, start, lens, nh, p, seed, max_len)
            ctx.save_for_backward(qkv, start, lens)
        ctx.cfg = (nh, p, seed, max_len)
        return o

    @staticmethod
    def backward(ctx, g):
        nh, p, seed, max_len = ctx.cfg
        if g.is_cuda:
            qkv, o, lse, start, lens = ctx.saved_tensors
            dqkv = _ops().attn_bwd(qkv, o, g.contiguous(), lse, start, lens, nh, p, seed, max_len)
        else:
            qkv, start, lens = ctx.saved_tensors
            with torch.enable_grad():
                x = qkv.detach().float().requires_grad_()
                o, _ = _ref_attn(x, start, lens, nh, p, seed, max_len)
                o.float().backward(g.float())
            dqkv = x.grad.to(qkv.dtype)
        return dqkv, None, None, None, None, None, None


def gpt2_hidden(tr, input_ids: torch.Tensor, token_type_ids: Optional[torch.Tensor] = None,
                lengths: Optional[torch.Tensor] = None):
    """``ln_f`` output of HF ``GPT2Model`` ``tr`` for ``input_ids`` [..., L]
    (same as ``tr(input_ids, token_type_ids=...)[0]``) on the native junction
    kernels.  Dropout follows ``tr.training`` like the HF modules.

    ``lengths`` (host int64, one per sequence; PersonaChat: mc_token_ids + 1)
    marks each row's real tokens, padding being at the end: every token-wise
    op (embeddings, GEMMs, junctions) then runs on the real tokens only and
    just the attention sees the padded [N, heads, L, d] layout.  With causal
    attention right padding never reaches a real position, so the hidden
    states at real positions -- everything the losses read -- are the padded
    forward's; padded positions come back as 0."""
    cfg = tr.config
    shp = input_ids.shape
    L = shp[-1]
    H = cfg.n_embd
    ids = input_ids.reshape(-1, L)
    Nn = ids.shape[0]
    M = Nn * L
    nh = cfg.n_head
    eps = float(cfg.layer_norm_epsilon)
    train = tr.training

    def _p(mod, default):  # the HF dropout module's rate (tests may zero it)
        return float(getattr(mod, "p", default)) if train else 0.0

    pe = _p(getattr(tr, "drop", None), cfg.embd_pdrop)
    seeds = getattr(tr, "_commeff_seeds", None)
    if seeds is None:
        seeds = _Seeds(torch.initial_seed())
        tr._commeff_seeds = seeds
    tok = inv = sstart = slen = None
    max_len = L
    if lengths is not None and not lengths.is_cuda:
        max_len = int(lengths.max()) if lengths.numel() else 0
        if int(lengths.sum()) < M:
            ti = real_token_index(lengths, L, ids.device)
            if ti is not None:
                tok, inv, sstart, slen = ti
    Mr = M if tok is None else tok.shape[0]
    # fused short-sequence attention (csrc/attention.hip) straight on the
    # token rows; the padded-layout SDPA path otherwise
    fused_attn = (_ATTN["enabled"] and ids.is_cuda and H // nh == 64 and max_len <= ATTN_MAX_LEN)
    if fused_attn and sstart is None:
        import numpy as np
        se = np.concatenate([np.arange(Nn) * L, np.full(Nn, L)]).astype(np.int32)
        from ..parallel.dist import h2d
        se = h2d(se, ids.device)
        sstart, slen = se[:Nn], se[Nn:]
    if _embed_native_ok(tr, ids):
        # one native gather-add (real token rows only) and its sort-free backward
        tt_flat = token_type_ids.reshape(M).contiguous() if token_type_ids is not None else None
        e = _Embed.apply(tr.wte.weight, tr.wpe.weight, ids.reshape(M).contiguous(), tt_flat, tok, L)
    elif tok is None:
        pos = torch.arange(L, device=ids.device)
        e = (tr.wte(ids) + tr.wpe(pos)).reshape(M, H)
        if token_type_ids is not None:
            e = e + tr.wte(token_type_ids.reshape(M))
    else:
        tl = tok.long()
        e = tr.wte(ids.reshape(M).index_select(0, tl)) + tr.wpe(tl % L)
        if token_type_ids is not None:
            e = e + tr.wte(token_type_ids.reshape(M).index_select(0, tl))
    blocks = tr.h
    ln = blocks[0].ln_1
    h, y = _EmbedLN.apply(e, ln.weight, ln.bias, pe, seeds.next(), eps)
    for i, blk in enumerate(blocks):
        at = blk.attn
        qkv = _Linear.apply(y, at.c_attn.weight, at.c_attn.bias)
        pa = _p(getattr(at, "attn_dropout", None), cfg.attn_pdrop)
        if fused_attn:
            o = _Attention.apply(qkv, sstart, slen, nh, pa, seeds.next(), max_len)
        else:
            # token rows -> padded per-head q, k, v and back in one kernel each
            # (the layout change, the padding and, backward, the q/k/v
            # gradient concatenation in the same pass)
            q, k, v = _RowsToHeads.apply(qkv, tok, inv, Nn, L, nh)
            o = F.scaled_dot_product_attention(q, k, v, dropout_p=pa, is_causal=True)
            o = _HeadsToRows.apply(o, tok, inv, Mr)
        h, y = _ResidLN.apply(h, o, at.c_proj.weight, at.c_proj.bias, blk.ln_2.weight,
                              blk.ln_2.bias, _p(getattr(at, "resid_dropout", None), cfg.resid_pdrop),
                              seeds.next(), eps)
        f = _FcGelu.apply(y, blk.mlp.c_fc.weight, blk.mlp.c_fc.bias)
        nxt = blocks[i + 1].ln_1 if i + 1 < len(blocks) else tr.ln_f
        h, y = _ResidLN.apply(h, f, blk.mlp.c_proj.weight, blk.mlp.c_proj.bias, nxt.weight,
                              nxt.bias, _p(getattr(blk.mlp, "dropout", None), cfg.resid_pdrop),
                              seeds.next(), eps)
    if tok is not None:
        y = _ToPadded.apply(y, tok, M)
    return y.view(*shp, H)
