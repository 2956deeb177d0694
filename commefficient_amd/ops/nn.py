"""Autograd wrappers for fused native NN kernels used by the models.

``relu_maxpool(x, k)`` = ``max_pool2d(relu(x), k)`` (relu and max commute).
On a HIP device with a bf16 channels_last input it runs the fused gfx950
kernels of csrc/pool.hip (one read of the conv output forward, one coalesced
write of the input gradient backward); otherwise it is the plain PyTorch
composition (CPU runs, fp32 runs, odd shapes).
"""
from __future__ import annotations

import contextlib
import os
import weakref

import torch
import torch.nn.functional as F

from .._ext import ops as _ops
from . import lanes as _lanes


class _ReluMaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k):
        y, idx = _ops().relu_maxpool(x, k)
        ctx.save_for_backward(idx)
        ctx.k = k
        return y

    @staticmethod
    def backward(ctx, gy):
        (idx,) = ctx.saved_tensors
        return _ops().relu_maxpool_backward(gy.to(torch.bfloat16), idx, ctx.k), None


# ``stock_ops()``: every model op takes its plain PyTorch composition (no
# native kernels, no flat-buffer gradient sinks) -- for torch.func transforms
# (vmap over per-client weight copies in the batched FedAvg local SGD,
# parallel/fed_model.py), which the native autograd Functions do not support
_STOCK = [False]


class stock_ops:
    def __enter__(self):
        self.prev = _STOCK[0]
        _STOCK[0] = True
        return self

    def __exit__(self, *exc):
        _STOCK[0] = self.prev
        return False


def stock_active() -> bool:
    return _STOCK[0]


def fused_ok(x: torch.Tensor, k: int) -> bool:
    return (not _STOCK[0] and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and k in (2, 4)
            and x.shape[1] % 8 == 0 and x.shape[2] % k == 0 and x.shape[3] % k == 0
            and x.is_contiguous(memory_format=torch.channels_last))


def relu_maxpool(x: torch.Tensor, k: int) -> torch.Tensor:
    if fused_ok(x, k):
        return _ReluMaxPool.apply(x, k)
    return F.max_pool2d(F.relu(x), k)


# ---------------------------------------------------------------- conv3x3
# Backend switch for 3x3 convolutions that fit the native MFMA kernels
# (csrc/conv.hip): "native" (default) or "miopen" (torch.nn.functional.conv2d).
_CONV_BACKEND = ["native"]

# Listeners told when a native backward has written a parameter's gradient
# straight into its flat-buffer ``.grad`` (and handed autograd None, so no
# AccumulateGrad node and no post-accumulate hook runs for it): the dense
# modes' overlapped bucket all-reduce (parallel/overlap.py) counts these as
# "gradient ready".  Called on the stream that wrote the gradient.
_GRAD_READY = []


def add_grad_ready_listener(fn):
    _GRAD_READY.append(fn)


def remove_grad_ready_listener(fn):
    if fn in _GRAD_READY:
        _GRAD_READY.remove(fn)


def _grad_written(*params):
    if _GRAD_READY:
        for p in params:
            if p is not None:
                for fn in _GRAD_READY:
                    fn(p)


def set_conv_backend(name: str) -> None:
    if name not in ("native", "miopen"):
        raise ValueError(f"unknown conv backend {name!r}")
    _CONV_BACKEND[0] = name


def conv_backend() -> str:
    return _CONV_BACKEND[0]


# bf16 GEMM images of conv weights prepared for the current forward pass
# (one batched launch for the whole model, see prepared_conv_weights)
_PREP: dict = {}


class _ImageCache:
    """The bf16 GEMM images of one set of conv weights, kept across forward
    passes.  They are reused only after a sparse server step (FetchSGD /
    true top-k: k of d coordinates change) has patched the changed
    coordinates in place (``weights_begin_update`` / ``weights_end_update``);
    any other change of the weights -- a dense server step, local SGD steps
    on a work buffer, a resume -- leaves them stale, so a freshly converted
    set is never reused as is."""

    __slots__ = ("weights", "images", "versions", "valid", "synced")

    def __init__(self, weights, images):
        self.weights = weights
        self.images = images
        self.versions = [w._version for w in weights]
        self.valid = False   # reusable by the next pass (set by a patch)
        self.synced = True   # converted from the weights as they are now

    def _unchanged(self) -> bool:
        return all(w._version == v for w, v in zip(self.weights, self.versions))

    def fresh(self) -> bool:
        return self.valid and self._unchanged()

    # weight-mirror protocol (weights_begin_update / weights_end_update)
    def begin(self, w_flat: torch.Tensor) -> bool:
        lo, hi = w_flat.data_ptr(), w_flat.data_ptr() + 4 * w_flat.numel()
        usable = self.valid or self.synced
        ok = (usable and self._unchanged() and len(self.weights) <= 16
              and all(lo <= w.data_ptr() < hi for w in self.weights))
        self.valid = self.synced = False
        if usable and not ok:
            _IMG_GEN[0] += 1  # in sync until now, stale from here on: recorded readers re-record
        return ok

    def patch(self, w_flat: torch.Tensor, idx: torch.Tensor) -> None:
        _ops().conv_images_patch(w_flat, idx, self.weights, self.images)
        self.versions = [w._version for w in self.weights]
        self.valid = True


_IMAGES: dict = {}  # key: weight data pointers -> _ImageCache (one model at a time)
# bumped whenever the kept images are replaced or dropped: recorded rounds
# that read them (parallel/tape.py) are recorded again
_IMG_GEN = [0]


def image_generation() -> int:
    return _IMG_GEN[0]
# other derived copies of the flat weights (parallel/flat.py bf16 replica),
# weakly held: a torn-down FedModel's replica is not kept alive or updated
_MIRRORS = weakref.WeakSet()
_IMAGE_CACHE_ON = [True]


def set_conv_image_cache(on: bool) -> None:
    """Keep derived weight copies (conv images, the bf16 replica) across
    passes; COMMEFF_WEIGHT_MIRRORS=0 turns this off (re-derive every pass)."""
    _IMAGE_CACHE_ON[0] = bool(on)
    _IMAGES.clear()
    _IMG_GEN[0] += 1


def register_weight_mirror(m) -> None:
    """``m`` (begin(w_flat) -> bool, patch(w_flat, idx)) follows sparse
    server steps like the conv images (weakly held by identity)."""
    _MIRRORS.add(m)


def mirrors_enabled() -> bool:
    return _IMAGE_CACHE_ON[0]


def invalidate_conv_images() -> None:
    """The flat weights were rewritten outside a server step (e.g. a resume):
    kept derived copies must be rebuilt."""
    for c in list(_IMAGES.values()) + list(_MIRRORS):
        c.begin(torch.empty(0))
    _IMG_GEN[0] += 1


class prepared_conv_weights:
    """``with prepared_conv_weights(ws): model(x)`` -- converts every weight in
    ``ws`` to its two bf16 GEMM images (forward [K,3,3,C] and flipped dgrad
    [C,3,3,K]) in ONE kernel launch, or reuses the images kept from the last
    pass when the weights have not changed since (or were patched by a sparse
    server update); the native conv units of this forward pick them up
    instead of preparing their weight one by one."""

    def __init__(self, weights, plain=None):
        self.weights = [w for w in weights if w.is_cuda and w.dtype == torch.float32
                        and w.dim() == 4 and tuple(w.shape[2:]) == (3, 3)
                        and w.shape[1] % 64 == 0]
        self.keys = []
        # ``plain`` = (flat fp32 buffer, 1x1 weights that are views into it):
        # their bf16 GEMM operands come from ONE cast of the span they cover
        # into a kept bf16 buffer (ResNet-101: 62 per-weight cast launches
        # per round before)
        self.plain = plain

    def __enter__(self):
        if self.weights and _CONV_BACKEND[0] == "native" and not _STOCK[0]:
            ws = [w.detach() for w in self.weights]
            capturing = torch.cuda.is_current_stream_capturing()
            ck = tuple(w.data_ptr() for w in ws)
            cache = _IMAGES.get(ck) if _IMAGE_CACHE_ON[0] else None
            if cache is not None and cache.fresh():
                # (also while a round is recorded, parallel/tape.py: the replays
                # read these images, which the recorded server step keeps
                # patched; a replaced cache bumps image_generation() and the
                # engine records its rounds again)
                out = cache.images
            else:
                out = _ops().conv_weight_prep_multi(ws)
                if not capturing and _IMAGE_CACHE_ON[0]:
                    _IMAGES.clear()
                    _IMAGES[ck] = _ImageCache(ws, out)
                    _IMG_GEN[0] += 1
            for i, w in enumerate(self.weights):
                key = (w.data_ptr(), w._version)
                _PREP[key] = (out[2 * i], out[2 * i + 1])
                self.keys.append(key)
        if self.plain is not None and _CONV_BACKEND[0] == "native" and not _STOCK[0]:
            self._cast_plain(*self.plain)
        return self

    def _cast_plain(self, flat, ws):
        if not (flat.is_cuda and flat.dtype == torch.float32 and flat.dim() == 1 and flat.is_contiguous()):
            return
        base, d = flat.data_ptr(), flat.numel()
        offs = []
        for w in ws:
            o = (w.data_ptr() - base) // 4
            if w.dtype == torch.float32 and w.is_contiguous() and 0 <= o and o + w.numel() <= d:
                offs.append((w, o))
        if not offs:
            return
        lo = min(o for _, o in offs)
        hi = max(o + w.numel() for w, o in offs)
        buf = _PLAIN_BUF.get("buf")
        if buf is None or buf.numel() != d or buf.device != flat.device:
            # kept across rounds: one stable address (recorded rounds read it)
            buf = torch.empty(d, dtype=torch.bfloat16, device=flat.device)
            _PLAIN_BUF["buf"] = buf
        _ops().fa_cast_rows(buf, flat, d, 1, lo, hi - lo)
        for w, o in offs:
            key = (w.data_ptr(), w._version)
            _PREP1[key] = buf[o:o + w.numel()].view(w.shape[0], -1)
            self.keys.append(key)

    def __exit__(self, *exc):
        for k in self.keys:
            _PREP.pop(k, None)
            _PREP1.pop(k, None)
        return False


_PREP1: dict = {}  # (weight ptr, version) -> its bf16 [K, C] view (prepared_conv_weights plain)
_PLAIN_BUF: dict = {}


def _prep1(weight: torch.Tensor, k: int, c: int) -> torch.Tensor:
    """bf16 [k, c] GEMM operand of a 1x1 conv weight: the prepared one, else a cast."""
    hit = _PREP1.get((weight.data_ptr(), weight._version))
    return hit if hit is not None else weight.detach().view(k, c).to(torch.bfloat16)


def weights_begin_update(w_flat: torch.Tensor):
    """Call before a server step modifies the flat weights ``w_flat``: every
    kept derived copy becomes stale; returns the ones that were in sync with
    ``w_flat`` for ``weights_end_update``."""
    if not w_flat.is_cuda:
        return []
    return [m for m in list(_IMAGES.values()) + list(_MIRRORS) if m.begin(w_flat)]


def weights_end_update(sync, w_flat: torch.Tensor, idx: torch.Tensor) -> None:
    """The server step changed exactly the coordinates ``idx`` of ``w_flat``:
    patch those into the copies that were in sync (one small kernel each)."""
    if sync:
        idx = idx.contiguous()
        for m in sync:
            m.patch(w_flat, idx)


def _prep(weight: torch.Tensor):
    hit = _PREP.get((weight.data_ptr(), weight._version))
    return hit if hit is not None else _ops().conv_weight_prep(weight.detach().contiguous())


def _wgrad_to(g: torch.Tensor, x: torch.Tensor, weight: torch.Tensor):
    """Weight gradient of a native conv.  When ``weight.grad`` already exists
    (FedModel keeps every .grad as a view of its flat gradient buffer) the
    split-K reduction accumulates straight into it and None is handed back to
    autograd -- no separate dW tensor and no AccumulateGrad add pass -- on the
    side lane (ops/lanes.py: it overlaps the input gradients of the layers
    below; the engine joins it after the backward)."""
    gr = weight.grad
    if (gr is not None and gr.dtype == torch.float32 and gr.is_contiguous()
            and gr.device == g.device and tuple(gr.shape) == tuple(weight.shape)):
        with _lanes.fork(g, x):
            _ops().conv3x3_wgrad_into(g, x, gr)
        _grad_written(weight)
        return None
    return _ops().conv3x3_wgrad(g, x)


def _pool_fusable(x: torch.Tensor, weight: torch.Tensor) -> bool:
    """The fused conv + relu + maxpool2 epilogue needs whole image-row pairs
    per 128-pixel tile (csrc/conv.hip ``conv3x3_pool_supported``)."""
    H, W = x.shape[2], x.shape[3]
    return weight.shape[0] % 128 == 0 and H % 2 == 0 and W % 2 == 0 and 128 % (2 * W) == 0


class _UnpoolLink:
    """Hand-off between a fused conv + relu + 2x2 max-pool unit and the native
    unit that consumes its pooled output (ResNet-9: layer1 -> res1, layer2 ->
    layer3, layer3 -> res3).  The consumer's backward computes its input
    gradient with the pool backward fused into the dgrad epilogue
    (``conv3x3_fwd_unpool``: the full-resolution gradient, each value at its
    window's argmax) and parks it here; autograd gets a zero-stride zero
    tensor of the pooled shape instead, and the producer's backward takes the
    parked gradient (adding the unfused expansion of anything else autograd
    accumulated into its output gradient) -- one kernel and one pooled-size
    round trip fewer per pooled layer."""

    __slots__ = ("idx", "grad", "dummy", "claimed")

    def __init__(self, idx):
        self.idx = idx
        self.grad = None
        self.dummy = None
        self.claimed = False  # one consumer only (a second one uses the unfused path)

    def park(self, full, like):
        self.grad = full
        key = (like.dtype, like.device)
        z = _ZERO.get(key)
        if z is None:  # one cached zero per dtype/device: no fill kernel per backward
            z = _ZERO[key] = torch.zeros((1, 1, 1, 1), dtype=like.dtype, device=like.device)
        self.dummy = z.expand(like.shape)
        return self.dummy

    def take(self, gout):
        """The producer's full-resolution gradient (None: nothing parked)."""
        full, dummy = self.grad, self.dummy
        self.grad = self.dummy = None
        if full is None:
            return None
        if gout is dummy or (gout.data_ptr() == dummy.data_ptr() and gout.stride() == dummy.stride()):
            return full
        # autograd added other consumers' gradients to the dummy's zeros
        g = gout.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        return full + _ops().relu_maxpool_backward(g, self.idx, 2)


class _MaskLink:
    """Hand-off between a native residual unit (its output's relu mask ``y2``)
    and the native conv that consumes that output (ResNet-9: res1 ->
    layer2): the consumer's dgrad epilogue also writes the gradient masked by
    ``y2`` (``conv3x3_fwd_dual``), which the residual unit's backward takes
    instead of a separate relu-mask pass -- when the gradient it receives is
    exactly that dgrad (one consumer; otherwise it masks what it got)."""

    __slots__ = ("mask", "src", "masked", "claimed")

    def __init__(self, mask):
        self.mask = mask
        self.src = self.masked = None
        self.claimed = False

    def take(self, g):
        src, masked = self.src, self.masked
        self.src = self.masked = None
        if masked is not None and g.data_ptr() == src.data_ptr() and g.shape == src.shape \
                and g.stride() == src.stride():
            return masked
        return None


_UNPOOL_ON = [True]
_ZERO: dict = {}


def set_fused_unpool(on: bool) -> None:
    """Fuse the relu + max-pool backward into the consumer's dgrad epilogue
    (default on; off = the separate csrc/pool.hip backward kernel)."""
    _UNPOOL_ON[0] = bool(on)


def _mask_link_of(x: torch.Tensor):
    link = getattr(x, "_commeff_mask", None)
    if not (_UNPOOL_ON[0] and link is not None and not link.claimed and link.mask.shape == x.shape
            and torch.is_grad_enabled() and x.requires_grad):
        return None
    link.claimed = True
    return link


def _link_of(x: torch.Tensor):
    link = getattr(x, "_commeff_unpool", None)
    if not (_UNPOOL_ON[0] and link is not None and not link.claimed and link.idx.shape == x.shape
            and torch.is_grad_enabled() and x.requires_grad):
        return None
    link.claimed = True
    return link


class _Conv3x3Act(torch.autograd.Function):
    """relu(conv3x3(x, w)) or maxpool_k(relu(conv3x3(x, w))), no bias.

    Forward: the MFMA implicit-GEMM kernel with a fused ReLU epilogue (or the
    fused relu+maxpool kernel on the conv output).  Backward: relu mask /
    pool scatter, dgrad = the same forward kernel on the flipped, transposed
    weight, wgrad = the transposed-LDS-read MFMA kernel with a deterministic
    split-K reduction straight into the fp32 [K, C, 3, 3] gradient.
    """

    last_out_link = None  # forward -> conv3x3_relu_pool side channel (no autograd state)

    @staticmethod
    def forward(ctx, x, weight, pool_k, in_link=None, in_mask=None):
        wf, wt = _prep(weight)
        ctx.in_link = in_link
        ctx.in_mask = in_mask
        ctx.out_link = None
        if pool_k == 2 and _pool_fusable(x, weight):
            # relu + 2x2 max-pool in the conv epilogue: the full-resolution
            # activation is never written
            out, idx = _ops().conv3x3_fwd_pool2(x, wf)
            ctx.save_for_backward(x, wt, idx)
            ctx.out_link = _UnpoolLink(idx)
        elif pool_k:
            y = _ops().conv3x3_fwd(x, wf, False)
            out, idx = _ops().relu_maxpool(y, pool_k)
            del y
            ctx.save_for_backward(x, wt, idx)
        else:
            out = _ops().conv3x3_fwd(x, wf, True)
            ctx.save_for_backward(x, wt, out)
        ctx.pool_k = pool_k
        ctx.weight = weight
        _Conv3x3Act.last_out_link = ctx.out_link
        return out

    @staticmethod
    def backward(ctx, gout):
        x, wt, aux = ctx.saved_tensors
        g = ctx.out_link.take(gout) if ctx.out_link is not None else None
        if g is None:
            gout = gout.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            if ctx.pool_k:
                g = _ops().relu_maxpool_backward(gout, aux, ctx.pool_k)
            else:
                g = _ops().relu_mask(gout, aux)
        # (the weight gradient first: on the side lane it overlaps the dgrad)
        gw = _wgrad_to(g, x, ctx.weight) if ctx.needs_input_grad[1] else None
        gx = None
        if ctx.needs_input_grad[0]:
            link = ctx.in_link
            if link is not None:  # the input's relu + max-pool backward in the epilogue
                gx = link.park(_ops().conv3x3_fwd_unpool(g, wt, None, link.idx), x)
            elif ctx.in_mask is not None:  # + the producer's relu-masked copy
                gx, gxm = _ops().conv3x3_fwd_dual(g, wt, ctx.in_mask.mask)
                ctx.in_mask.src, ctx.in_mask.masked = gx, gxm
            else:
                gx = _ops().conv3x3_fwd(g, wt, False)
        return gx, gw, None, None, None


class _ResidualUnit(torch.autograd.Function):
    """``x + relu(conv3x3(relu(conv3x3(x, w1)), w2))`` -- ResNet-9's Residual
    (reference models/resnet9.py:61-72) as one native unit.

    Forward: the second conv's epilogue applies the ReLU, adds the skip input
    and also emits the pre-add activation (its ReLU mask is needed backward).
    Backward: one relu-mask kernel; dgrad of conv2 masks by relu(conv1)'s
    output in its epilogue (= conv1's ReLU backward); dgrad of conv1 adds the
    skip gradient in its epilogue.  Two elementwise passes fewer each way
    than the per-op composition.
    """

    last_mask_link = None  # forward -> residual_unit side channel (no autograd state)

    @staticmethod
    def forward(ctx, x, w1, w2, in_link=None):
        w1f, w1t = _prep(w1)
        w2f, w2t = _prep(w2)
        y1 = _ops().conv3x3_fwd(x, w1f, True)
        out, y2 = _ops().conv3x3_relu_add(y1, w2f, x)
        ctx.save_for_backward(x, y1, y2, w1t, w2t)
        ctx.w1, ctx.w2 = w1, w2
        ctx.in_link = in_link
        ctx.out_mask = _MaskLink(y2)
        _ResidualUnit.last_mask_link = ctx.out_mask
        return out

    @staticmethod
    def backward(ctx, g):
        x, y1, y2, w1t, w2t = ctx.saved_tensors
        g = g.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        g2 = ctx.out_mask.take(g)  # masked by the consumer's dgrad epilogue
        if g2 is None:
            g2 = _ops().relu_mask(g, y2)
        dw2 = _wgrad_to(g2, y1, ctx.w2) if ctx.needs_input_grad[2] else None
        g1 = _ops().conv3x3_fwd(g2, w2t, False, y1)  # masked by relu(conv1) > 0
        dw1 = _wgrad_to(g1, x, ctx.w1) if ctx.needs_input_grad[1] else None
        gx = None
        if ctx.needs_input_grad[0]:
            link = ctx.in_link
            if link is not None:  # + the input's relu + max-pool backward in the epilogue
                gx = link.park(_ops().conv3x3_fwd_unpool(g1, w1t, g, link.idx), x)
            else:
                gx = _ops().conv3x3_fwd(g1, w1t, False, None, g)
        return gx, dw1, dw2, None


def residual_unit(x: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor) -> torch.Tensor:
    """``x + relu(conv2(relu(conv1(x))))`` (3x3, pad 1, no bias)."""
    if conv3x3_native_ok(x, w1) and conv3x3_native_ok(x, w2) and w1.shape[0] == x.shape[1]:
        out = _ResidualUnit.apply(x, w1, w2, _link_of(x))
        if _ResidualUnit.last_mask_link is not None and out.requires_grad:
            out._commeff_mask = _ResidualUnit.last_mask_link
        _ResidualUnit.last_mask_link = None
        return out
    y = F.relu(F.conv2d(x, w1, padding=1))
    return x + F.relu(F.conv2d(y, w2, padding=1))


def conv3x3_native_ok(x: torch.Tensor, weight: torch.Tensor) -> bool:
    return (_CONV_BACKEND[0] == "native" and not _STOCK[0] and x.is_cuda
            and x.dtype == torch.bfloat16
            and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)
            and weight.dtype == torch.float32 and weight.dim() == 4
            and tuple(weight.shape[2:]) == (3, 3) and weight.shape[1] == x.shape[1]
            and x.shape[1] % 64 == 0 and weight.shape[0] % 128 == 0)


def conv3x3_relu_pool(x: torch.Tensor, weight: torch.Tensor, pool_k: int = 0) -> torch.Tensor:
    """``max_pool2d(relu(conv2d(x, weight, padding=1)), pool_k)`` (no pool when
    ``pool_k == 0``).  Native MFMA kernels when :func:`conv3x3_native_ok`,
    else the PyTorch (MIOpen) composition."""
    if conv3x3_native_ok(x, weight) and (
            pool_k == 0 or (x.shape[2] % pool_k == 0 and x.shape[3] % pool_k == 0)):
        out = _Conv3x3Act.apply(x, weight, int(pool_k), _link_of(x), _mask_link_of(x))
        link = _Conv3x3Act.last_out_link
        if link is not None:
            out._commeff_unpool = link
        return out
    y = F.conv2d(x, weight, padding=1)
    return relu_maxpool(y, pool_k) if pool_k else F.relu(y)


class _InputConv(torch.autograd.Function):
    """relu(conv3x3(x, w)) for the 3-channel network input (csrc/conv_prep.hip):
    MFMA forward with a fused ReLU that also emits a 1-bit ReLU mask per
    output; backward computes only dW (the input is data) from gy and the
    mask, accumulating into an existing flat-buffer ``.grad``."""

    @staticmethod
    def forward(ctx, x, weight):
        y, mask = _ops().conv_prep_fwd(x, weight.detach().contiguous())
        ctx.save_for_backward(x, mask)
        ctx.weight = weight
        return y

    @staticmethod
    def backward(ctx, gy):
        x, mask = ctx.saved_tensors
        if not ctx.needs_input_grad[1]:
            return None, None
        gr = ctx.weight.grad
        if (gr is not None and gr.dtype == torch.float32 and gr.is_contiguous()
                and gr.device == gy.device and gr.shape == ctx.weight.shape):
            _ops().conv_prep_wgrad_into(gy, mask, x, gr)
            _grad_written(ctx.weight)
            return None, None
        return None, _ops().conv_prep_wgrad(gy, mask, x)


def input_conv_native_ok(x: torch.Tensor, weight: torch.Tensor) -> bool:
    """The augmentation kernel's 3-channel bf16 batch (4-channel pixel stride)
    into a [64, 3, 3, 3] conv."""
    if not (_CONV_BACKEND[0] == "native" and not _STOCK[0] and x.is_cuda
            and x.dtype == torch.bfloat16
            and x.dim() == 4 and x.shape[1] == 3 and not x.requires_grad
            and weight.dtype == torch.float32 and tuple(weight.shape) == (64, 3, 3, 3)):
        return False
    H, W = x.shape[2], x.shape[3]
    return x.stride() == (4 * H * W, 1, 4 * W, 4)


def conv3x3_input_relu(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """``relu(conv2d(x, weight, padding=1))`` for the network input."""
    if input_conv_native_ok(x, weight):
        return _InputConv.apply(x, weight)
    return F.relu(F.conv2d(x, weight, padding=1))


# ------------------------------------------------------------ head
class _FusedHead(torch.autograd.Function):
    """``CE(scale * linear(maxpool_HxW(relu(x))), targets)`` per example, plus
    top-1 correctness -- ResNet-9's pool/flatten/linear/Mul head and the CV
    loss in one native kernel each way (csrc/head.hip).  The weight gradient
    accumulates straight into an existing flat-buffer ``.grad``."""

    @staticmethod
    def forward(ctx, x, weight, targets, scale, in_mask=None):
        loss, correct, gunit, pooled, codes = _ops().head_fwd(x, weight.detach(), targets,
                                                              float(scale))
        ctx.save_for_backward(gunit, pooled, codes)
        ctx.weight, ctx.scale, ctx.hw = weight, float(scale), (x.shape[2], x.shape[3])
        # a native residual unit's output (link taken by fused_head_loss: grad
        # mode is off in here): the backward also writes the gradient masked
        # by its ReLU (dual output, no relu_mask pass)
        ctx.in_mask = in_mask
        ctx.mark_non_differentiable(correct)
        ctx.set_materialize_grads(False)  # no zeros fill for the unused gradient of `correct`
        return loss, correct

    @staticmethod
    def backward(ctx, gl, gc):
        if gl is None:  # (grads are not materialised) the loss got no gradient
            return None, None, None, None, None
        gunit, pooled, codes = ctx.saved_tensors
        w = ctx.weight
        gr = w.grad
        into = (gr is not None and gr.dtype == torch.float32 and gr.is_contiguous()
                and gr.shape == w.shape and gr.device == w.device)
        dw = gr if into else torch.empty_like(w, dtype=torch.float32)
        if ctx.in_mask is not None:
            dx, dxm = _ops().head_bwd_dual(gl.contiguous(), gunit, w.detach(), pooled, codes, ctx.hw[0],
                                           ctx.hw[1], ctx.scale, dw, 1.0 if into else 0.0, ctx.in_mask.mask)
            ctx.in_mask.src, ctx.in_mask.masked = dx, dxm
        else:
            dx = _ops().head_bwd(gl.contiguous(), gunit, w.detach(), pooled, codes, ctx.hw[0],
                                 ctx.hw[1], ctx.scale, dw, 1.0 if into else 0.0)
        if into:
            _grad_written(w)
        return dx, (None if into else dw), None, None, None


def head_native_ok(x: torch.Tensor, weight: torch.Tensor) -> bool:
    return (not _STOCK[0] and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 8 == 0
            and x.shape[2] * x.shape[3] <= 255 and weight.dtype == torch.float32
            and weight.dim() == 2 and weight.shape[1] == x.shape[1] and weight.shape[0] <= 128)


def fused_head_loss(x, weight, targets, scale: float):
    """(per-example CE loss, correct) of ``scale * maxpool_all(relu(x)) @ weight.T``."""
    link = _mask_link_of(x)
    if link is not None and not (link.mask.dtype == torch.bfloat16
                                 and link.mask.is_contiguous(memory_format=torch.channels_last)):
        link = None
    return _FusedHead.apply(x, weight, targets.contiguous(), float(scale), link)


# ------------------------------------------------------------ ghost batch norm
class _GhostBN(torch.autograd.Function):
    """Per-group batch norm over NHWC bf16 (csrc/bn.hip): 3 kernels forward,
    3 backward; running statistics updated in place with the group-averaged
    moments (the torch path in models/common.py GhostBatchNorm2d)."""

    @staticmethod
    def forward(ctx, x, weight, bias, groups, eps, momentum, running_mean, running_var, relu, nbt,
                gg=None, addend=None, tstats=None):
        if addend is not None:  # y = relu(bn(x) + addend): a residual block's tail
            addend = addend.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y, stat, bits = _ops().ghost_bn_fwd(x, weight, bias, int(groups), float(eps), float(momentum),
                                            running_mean, running_var, bool(relu), nbt, addend, tstats)
        # the backward's ReLU gate: 1 bit per element (y itself is 16)
        ctx.save_for_backward(x, stat, weight, bits if relu else None)
        ctx.groups = int(groups)
        ctx.params = (weight, bias)
        ctx.gg = gg
        ctx.has_add = addend is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, stat, weight, y = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        # existing fp32 .grad tensors (FedModel's flat-buffer views) receive
        # dweight / dbias in place: no AccumulateGrad launches
        pw, pb = ctx.params
        # the residual addend's gradient: the ReLU-masked dy, written by the
        # backward apply kernel
        dadd = torch.empty_like(dy) if ctx.has_add else None
        if dadd is not None:
            # a fresh buffer that only the residual branch consumes: its
            # consumer may accumulate into it in place (_Conv1x1Pass)
            dadd._commeff_fresh = True
        if ctx.gg is not None and pw is not None:
            # grouped (per-client) dweight / dbias rows, ops/grouped.py; the
            # BN groups are the gradient groups
            assert ctx.gg.G == ctx.groups, "grouped grads need ghost-BN groups == gradient groups"
            dx, _, _ = _ops().ghost_bn_bwd(dy, x, stat, weight, ctx.groups, y, None, None,
                                           ctx.gg.view(pw), ctx.gg.view(pb), dadd)
            return dx, None, None, None, None, None, None, None, None, None, None, dadd, None
        gw = pw.grad if pw is not None else None
        gb = pb.grad if pb is not None else None
        into = (gw is not None and gb is not None and gw.dtype == torch.float32
                and gb.dtype == torch.float32 and gw.is_contiguous() and gb.is_contiguous()
                and gw.device == x.device and gb.device == x.device
                and ctx.needs_input_grad[1] and ctx.needs_input_grad[2])
        dx, dw, db = _ops().ghost_bn_bwd(dy, x, stat, weight, ctx.groups, y,
                                         gw if into else None, gb if into else None, None, None,
                                         dadd)
        if weight is None or into:
            dw = db = None
        if into:
            _grad_written(pw, pb)
        return dx, dw, db, None, None, None, None, None, None, None, None, dadd, None


def ghost_bn_native_ok(x: torch.Tensor, weight) -> bool:
    return (not _STOCK[0] and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last)
            and x.shape[1] % 8 == 0 and x.shape[1] <= 2048
            and (weight is None or weight.dtype == torch.float32))


def ghost_batch_norm(x, weight, bias, groups: int, eps: float, momentum: float,
                     running_mean=None, running_var=None, relu: bool = False,
                     num_batches_tracked=None, gg=None, addend=None, tstats=None):
    """Per-group batch norm (+ ReLU when ``relu``) on the native kernels; the
    running statistics and ``num_batches_tracked`` are updated on the device.
    ``gg``: per-group weight gradients (ops/grouped.py).  ``addend``: y =
    relu(bn(x) + addend) in the same pass (needs ``relu``)."""
    assert addend is None or relu, "the fused residual add is followed by the ReLU"
    return _GhostBN.apply(x, weight, bias, groups, eps, momentum, running_mean, running_var, relu,
                          num_batches_tracked, gg, addend, tstats)


# ------------------------------------------------------------ loss
class _FusedCE(torch.autograd.Function):
    """Per-example cross-entropy + top-1 correctness in one kernel
    (csrc/loss.hip); the unit gradient softmax - onehot is produced in the
    same pass and scaled by dL/dloss in backward."""

    @staticmethod
    def forward(ctx, logits, targets):
        # (rows of a padded buffer -- the native LM head's logits -- are read
        # in place; the unit gradient comes back in the same row layout)
        x = logits if logits.stride(-1) == 1 else logits.contiguous()
        loss, correct, gunit = _ops().ce_fwd(x, targets.contiguous())
        ctx.save_for_backward(gunit)
        ctx.mark_non_differentiable(correct)
        return loss, correct

    @staticmethod
    def backward(ctx, gl, gc):
        (gunit,) = ctx.saved_tensors
        # the saved unit gradient is scaled in place (backward runs once)
        _ops().scale_rows(gunit, gl.float().contiguous())
        return gunit, None


def cross_entropy_correct(logits: torch.Tensor, targets: torch.Tensor):
    """(per-example CE loss f32, top-1 correct f32) of ``logits`` [B, C]."""
    if (not _STOCK[0] and logits.is_cuda and logits.dim() == 2 and targets.dtype == torch.int64
            and logits.dtype in (torch.bfloat16, torch.float32)):
        return _FusedCE.apply(logits, targets)
    per_ex = F.cross_entropy(logits.float(), targets, reduction="none")
    return per_ex, (logits.argmax(dim=1) == targets).float()


# ------------------------------------------------------------ generic convs
# ResNet-family convolutions (models/common.py NativeConv2d).  MIOpen's
# per-call host cost (solver lookup, find-db, workspace) and its bf16-grad ->
# fp32 cast + AccumulateGrad passes dominated the per-client ImageNet round
# (profiles/r2_v1_imagenet_round_kernels.txt: >50 % GPU idle at ~1,650 kernels
# per client).  Here:
#   * 1x1 convs are plain GEMMs on the NHWC activation ([P, C] x [C, K]) on
#     hipBLASLt; the weight gradient is a bf16 x bf16 -> fp32 GEMM that
#     accumulates straight into the flat fp32 gradient view;
#   * stride-1 3x3 convs with C % 64 == 0 and K % 64 == 0 run on the native
#     MFMA kernels of csrc/conv.hip (forward, dgrad on the flipped weights,
#     wgrad accumulating into the flat gradient when K % 128 == 0, else the
#     column-image wgrad below);
#   * every other bias-free, ungrouped conv of a bf16 channels-innermost
#     activation (the 7x7/s2 stem, strided 3x3, odd kernel sizes) is an
#     explicit GEMM over a bf16 column image (csrc/im2col.hip): im2col ->
#     hipBLASLt GEMM forward, GEMM + native col2im gather for dgrad, split-K
#     GEMM + native permute-add into the flat gradient for wgrad;
#   * grouped / dilated convs stay on MIOpen.
# Under ``ops.grouped.grouped_grads`` every path writes per-group weight
# gradients instead (see ops/grouped.py).
def _wlane(weight: torch.Tensor, gg, *inputs):
    """The side lane (ops/lanes.py) for a weight gradient accumulated into a
    sink -- the flat gradient or per-group rows -- that nothing in the
    backward reads; inline otherwise (a gradient handed back to autograd)."""
    if gg is not None or _grad_view(weight, weight.shape) is not None:
        return _lanes.fork(*inputs)
    return contextlib.nullcontext()


def _grad_view(weight: torch.Tensor, shape):
    """``weight.grad`` viewed as ``shape`` when it can receive an in-place fp32
    accumulation (FedModel keeps every .grad as a flat-buffer view)."""
    gr = weight.grad
    if (gr is not None and gr.dtype == torch.float32 and gr.is_contiguous()
            and gr.device == weight.device and tuple(gr.shape) == tuple(weight.shape)):
        return gr.view(shape)
    return None


# forward / input-gradient GEMMs of the 1x1 and column-image convs on the
# native MFMA kernels (csrc/gemm.hip); COMMEFF_GEMM=blas: hipBLASLt
_GEMM_NATIVE = [__import__("os").environ.get("COMMEFF_GEMM", "native") == "native"]


def _gemm_ok(a: torch.Tensor, b: torch.Tensor, n: int) -> bool:
    return (_GEMM_NATIVE[0] and a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
            and a.dim() == 2 and b.dim() == 2 and a.stride(1) == 1 and b.stride(1) == 1
            and n % 64 == 0 and a.shape[1] % 64 == 0 and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0)


def _mm_nt(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b^T with b [N, K] (a conv forward: rows of pixels x weight rows)."""
    if _gemm_ok(a, b, b.shape[0]):
        return _ops().mm_nt(a, b)
    return torch.mm(a, b.t())


# Ghost-BN statistics from the producing GEMM's epilogue: inside a merged
# BatchNorm forward (models/common.py ghost_batchnorm sets "G"), the native
# 1x1 / column-image conv forwards also write the per-128-row-tile moments of
# their output (csrc/gemm.hip GemmArgs::stats) and hand them to the consuming
# GhostBatchNorm2d on the output tensor (``_commeff_bnstats``), which then
# skips its statistics pass over x (csrc/bn.hip bn_fwd_finalize_tiles_kernel).
# Opt-in (COMMEFF_BN_EPI=1): on the ResNet-101 round the epilogue cost
# (+~20 us per forward GEMM: the 1x1 GEMMs run many waves of short-K tiles)
# outweighed the statistics pass it removes (profiles/r4_experiments.md).
_EPI = {"G": 0, "on": os.environ.get("COMMEFF_BN_EPI", "0") == "1", "last": None, "pair": None}


def _mm_nt_conv(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """_mm_nt for a conv forward; leaves the output's tile moments in
    ``_EPI["last"]`` when a ghost BN of G groups will consume it."""
    G = _EPI["G"]
    M = a.shape[0]
    if _EPI["on"] and G >= 1 and M % G == 0 and M // G >= 128 and _gemm_ok(a, b, b.shape[0]):
        y, st = _ops().mm_nt_bnstats(a, b, G)
        _EPI["last"] = (st, G)
        return y
    return _mm_nt(a, b)


def _with_bnstats(out: torch.Tensor) -> torch.Tensor:
    """Attach the moments the conv forward just computed to its output."""
    hit, _EPI["last"] = _EPI["last"], None
    if hit is not None:
        out._commeff_bnstats = (hit[0], hit[1], out._version)
    return out


def take_bnstats(x: torch.Tensor, G: int):
    """The producing GEMM's tile moments of ``x`` for a ghost BN of G groups,
    or None (not a fresh native conv output, modified in place since, or other
    groups)."""
    hit = getattr(x, "_commeff_bnstats", None)
    if hit is None:
        return None
    x._commeff_bnstats = None  # consumed once (and not kept alive with x)
    if hit[1] != G or hit[2] != x._version:
        return None
    return hit[0]


def _mm_nn(a: torch.Tensor, b: torch.Tensor, acc: torch.Tensor = None, in_place: bool = False):
    """a @ b with b [K, N] (a conv input gradient), + ``acc`` (in place into
    it when ``in_place``)."""
    if _gemm_ok(a, b, b.shape[1]) and (acc is None or (acc.dtype == torch.bfloat16 and acc.stride(1) == 1
                                                        and acc.stride(0) % 8 == 0)):
        if acc is None:
            return _ops().mm_nn(a, b)
        out = acc if in_place else acc.clone()
        return _ops().mm_nn(a, b, None, out, 1.0)
    if acc is None:
        return torch.mm(a, b)
    return torch.addmm(acc, a, b, out=acc) if in_place else torch.addmm(acc, a, b)


def _nhwc2d(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels_last -> its [N*H*W, C] row-major image (a view)."""
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _wgrad_splits(Pg: int, K: int, C: int, G: int) -> int:
    """Split-K factor of a [K, C] weight-gradient GEMM over G groups of Pg rows."""
    tiles = max(1, (K // 128) * (C // 128))
    S = 1
    while S < 64 and Pg % (2 * S) == 0 and Pg // (2 * S) >= 256 and G * S * tiles < 1024:
        S *= 2
    return S


def _wgrad_parts(g2d: torch.Tensor, x2d: torch.Tensor, G: int = 1):
    """(parts [G*S, K, C] fp32, S): the split-K partial products of
    g2d^T x2d for each group of P/G rows, unsummed."""
    P, K = g2d.shape
    C = x2d.shape[1]
    Pg = P // G
    if _WGRAD_TN and _wgrad_tn_ok(g2d, x2d, None, G):
        # the native split-K TN GEMM's slabs (csrc/gemm_tn.hip, slab-only)
        return _ops().gemm_tn_parts(g2d, x2d, G)
    S = _wgrad_splits(Pg, K, C, G)
    if G * S == 1:
        return torch.mm(g2d.t(), x2d, out_dtype=torch.float32).unsqueeze(0), 1
    return torch.bmm(g2d.view(G * S, Pg // S, K).transpose(1, 2), x2d.view(G * S, Pg // S, C),
                     out_dtype=torch.float32), S


# every weight gradient _wgrad_tn_ok accepts -- 1x1 convs, linears and the
# (implicit or materialised) column images of the stems and strided convs -- on
# the native split-K TN GEMM (256 x 256 tiles for 256-multiples, 128 x 128
# otherwise; round 5: no slower than hipBLASLt's batched GEMMs on the narrow
# shapes, profiles/r5_experiments.md); False routes them to hipBLASLt (A/B)
_WGRAD_TN = True


def _wgrad_tn_ok(g2d: torch.Tensor, x2d: torch.Tensor, into, G: int) -> bool:
    """csrc/gemm_tn.hip serves the weight gradient: K a multiple of 64 and C
    of 8 (256-multiples on its 256 x 256 tiles, the narrow 64 / 128-channel
    layers and the stem's 152 column-image columns on its 128 x 128 tiles),
    bf16 rows with unit column stride, 16-byte aligned; ``into`` fp32 with
    16-byte aligned rows (or absent)."""
    P, K = g2d.shape
    C = x2d.shape[1]
    if not (_GEMM_NATIVE[0] and g2d.is_cuda and K % 64 == 0 and C % 8 == 0 and P % G == 0
            and g2d.dtype == torch.bfloat16 and x2d.dtype == torch.bfloat16
            and g2d.stride(1) == 1 and x2d.stride(1) == 1 and g2d.stride(0) % 8 == 0
            and x2d.stride(0) % 8 == 0 and g2d.data_ptr() % 16 == 0 and x2d.data_ptr() % 16 == 0):
        return False
    if into is None:
        return True
    if into.dtype != torch.float32 or into.device != g2d.device or into.data_ptr() % 16 != 0:
        return False
    v = into.view(G, K, C) if (G > 1 or into.dim() == 3) else into.view(K, C)
    return v.stride(-1) == 1 and v.stride(-2) % 4 == 0 and (v.dim() == 2 or v.stride(0) % 4 == 0)


def _wgrad_gemm(g2d: torch.Tensor, x2d: torch.Tensor, into=None, G: int = 1) -> torch.Tensor:
    """dW (+)= g2d^T x2d, a reduction over the P rows, per group of P/G rows.

    ``into``: [K, C] (G == 1) or [G, K, C] (rows may be strided) fp32.
    P is 10^3-10^5 while K x C can be as small as 64 x 256, so one GEMM
    launches only a handful of output tiles, each looping over all of P
    (hipBLASLt picked 64x64 tiles without split-K: 12 TF/s, ~270 us per
    ResNet-101 layer-4 weight gradient).  Each group's rows are split into S
    chunks so G x S x tiles fills the chip: one batched bf16 x bf16 -> fp32
    GEMM writes the G x S partial products, one reduction adds them.
    Without a split the GEMM accumulates straight into ``into`` (beta = 1)."""
    P, K = g2d.shape
    C = x2d.shape[1]
    Pg = P // G
    if _WGRAD_TN and _wgrad_tn_ok(g2d, x2d, into, G):
        # native split-K TN GEMM (csrc/gemm_tn.hip), all groups in one launch,
        # splits summed in a fixed order into the flat (or per-group) gradient
        sink = into if into is not None else torch.zeros(
            (G, K, C) if G > 1 else (K, C), dtype=torch.float32, device=g2d.device)
        if G > 1:
            _ops().gemm_tn_acc_grouped(sink.view(G, K, C), g2d, x2d, G)
        else:
            _ops().gemm_tn_acc(sink.view(K, C), g2d, x2d)
        return sink
    S = _wgrad_splits(Pg, K, C, G)
    if G == 1 and S == 1:
        if into is not None:
            return torch.addmm(into, g2d.t(), x2d, out_dtype=torch.float32, out=into)
        return torch.mm(g2d.t(), x2d, out_dtype=torch.float32)
    part = torch.bmm(g2d.view(G * S, Pg // S, K).transpose(1, 2), x2d.view(G * S, Pg // S, C),
                     out_dtype=torch.float32)
    if into is not None and part.is_cuda and into.stride(-1) == 1 and into.stride(-2) == C:
        # one native pass: the splits summed in order and added into the flat
        # (or per-group) gradient (csrc/im2col.hip; was a reduce + an add kernel)
        _ops().wgrad_rsc_add(into.view(G, K, C), part, S, C, 1, True)
        return into
    if S > 1:
        part = part.view(G, S, K, C).sum(1)
    part = part.view(G, K, C) if G > 1 else part.view(K, C)
    if into is not None:
        return into.add_(part)
    return part


class _Conv1x1(torch.autograd.Function):
    """1x1 conv as a GEMM on the NHWC image; with stride s the subsampled
    input is a 1x1 column image (csrc/im2col.hip) and the input gradient
    comes back through the col2im gather (zeros off the stride grid), both
    single native passes."""

    @staticmethod
    def forward(ctx, x, weight, stride, gg):
        n, c, H, W = x.shape
        k = weight.shape[0]
        if stride > 1:
            x2d = _ops().im2col(x, 1, 1, stride, 0, c)
            h, w = (H - 1) // stride + 1, (W - 1) // stride + 1
        else:
            x2d, h, w = _nhwc2d(x), H, W
        wb = _prep1(weight, k, c)
        y2d = _mm_nt_conv(x2d, wb)
        ctx.save_for_backward(x2d, wb)
        ctx.weight, ctx.stride, ctx.gg = weight, stride, gg
        ctx.dims = (n, c, H, W, h, w)
        return y2d.view(n, h, w, k).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        x2d, wb = ctx.saved_tensors
        n, c, H, W, h, w = ctx.dims
        k = wb.shape[0]
        g2d = _nhwc2d(gy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        gw = None
        if ctx.needs_input_grad[1]:  # (first: on the side lane it overlaps the dgrad)
            with _wlane(ctx.weight, ctx.gg, g2d, x2d):
                gw = _wgrad_1x1(ctx.weight, ctx.gg, g2d, x2d, k, c)
        gx = None
        if ctx.needs_input_grad[0]:
            gsub = _mm_nn(g2d, wb)
            s = ctx.stride
            if s > 1:
                gx = _ops().col2im(gsub, n, H, W, c, 1, 1, s, 0)
            else:
                gx = gsub.view(n, h, w, c).permute(0, 3, 1, 2)
        return gx, gw, None, None


class _Conv1x1Pass(torch.autograd.Function):
    """(conv1x1(x), x) for a residual block whose input also feeds the
    identity branch: backward receives both gradients and sums them inside
    the dgrad GEMM (D = dY W + dX_identity, beta = 1) instead of a separate
    autograd accumulation pass over the block input."""

    @staticmethod
    def forward(ctx, x, weight, gg):
        n, c, h, w = x.shape
        k = weight.shape[0]
        wb = _prep1(weight, k, c)
        y2d = _mm_nt_conv(_nhwc2d(x), wb)
        ctx.save_for_backward(x, wb)
        ctx.weight, ctx.gg = weight, gg
        return y2d.view(n, h, w, k).permute(0, 3, 1, 2), x.view_as(x)

    @staticmethod
    def backward(ctx, gy, gid):
        x, wb = ctx.saved_tensors
        n, c, h, w = x.shape
        k = wb.shape[0]
        g2d = _nhwc2d(gy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        gw = None
        if ctx.needs_input_grad[1]:
            x2d = _nhwc2d(x)
            with _wlane(ctx.weight, ctx.gg, g2d, x2d):
                gw = _wgrad_1x1(ctx.weight, ctx.gg, g2d, x2d, k, c)
        gx = None
        if ctx.needs_input_grad[0]:
            if gid is not None:
                gi = _nhwc2d(gid.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
                if getattr(gid, "_commeff_fresh", False) and gi.data_ptr() == gid.data_ptr():
                    # the identity gradient is the residual BN backward's fresh
                    # dadd, consumed only here: accumulate into it in place (an
                    # out-of-place addmm first copies it: ~36 us per block of a
                    # ResNet-101 round)
                    gx2d = _mm_nn(g2d, wb, gi, in_place=True)
                else:
                    # autograd may hand the same tensor to another consumer
                    # (unfused relu(y + addend) path): never write into it
                    gx2d = _mm_nn(g2d, wb, gi)
            else:
                gx2d = _mm_nn(g2d, wb)
            gx = gx2d.view(n, h, w, c).permute(0, 3, 1, 2)
        return gx, gw, None


def _wgrad_1x1(ctx_weight, gg, g2d, x2d, k, c):
    """dW of a 1x1 conv into its grouped rows / flat .grad (None) or returned."""
    if gg is not None:
        _wgrad_gemm(g2d, x2d, gg.view(ctx_weight).view(gg.G, k, c), gg.G)
        return None
    into = _grad_view(ctx_weight, (k, c))
    gw = _wgrad_gemm(g2d, x2d, into)
    if into is not None:
        _grad_written(ctx_weight)
        return None
    return gw.view(k, c, 1, 1)


class _Conv1x1Pair(torch.autograd.Function):
    """(conv1x1(x, w1), conv1x1_stride_s(x, w2)): a downsampling bottleneck's
    conv1 and shortcut conv read the same input; backward writes the
    shortcut's input gradient (col2im onto the stride grid when s > 1) and the
    conv1 dgrad GEMM accumulates into it in place -- no autograd accumulation
    pass over the block input (4 stock bf16 adds per ResNet-101 round, 377 us)."""

    @staticmethod
    def forward(ctx, x, w1, w2, stride, gg1, gg2):
        n, c, H, W = x.shape
        k1, k2 = w1.shape[0], w2.shape[0]
        x2d = _nhwc2d(x)
        w1b, w2b = _prep1(w1, k1, c), _prep1(w2, k2, c)
        y1 = _mm_nt_conv(x2d, w1b)
        st1, _EPI["last"] = _EPI["last"], None
        if stride > 1:
            xs = _ops().im2col(x, 1, 1, stride, 0, c)
            h, w = (H - 1) // stride + 1, (W - 1) // stride + 1
        else:
            xs, h, w = x2d, H, W
        y2 = _mm_nt_conv(xs, w2b)
        # (the outputs' GEMM-epilogue BN moments, attached by conv1x1_pair)
        _EPI["pair"], _EPI["last"] = (st1, _EPI["last"]), None
        ctx.save_for_backward(x2d, xs, w1b, w2b)
        ctx.w, ctx.gg, ctx.stride, ctx.dims = (w1, w2), (gg1, gg2), stride, (n, c, H, W, h, w)
        return (y1.view(n, H, W, k1).permute(0, 3, 1, 2), y2.view(n, h, w, k2).permute(0, 3, 1, 2))

    @staticmethod
    def backward(ctx, g1, g2):
        x2d, xs, w1b, w2b = ctx.saved_tensors
        n, c, H, W, h, w = ctx.dims
        k1, k2 = w1b.shape[0], w2b.shape[0]
        s = ctx.stride

        def flat2d(g):
            return _nhwc2d(g.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        g1d = flat2d(g1) if g1 is not None else None
        g2d = flat2d(g2) if g2 is not None else None
        gw1 = gw2 = None
        if ctx.needs_input_grad[1] and g1d is not None:
            with _wlane(ctx.w[0], ctx.gg[0], g1d, x2d):
                gw1 = _wgrad_1x1(ctx.w[0], ctx.gg[0], g1d, x2d, k1, c)
        if ctx.needs_input_grad[2] and g2d is not None:
            with _wlane(ctx.w[1], ctx.gg[1], g2d, xs):
                gw2 = _wgrad_1x1(ctx.w[1], ctx.gg[1], g2d, xs, k2, c)
        gx = None
        if ctx.needs_input_grad[0]:
            acc = None
            if g2d is not None:
                gsub = _mm_nn(g2d, w2b)
                acc = _ops().col2im(gsub, n, H, W, c, 1, 1, s, 0) if s > 1 else gsub
                acc2d = _nhwc2d(acc) if s > 1 else acc
            if g1d is not None:
                acc2d = _mm_nn(g1d, w1b, acc2d, in_place=True) if acc is not None else _mm_nn(g1d, w1b)
            gx = acc2d.view(n, H, W, c).permute(0, 3, 1, 2)
        return gx, gw1, gw2, None, None, None


def conv1x1_pair(x, w1, w2, stride: int, gg1=None, gg2=None):
    """(conv1x1(x, w1), conv1x1(x, w2, stride)) with one input gradient pass."""
    _EPI["last"] = _EPI["pair"] = None
    y1, y2 = _Conv1x1Pair.apply(x, w1, w2, int(stride), gg1, gg2)
    sts, _EPI["pair"] = _EPI["pair"], None
    for y, st in zip((y1, y2), sts or (None, None)):
        _EPI["last"] = st
        _with_bnstats(y)
    return y1, y2


def conv1x1_passthrough(x, weight, gg=None):
    """(conv1x1(x, weight), x) with the two input gradients summed in one GEMM."""
    _EPI["last"] = None
    y, xi = _Conv1x1Pass.apply(x, weight, gg)
    return _with_bnstats(y), xi


def _wgrad_mopen(g, x, weight, stride, padding, dilation, groups):
    """MIOpen weight gradient (fp32) of one conv."""
    return torch.ops.aten.convolution_backward(
        g, x, weight.detach().to(g.dtype), None, list(stride), list(padding), list(dilation), False,
        [0, 0], groups, [False, True, False])[1].float()


def _grouped_wgrad_slices(g, x, gview, fn):
    """Per-group weight gradients from each group's slice of the batch."""
    G = gview.shape[0]
    ng = g.shape[0] // G
    for j in range(G):
        fn(g[j * ng:(j + 1) * ng], x[j * ng:(j + 1) * ng], gview[j])


class _Conv3x3(torch.autograd.Function):
    """conv3x3 (stride 1, pad 1, no bias) on the native MFMA kernels."""

    @staticmethod
    def forward(ctx, x, weight, gg):
        wf, wt = _prep(weight)
        ctx.save_for_backward(x, wt)
        ctx.weight, ctx.gg = weight, gg
        return _ops().conv3x3_fwd(x, wf, False)

    @staticmethod
    def backward(ctx, gy):
        x, wt = ctx.saved_tensors
        g = gy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        gw = None
        if ctx.needs_input_grad[1]:  # (first: on the side lane it overlaps the dgrad)
            w = ctx.weight
            native = w.shape[0] % 128 == 0  # the native wgrad tiles need K % 128 == 0
            if native and ctx.gg is not None:
                # every group's split-K slabs in one launch + a per-group reduction
                gv = ctx.gg.view(w)
                with _lanes.fork(g, x):
                    _ops().conv3x3_wgrad_grouped(g, x, gv.shape[0], gv.view(gv.shape[0], -1))
            elif native:
                gw = _wgrad_to(g, x, w)
            elif (_IMP_COL[0] and _GEMM_NATIVE[0] and x.shape[1] % 8 == 0 and _gpu_bf16_nhwc(x)
                  and x.data_ptr() % 16 == 0 and (ctx.gg is None or x.shape[0] % ctx.gg.G == 0)):
                # K % 128 != 0: the TN GEMM over the implicit column image of x
                g2 = _nhwc2d(g)
                with _wlane(w, ctx.gg, g2, x):
                    gw = _col_wgrad(g2, x, w, ctx.gg, (1, 1))
            else:  # column-image GEMM (csrc/im2col.hip)
                col = _ops().im2col(x, 3, 3, 1, 1, 9 * x.shape[1])
                g2 = _nhwc2d(g)
                with _wlane(w, ctx.gg, g2, col):
                    gw = _col_wgrad(g2, col, w, ctx.gg)
        gx = _ops().conv3x3_fwd(g, wt, False) if ctx.needs_input_grad[0] else None
        return gx, gw, None


def _col_width(C: int, R: int, S: int) -> int:
    """Column-image row length: R*S*C rounded up to 64 on the native GEMMs (a
    whole number of their 64-deep K-steps: the 7x7 stem's 147 columns -> 192,
    its forward then the native NT GEMM instead of hipBLASLt), else to 8
    (16-byte rows)."""
    q = 64 if _GEMM_NATIVE[0] else 8
    return -(-C * R * S // q) * q


def _col_image(weight: torch.Tensor, Kc: int) -> torch.Tensor:
    """bf16 [K, Kc] GEMM image of ``weight`` with (r, s, c) columns -- for a
    3x3 with C % 64 == 0 the forward image of ``prepared_conv_weights`` when
    this pass prepared it (same layout), else one conversion kernel."""
    K, C, R, S = weight.shape
    if (R, S) == (3, 3) and Kc == 9 * C:
        hit = _PREP.get((weight.data_ptr(), weight._version))
        if hit is not None:
            return hit[0].view(K, Kc)
    return _ops().conv_weight_rsc(weight.detach().contiguous(), Kc)


def _col_wgrad(g2d: torch.Tensor, col: torch.Tensor, weight: torch.Tensor, gg, imp=None):
    """dW of a column-image conv: split-K GEMMs of g2d^T col, then one native
    pass that sums the splits in order, permutes (r, s, c) -> (c, r, s) and
    accumulates into the flat fp32 gradient (or the per-group rows of
    ``gg``).  Returns the gradient for autograd, None when accumulated.
    ``imp`` (stride, pad): ``col`` is the conv's input image and the native TN
    GEMM gathers its column image per tap (no im2col)."""
    K, C, R, S = weight.shape
    G = gg.G if gg is not None else 1
    if imp is not None:
        parts, splits = _ops().gemm_tn_parts_imp(g2d, col, G, R, imp[0], imp[1])
    else:
        parts, splits = _wgrad_parts(g2d, col, G)
    if gg is not None:
        _ops().wgrad_rsc_add(gg.view(weight).view(G, K, C * R * S), parts, splits, C, R * S, True)
        return None
    into = _grad_view(weight, (1, K, C * R * S))
    dst = into if into is not None else torch.empty(1, K, C * R * S, dtype=torch.float32,
                                                     device=g2d.device)
    _ops().wgrad_rsc_add(dst, parts, splits, C, R * S, into is not None)
    if into is not None:
        _grad_written(weight)
        return None
    return dst.view(weight.shape)


class _ConvCol(torch.autograd.Function):
    """Bias-free, ungrouped conv of a bf16 channels-innermost activation as an
    explicit GEMM over its bf16 column image (csrc/im2col.hip): the 7x7/s2
    stem (3 channels, any pixel stride: no dgrad, the input is data), the
    strided 3x3 of each ResNet stage's first bottleneck, any other kernel size.
    The column image is kept for the weight gradient instead of the input."""

    @staticmethod
    def forward(ctx, x, weight, stride, pad, gg):
        K, C, R, S = weight.shape
        N, _, H, W = x.shape
        Kc = _col_width(C, R, S)
        wt = _col_image(weight, Kc)
        OH, OW = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
        # implicit column image (the strided 3x3 of each stage's first block):
        # the native NT GEMM gathers it per tap from x, the weight gradient's
        # TN GEMM likewise; x is kept instead of the 9x larger image
        imp = (_IMP_COL[0] and _GEMM_NATIVE[0] and R == S and Kc == R * S * C and C % 64 == 0
               and K % 64 == 0 and _gpu_bf16_nhwc(x) and x.data_ptr() % 16 == 0
               and (gg is None or N % gg.G == 0))
        if imp:
            G, M = _EPI["G"], N * OH * OW
            st_on = _EPI["on"] and G >= 1 and M % G == 0 and M // G >= 128
            y2d, st = _ops().conv_nt_imp(x, wt, R, stride, pad, G if st_on else 0)
            if st_on:
                _EPI["last"] = (st, G)
            ctx.save_for_backward(x, wt)
        else:
            col = _ops().im2col(x, R, S, stride, pad, Kc)
            y2d = _mm_nt_conv(col, wt)
            ctx.save_for_backward(col, wt)
        ctx.imp = imp
        ctx.geo = (N, C, H, W, R, S, stride, pad)
        ctx.weight, ctx.gg = weight, gg
        return y2d.view(N, OH, OW, K).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        col, wt = ctx.saved_tensors
        N, C, H, W, R, S, stride, pad = ctx.geo
        g2d = _nhwc2d(gy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        gw = None
        if ctx.needs_input_grad[1]:
            with _wlane(ctx.weight, ctx.gg, g2d, col):
                gw = _col_wgrad(g2d, col, ctx.weight, ctx.gg, (stride, pad) if ctx.imp else None)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = _ops().col2im(_mm_nn(g2d, wt), N, H, W, C, R, S, stride, pad)
        return gx, gw, None, None, None


# strided 3x3 convs on the implicit column image (False: im2col + GEMMs)
_IMP_COL = [True]


class _MaxPool(torch.autograd.Function):
    """k x k / stride s / padding p max-pool on NHWC bf16 (csrc/im2col.hip):
    1-byte window codes forward, a gather backward (no atomics, no zero fill)."""

    @staticmethod
    def forward(ctx, x, k, s, p):
        y, codes = _ops().maxpool_fwd(x, k, s, p)
        ctx.save_for_backward(codes)
        ctx.conf = (x.shape[2], x.shape[3], k, s, p)
        return y

    @staticmethod
    def backward(ctx, gy):
        (codes,) = ctx.saved_tensors
        H, W, k, s, p = ctx.conf
        return _ops().maxpool_bwd(gy.to(torch.bfloat16), codes, H, W, k, s, p), None, None, None


def maxpool_native_ok(x: torch.Tensor, k: int, s: int, p: int) -> bool:
    return (not _STOCK[0] and _gpu_bf16_nhwc(x) and x.shape[1] % 8 == 0 and 1 <= k <= 15
            and s >= 1 and 0 <= 2 * p <= k)


def max_pool2d(x: torch.Tensor, k: int, s: int, p: int = 0) -> torch.Tensor:
    """``F.max_pool2d(x, k, s, p)`` on the native kernels when they apply."""
    if maxpool_native_ok(x, k, s, p):
        return _MaxPool.apply(x, int(k), int(s), int(p))
    return F.max_pool2d(x, k, s, p)


class _ConvGrouped(torch.autograd.Function):
    """Any convolution (MIOpen) with per-group weight gradients."""

    @staticmethod
    def forward(ctx, x, weight, stride, padding, dilation, groups, gg):
        wc = weight.detach().to(x.dtype)
        ctx.save_for_backward(x, wc)
        ctx.conf = (tuple(stride), tuple(padding), tuple(dilation), groups)
        ctx.weight, ctx.gg = weight, gg
        return F.conv2d(x, wc, None, stride, padding, dilation, groups)

    @staticmethod
    def backward(ctx, gy):
        x, wc = ctx.saved_tensors
        stride, padding, dilation, groups = ctx.conf
        g = gy.to(x.dtype)
        if x.is_cuda and x.is_contiguous(memory_format=torch.channels_last):
            g = g.contiguous(memory_format=torch.channels_last)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.ops.aten.convolution_backward(
                g, x, wc, None, list(stride), list(padding), list(dilation), False, [0, 0], groups,
                [True, False, False])[0]
        _grouped_wgrad_slices(g, x, ctx.gg.view(ctx.weight),
                              lambda gs, xs, dst: dst.add_(
                                  _wgrad_mopen(gs, xs, wc, stride, padding, dilation, groups)))
        return gx, None, None, None, None, None, None


def _gpu_bf16_nhwc(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last))


def conv2d_native_kind(x: torch.Tensor, weight: torch.Tensor, stride, padding, dilation,
                       groups) -> str:
    """Which native path serves this convolution: "1x1", "3x3", "col" (column
    image) or "" (MIOpen)."""
    if _CONV_BACKEND[0] != "native" or _STOCK[0] or groups != 1:
        return ""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.stride(1) == 1):
        return ""
    if weight.dtype != torch.float32 or weight.dim() != 4 or weight.shape[1] != x.shape[1]:
        return ""
    kh, kw = weight.shape[2], weight.shape[3]
    s = stride if isinstance(stride, int) else (stride[0] if stride[0] == stride[1] else -1)
    p = padding if isinstance(padding, int) else (padding[0] if padding[0] == padding[1] else -1)
    dl = dilation if isinstance(dilation, int) else (dilation[0] if dilation[0] == dilation[1]
                                                     else -1)
    if dl != 1 or s < 1 or p < 0:
        return ""
    C, K = x.shape[1], weight.shape[0]
    dense = x.is_contiguous(memory_format=torch.channels_last)
    if dense and (kh, kw) == (1, 1) and p == 0 and C % 8 == 0 and K % 8 == 0:
        return "1x1"
    if dense and (kh, kw) == (3, 3) and s == 1 and p == 1 and C % 64 == 0 and K % 64 == 0:
        return "3x3"
    if K % 8 == 0 and p < kh and p < kw and x.stride(3) >= C and (
            (dense and C % 8 == 0) or not x.requires_grad):
        # the col2im dgrad gather needs C % 8 == 0; a data input needs none
        return "col"
    return ""


def conv2d_native(x: torch.Tensor, weight: torch.Tensor, kind: str, stride: int = 1, gg=None,
                  padding: int = 0):
    _EPI["last"] = None
    if kind == "1x1":
        return _with_bnstats(_Conv1x1.apply(x, weight, int(stride), gg))
    if kind == "col":
        return _with_bnstats(_ConvCol.apply(x, weight, int(stride), int(padding), gg))
    return _Conv3x3.apply(x, weight, gg)


def conv2d_grouped(x, weight, stride, padding, dilation, groups, gg):
    """Convolution whose weight gradient goes to the per-group rows of ``gg``."""
    if weight.dtype != x.dtype and not torch.is_autocast_enabled(x.device.type):
        x = x.to(weight.dtype)
    elif torch.is_autocast_enabled(x.device.type) and x.is_floating_point():
        x = x.to(torch.get_autocast_dtype(x.device.type))
    return _ConvGrouped.apply(x, weight, stride, padding, dilation, groups, gg)


# ------------------------------------------------------------ grouped linear
class _LinearGrouped(torch.autograd.Function):
    """y = x W^T + b with per-group dW / db (batched GEMM over the groups)."""

    @staticmethod
    def forward(ctx, x, weight, bias, gg):
        wc = weight.detach().to(x.dtype)
        ctx.save_for_backward(x, wc)
        ctx.params, ctx.gg = (weight, bias), gg
        y = F.linear(x, wc, None if bias is None else bias.detach().to(x.dtype))
        return y

    @staticmethod
    def backward(ctx, gy):
        x, wc = ctx.saved_tensors
        weight, bias = ctx.params
        gg = ctx.gg
        G = gg.G
        g = gy.to(x.dtype)
        gx = g.matmul(wc) if ctx.needs_input_grad[0] else None
        out_f, in_f = wc.shape
        g2d, x2d = g.reshape(-1, out_f), x.reshape(-1, in_f)
        gw = gg.view(weight)
        if g2d.is_cuda and g2d.dtype == torch.bfloat16:
            _wgrad_gemm(g2d, x2d, gw, G)
        else:
            gw.add_(torch.bmm(g2d.view(G, -1, out_f).transpose(1, 2).float(),
                              x2d.view(G, -1, in_f).float()))
        if bias is not None:
            gw_b = gg.view(bias)
            gw_b.add_(g2d.view(G, -1, out_f).float().sum(1))
        return gx, None, None, None


def linear_grouped(x, weight, bias, gg):
    if torch.is_autocast_enabled(x.device.type) and x.is_floating_point():
        x = x.to(torch.get_autocast_dtype(x.device.type))
    elif x.dtype != weight.dtype:
        x = x.to(weight.dtype)
    return _LinearGrouped.apply(x, weight, bias, gg)


# ------------------------------------------------------------ grouped affine
class _AffineGrouped(torch.autograd.Function):
    """y = xhat * w + b per channel (dim 1) of an [N, C, ...] tensor, with
    per-group dw / db: the torch fallback of ghost BN under grouped grads."""

    @staticmethod
    def forward(ctx, xhat, weight, bias, gg):
        shape = [1, -1] + [1] * (xhat.dim() - 2)
        ctx.save_for_backward(xhat, weight)
        ctx.params, ctx.gg = (weight, bias), gg
        return xhat * weight.view(shape) + bias.view(shape)

    @staticmethod
    def backward(ctx, gy):
        xhat, weight = ctx.saved_tensors
        w, b = ctx.params
        G = ctx.gg.G
        shape = [1, -1] + [1] * (xhat.dim() - 2)
        red = [1] + list(range(3, xhat.dim() + 1))
        gyf = gy.float()
        gw = (gyf * xhat.float()).reshape(G, -1, *xhat.shape[1:]).sum(dim=red)
        gb = gyf.reshape(G, -1, *xhat.shape[1:]).sum(dim=red)
        ctx.gg.view(w).add_(gw)
        ctx.gg.view(b).add_(gb)
        return gy * weight.view(shape).to(gy.dtype), None, None, None


# ------------------------------------------------------------------------
# Batched FedAvg: per-client 3x3 convolutions on native kernels under vmap.
#
# The lockstep local SGD of a rank's G clients (parallel/fed_model.py
# _fedavg_batched) runs ONE torch.func.vmap(grad(loss)) per local step over a
# [G, d] stack of client weights; the model's ops take their stock PyTorch
# form there (stock_ops), and vmap turns every conv into a grouped MIOpen
# convolution (column images + GEMMs: ~90 of the 169 ms of a ResNet-18
# CIFAR-100 round of 100 clients x 5 local steps, profiles/r4_experiments.md).
# Inside ``vmap_native_convs()`` the stride-1 3x3 convs instead go through
# _GConv3x3, whose vmap rule stacks the clients along channels -- x [n, G C,
# H, W], weight [G kg, C, 3, 3] -- and runs the grouped halo kernels
# (csrc/conv.hip: each output-channel tile reads its own group's input
# channels and weight rows): forward, input gradient (the same kernel on the
# per-group flipped weights) and, where the halo wgrad tiles fit, the weight
# gradient; other shapes fall back to the grouped stock convolution.
_VMAP_NATIVE = [False]


class vmap_native_convs:
    """Opt-in (COMMEFF_GCONV=1): measured 174.8 vs 165.8 ms per ResNet-18
    CIFAR-100 FedAvg round (100 clients x 5 local steps) -- the grouped halo
    kernels replace ~45 ms of MIOpen column-image convolutions, but the round
    is bound by vmap's host time (GPU idle ~40 ms/round), the stock
    BatchNorm / elementwise work between the convs, the layout copies into the
    channel-stacked form, and the weight gradients of the 64-channel and
    8x8 / 4x4 layers, which have no grouped halo wgrad tiling yet and take the
    grouped stock path (profiles/r4_experiments.md)."""

    def __init__(self, enabled: bool = True):
        self.enabled = bool(enabled) and os.environ.get("COMMEFF_GCONV", "0") == "1"

    def __enter__(self):
        self.prev = _VMAP_NATIVE[0]
        _VMAP_NATIVE[0] = self.enabled
        return self

    def __exit__(self, *exc):
        _VMAP_NATIVE[0] = self.prev
        return False


def vmap_native_active() -> bool:
    return _VMAP_NATIVE[0]


def _bstack(t, bdim, B):
    return t.movedim(bdim, 0) if bdim is not None else t.unsqueeze(0).expand(B, *t.shape)


def _chan_stack(X):
    """[B, n, C, H, W] -> [n, B C, H, W] with channels_last memory (clients
    along channels): ONE copy into the kernels' [n, H, W, B C] layout."""
    B, n, C, H, W = X.shape
    return X.permute(1, 3, 4, 0, 2).contiguous().view(n, H, W, B * C).permute(0, 3, 1, 2)


def _chan_unstack(y, B):
    """[n, B K, H, W] (channels_last) -> [B, n, K, H, W] contiguous: one copy,
    so the stock ops between the convs (BatchNorm, ReLU, residual adds) run on
    dense per-client tensors instead of strided ones (their non-vectorised
    kernels cost more than the copy, r4 log)."""
    n, BK, H, W = y.shape
    return y.view(n, B, BK // B, H, W).transpose(0, 1).contiguous()


def _gconv_native_ok(x, G, C, kg) -> bool:
    return (x.is_cuda and _CONV_BACKEND[0] == "native" and C % 64 == 0 and kg % 64 == 0)


def _gconv_fwd(x, w, G):
    """y = grouped 3x3 conv (stride 1, pad 1) of x [n, G C, H, W] with w
    [G kg, C, 3, 3]: the grouped native kernel or the stock grouped conv."""
    C, kg = x.shape[1] // G, w.shape[0] // G
    if _gconv_native_ok(x, G, C, kg):
        xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wf = w.detach().to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()  # [G kg, 3, 3, C]
        y = _ops().conv3x3_fwd_grouped(xb, wf, G)
        if y.numel() or xb.numel() == 0:
            return y
    return F.conv2d(x, w.to(x.dtype), padding=1, groups=G)


class _GConv3x3Bwd(torch.autograd.Function):
    """(dx, dw) of _GConv3x3 (its own Function so vmap can stack it too)."""

    @staticmethod
    def forward(gy, x, w, G):
        C, kg = x.shape[1] // G, w.shape[0] // G
        if _gconv_native_ok(gy, G, C, kg):
            gyb = gy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            # per-group flipped, transposed weights [G C, 3, 3, kg]: the bf16
            # cast, then one flip of the permuted view (a contiguous result)
            wt = (w.detach().to(torch.bfloat16).view(G, kg, C, 3, 3).permute(0, 2, 3, 4, 1)
                  .flip(2, 3).reshape(G * C, 3, 3, kg))
            gx = _ops().conv3x3_fwd_grouped(gyb, wt, G)
            if gx.numel() == 0 and gyb.numel():
                gx = torch.nn.grad.conv2d_input(x.shape, w.to(gy.dtype), gy, padding=1, groups=G)
            gw = _ops().conv3x3_wgrad_grouped_ch(gyb, xb, G)
            if gw.numel() == 0 and xb.numel():
                gw = torch.nn.grad.conv2d_weight(xb, w.shape, gyb, padding=1, groups=G)
            return gx.to(x.dtype), gw.to(w.dtype)
        gx = torch.nn.grad.conv2d_input(x.shape, w.to(gy.dtype), gy, padding=1, groups=G)
        gw = torch.nn.grad.conv2d_weight(x.to(gy.dtype), w.shape, gy, padding=1, groups=G)
        return gx.to(x.dtype), gw.to(w.dtype)

    @staticmethod
    def setup_context(ctx, inputs, output):
        pass

    @staticmethod
    def backward(ctx, ggx, ggw):
        raise RuntimeError("_GConv3x3: no double backward")

    @staticmethod
    def vmap(info, in_dims, gy, x, w, G):
        B = info.batch_size
        bg, bx, bw, _ = in_dims
        GY, X, Wt = _bstack(gy, bg, B), _bstack(x, bx, B), _bstack(w, bw, B)
        gx, gw = _GConv3x3Bwd.apply(_chan_stack(GY), _chan_stack(X),
                                    Wt.reshape(B * Wt.shape[1], *Wt.shape[2:]), B * G)
        return (_chan_unstack(gx, B), gw.view(B, -1, *gw.shape[1:])), (0, 0)


class _GConv3x3(torch.autograd.Function):
    """Grouped stride-1 3x3 conv (G groups) whose vmap rule folds the vmapped
    dimension into the groups (clients stacked along channels)."""

    @staticmethod
    def forward(x, w, G):
        return _gconv_fwd(x, w, G)

    @staticmethod
    def setup_context(ctx, inputs, output):
        x, w, G = inputs
        ctx.save_for_backward(x, w)
        ctx.G = G

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx, gw = _GConv3x3Bwd.apply(gy, x, w, ctx.G)
        return gx, gw, None

    @staticmethod
    def vmap(info, in_dims, x, w, G):
        bx, bw, _ = in_dims
        B = info.batch_size
        X, Wt = _bstack(x, bx, B), _bstack(w, bw, B)
        y = _GConv3x3.apply(_chan_stack(X), Wt.reshape(B * Wt.shape[1], *Wt.shape[2:]), B * G)
        return _chan_unstack(y, B), 0


def gconv3x3(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """A stride-1, pad-1, bias-free 3x3 conv that becomes the grouped native
    kernel when vmapped over clients (see vmap_native_convs)."""
    return _GConv3x3.apply(x, weight, 1)
