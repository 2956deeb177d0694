"""Native batched FedAvg local SGD of a ResNet-18 round: G clients as ONE
explicit program (no vmap, no MIOpen, no stock elementwise ops in the loop).

Reference semantics: /root/reference/CommEfficient/fed_worker.py:61-113 --
every client copies the server weights, takes ``num_fedavg_epochs`` passes of
local SGD over its own data (gradient clipping to ``max_grad_norm``, weight
decay ``wd / num_workers`` at the client's current weights, step
``lr * decay**step``; utils.py:257-258, fed_worker.py:288-292) and uploads
``n (w0 - w)``.  Model: /root/reference/CommEfficient/models/fixup_resnet18.py
(the ResNet18 of models/fixup.py with --batchnorm): stem conv3x3 + ReLU,
PreActBlocks ``relu(bn1(conv1 x)) -> relu(bn2(conv2 .)) + shortcut(x)``, head
``linear(avg(x) || max(x))``.

Layout (MI355X-first):

* The G clients' weights are the rows of one fp32 [G, ld] matrix ``Wg``; their
  gradients the rows of ``Gg``.  Every kernel reads / writes its client's
  parameters in place -- weight gradients land in their rows directly (no
  per-parameter concatenation), one per-row clip + weight-decay + SGD kernel
  updates every client (csrc/fedavg.hip), and the first local step reads the
  server weights as a broadcast row (no G-fold copy).
* Activations are channel-stacked: [n, G*C, H, W] channels_last, i.e. each
  pixel row holds the G clients' C channels side by side.  The stride-1 3x3
  convolutions are the grouped halo MFMA kernels of csrc/conv.hip (forward,
  and the input gradient on per-client flipped weights; the weight gradient
  where a grouped halo tiling exists); batch norm is per channel, i.e. per
  (client, channel) -- each client normalises with its own batch statistics
  and keeps its own running statistics (csrc/bn.hip, channel-stacked path);
  the strided convolutions and 1x1 shortcuts are grouped column images
  (csrc/im2col.hip) times per-client weight images in strided-batched
  library GEMMs (the shortcut reads the column image's centre tap, which IS
  the stride-2 subsampled input, and its input gradient is added into that
  tap before the one col2im gather).
* The head pools the 4x4 maps of all clients in one kernel into per-client
  [n, 512] fp32 features; the classifier is a batched fp32 GEMM on the
  weight rows themselves.

``supported(model, args)`` says whether a model / configuration runs here;
FedModel falls back to the vmap composition otherwise.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch

from .. import _ext
from ..ops import lanes as _lanes


def _ops():
    return _ext.ops()


def _step_means(ts: List[torch.Tensor]) -> torch.Tensor:
    """Per-client mean over the local steps of the per-step means of [G, n_s]
    tensors: one stack + mean when every step has the same n (no per-step
    reduction kernels)."""
    if all(t.shape == ts[0].shape for t in ts):
        return torch.stack(ts).mean(dim=(0, 2))
    return sum(t.mean(1) for t in ts) / len(ts)


def _gview(t: torch.Tensor, G: int) -> torch.Tensor:
    """[n, G*K, H, W] channels_last -> [G, n*H*W, K] strided view (per-client
    GEMM operand / output: batch stride K, row stride G*K)."""
    n, GK, H, W = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * H * W, G, GK // G).transpose(0, 1)


# (the strided convs' forward / input gradients and the 4x4 input gradients on
# the native grouped GEMM: 29.64 vs 29.82 ms per round on hipBLASLt's strided
# batched GEMMs, same-box A/B)
_NATIVE_GMM = [True]


def _gmm(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor, nn: bool, beta: float = 0.0) -> None:
    """out_g = A_g op(B_g) (+ beta out_g), bf16, for every client g: the native
    grouped MFMA GEMM when the shapes allow it, else (b)addbmm.  nt: B_g is
    [N, K] (out = A B^T); nn: B_g is [K, N]."""
    if _NATIVE_GMM[0] and _ops().fa_gemm(A, B, out, nn, beta):
        return
    Bm = B if nn else B.transpose(1, 2)
    if beta:
        torch.baddbmm(out, A, Bm, beta=beta, out=out)
    else:
        torch.bmm(A, Bm, out=out)


def _carrier(x: torch.Tensor, G: int, P: int, N: int) -> torch.Tensor:
    """A [G, P, N] bf16 shape carrier (no storage) for an implicit column image"""
    return torch.empty((1, 1, 1), device=x.device, dtype=torch.bfloat16).expand(G, P, N)


class _Sink:
    """Where one local step's weight gradients go: rows ``dst`` (ld apart)
    receive ``beta * dst + alpha * grad`` -- the gradient rows (beta 0, alpha
    1; a per-row SGD kernel follows, needed for clipping) or the weight rows
    themselves (beta = 1 - lr wd, alpha = -lr: the SGD step fused into every
    producer), with the bf16 ``mirror`` of the updated weights.  ``src`` (sld
    apart, 0: one shared row) holds the weights the step starts from -- the
    first local step reads the server row there instead of a broadcast copy
    of it in ``dst``."""
    __slots__ = ("dst", "ld", "beta", "alpha", "mirror", "src", "sld")

    def __init__(self, dst, ld, beta, alpha, mirror, src=None, sld=0):
        self.dst, self.ld, self.beta, self.alpha, self.mirror = dst, ld, float(beta), float(alpha), mirror
        self.src, self.sld = src, int(sld)

    def src_rows(self, off, K, n):
        """[G, K, n] view of the weights ``beta`` scales (``dst``'s own without src)"""
        if self.src is None:
            return self.dst[:, off:off + K * n].view(-1, K, n)
        return ResNet18FedAvg._rows(self.src, self.sld, self.dst.shape[0], off, K, n)


class _Block:
    __slots__ = ("cin", "cout", "stride", "bn1w", "bn1b", "conv1", "bn2w", "bn2b", "conv2", "sc",
                 "m1", "m2")


class ResNet18FedAvg:
    """Explicit G-client forward / backward / local SGD of models.fixup.ResNet18
    (BatchNorm variant).  Construct once per FedModel; ``round(...)`` runs one
    pass of clients."""

    @staticmethod
    def supported(model, args) -> Tuple[bool, str]:
        from ..models.common import GhostBatchNorm2d
        from ..models.fixup import ResNet18
        if not isinstance(model, ResNet18):
            return False, "not the ResNet18 of models/fixup.py"
        if getattr(args, "dtype", "bf16") != "bf16":
            return False, "bf16 compute only"
        for m in model.modules():
            if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
                if not (isinstance(m, GhostBatchNorm2d) and m.affine and m.track_running_stats
                        and m.momentum is not None and m.fuse_relu):
                    return False, "BatchNorm layers must be affine GhostBatchNorm2d with ReLU"
        for p in model.parameters():
            if not p.requires_grad:
                return False, "frozen parameters"
        return True, ""

    def accepts(self, shape) -> Tuple[bool, str]:
        """Whether a client batch of this NCHW ``shape`` runs on the engine's
        kernels (checked before a round mutates anything): the input channels
        of the model's stem, and a final feature map of at most 256 pixels for
        the fused pooling head (fa_head_fwd / fa_head_bwd) -- e.g. 32 x 32
        CIFAR or 28 x 28 EMNIST images, not 224 x 224 ImageNet ones."""
        if len(shape) != 4:
            return False, f"input of shape {tuple(shape)}: NCHW images expected"
        _, c, h, w = shape
        if c != self.cin0:
            return False, f"{c} input channels, the stem takes {self.cin0}"
        for b in self.blocks:
            if b.stride == 2:
                h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        if h * w > 256:
            return False, f"final feature map {h}x{w} > 256 pixels (fused pooling head)"
        return True, ""

    def _aligned(self, names, flat) -> Dict[str, int]:
        """Internal row offsets: every parameter starts on a 16-byte boundary
        (the Fixup models' one-element scalars otherwise shift every conv
        weight off the kernels' 16-byte loads); the gaps are layout padding
        (perm -1: gathered as 0, never uploaded).  Sets the row length self.d."""
        off, segs, io = {}, [], 0
        for nm, fo, nel in zip(names, flat.offsets, flat.numels):
            off[nm] = io
            segs.append((io, int(fo), int(nel)))
            io += (int(nel) + 7) // 8 * 8
        self._segs = segs
        self.d = io
        return off

    def _perm_convs(self, device, convs) -> torch.Tensor:
        """int32 [d]: internal position -> flat coordinate (-1: padding); the
        3x3 conv weights ``convs`` (internal offset, K, C) in the kernels'
        (k, r, s, c) order, everything else in PyTorch's order."""
        if getattr(self, "_perm_t", None) is None or self._perm_t.device != device:
            import numpy as np
            perm = np.full(self.d, -1, dtype=np.int64)
            flat_of = {}
            for io, fo, nel in self._segs:
                perm[io:io + nel] = fo + np.arange(nel)
                flat_of[io] = fo
            for off, K, C in convs:
                # internal (k, t, c) <- PyTorch (k, c, t)
                k, t, c = np.meshgrid(np.arange(K), np.arange(9), np.arange(C), indexing="ij")
                perm[off:off + K * 9 * C] = flat_of[off] + ((k * C + c) * 9 + t).reshape(-1)
            self._perm_t = torch.from_numpy(perm.astype(np.int32)).to(device)
        return self._perm_t

    def __init__(self, model, flat, names: List[str]):
        self.model = model
        off = self._aligned(names, flat)
        self.off = off
        self.prep = off["prep.0.weight"]
        self.blocks: List[_Block] = []
        for li, layer in enumerate(model.layers):
            for bi, blk in enumerate(layer):
                p = f"layers.{li}.{bi}."
                b = _Block()
                b.cin, b.cout = blk.conv1.in_channels, blk.conv1.out_channels
                b.stride = blk.conv1.stride[0]
                b.bn1w, b.bn1b = off[p + "bn1.weight"], off[p + "bn1.bias"]
                b.bn2w, b.bn2b = off[p + "bn2.weight"], off[p + "bn2.bias"]
                b.conv1, b.conv2 = off[p + "conv1.weight"], off[p + "conv2.weight"]
                b.sc = off.get(p + "shortcut.0.weight")
                b.m1, b.m2 = blk.bn1, blk.bn2
                if b.sc is None and (b.stride != 1 or b.cin != b.cout):
                    raise ValueError("ResNet18FedAvg: block without a shortcut changes shape")
                if b.sc is not None and b.stride != 2:
                    raise ValueError("ResNet18FedAvg: stride-1 projection shortcuts are not wired")
                self.blocks.append(b)
        self.fc_w, self.fc_b = off["classifier.weight"], off["classifier.bias"]
        self.ncls = model.classifier.out_features
        self.feat = model.classifier.in_features
        self.c0 = model.prep[0].out_channels
        self.cin0 = model.prep[0].in_channels

    # ------------------------------------------------------------ layout
    def _perm(self, device) -> torch.Tensor:
        """int32 [d]: element j of a client row is flat coordinate perm[j].  The
        rows keep every 3x3 conv weight in the kernels' (k, r, s, c) order --
        the bf16 mirror then IS the grouped conv kernels' forward image and the column-GEMM image, and the weight
        gradients come out of the MFMA / GEMM reductions in that order -- and
        everything else in PyTorch's order."""
        convs = [(self.prep, self.c0, self.cin0)]
        for b in self.blocks:
            convs += [(b.conv1, b.cout, b.cin), (b.conv2, b.cout, b.cout)]
        return self._perm_convs(device, convs)

    _col_cache = None
    _col_ok = False

    def _stem_col(self, x: torch.Tensor, G: int, Kc0: int) -> torch.Tensor:
        """The stem's grouped column image of x; full-batch local steps read the
        same input every step, so it is built once per round (``run`` resets the
        cache)."""
        key = (x.data_ptr(), tuple(x.shape), tuple(x.stride()), G, Kc0)
        c = self._col_cache
        if self._col_ok and c is not None and c[0] == key:
            return c[1]
        col = _ops().im2col_grouped(x, G, 3, 3, 1, 1, Kc0, True)
        if self._col_ok:
            self._col_cache = (key, col)
        return col

    @staticmethod
    def _rows(Wt: torch.Tensor, ld: int, G: int, off: int, K: int, n: int) -> torch.Tensor:
        """[G, K, n] view of every client's [K][n] block at ``off`` (ld 0: the
        shared server row, batch stride 0)"""
        if ld:
            return Wt[:, off:off + K * n].view(G, K, n)
        return Wt[off:off + K * n].view(1, K, n).expand(G, K, n)

    # ----------------------------------------------------------- convs
    def _conv3(self, x, Wb, ldb, G, off, K, C):
        """stride-1 3x3 conv of channel-stacked x with the clients' weights"""
        # (4x4 maps too: the column-image GEMM measured slower here, 36.2 vs 35.8 ms)
        y = _ops().conv3x3_fwd_rows(x, Wb, G, off, ldb, K)
        if y.numel() == 0 and x.numel():  # no halo tiling: column image x weight rows
            col = _ops().im2col_grouped(x, G, 3, 3, 1, 1, 9 * C, False)
            n, _, H, Wd = x.shape
            y = torch.empty((n, G * K, H, Wd), device=x.device, dtype=torch.bfloat16,
                            memory_format=torch.channels_last)
            torch.bmm(col.transpose(0, 1), self._rows(Wb, ldb, G, off, K, 9 * C).transpose(1, 2),
                      out=_gview(y, G))
        return y

    def _conv3_dgrad(self, dy, Wb, ldb, G, off, K, C, addend=None):
        """input gradient of a stride-1 3x3 conv (+ ``addend``: the identity
        shortcut's gradient, fused into the halo kernel's epilogue)"""
        dx = torch.empty(0)
        # 4x4 maps: the column-image GEMM against the weight rows + col2im
        # (35.8 vs 36.3 ms per round against the halo kernel on a flipped
        # image; 29.69 vs 29.71 against the transposed-rows halo kernel)
        if dy.shape[3] >= 8:
            # the halo kernel reads the conv's own rows through transposed B
            # tiles (no flipped image per step)
            if C % 64 == 0 and self._DGRAD_BT[0]:
                dx = _ops().conv3x3_fwd_rows(dy, Wb, G, off, ldb, C, addend, True)
                if dx.numel():
                    return dx
            img = _ops().fa_dgrad_image(Wb, ldb, G, off, K, C)
            dx = _ops().conv3x3_fwd_rows(dy, img, G, 0, C * 9 * K if ldb else 0, C, addend)
            if dx.numel():
                return dx
        if dy.numel():
            n, _, H, Wd = dy.shape
            dcol = torch.empty((n * H * Wd, G, 9 * C), device=dy.device, dtype=torch.bfloat16)
            _gmm(_gview(dy, G), self._rows(Wb, ldb, G, off, K, 9 * C), dcol.transpose(0, 1), True)
            dx = _ops().col2im_grouped(dcol, G, n, H, Wd, C, 3, 3, 1, 1)
            if addend is not None:
                dx = _ops().fa_ew(dx, addend, 0)
        return dx

    # the per-client classifier step on the fused kernel (fedavg.hip
    # fa_linear_ce_kernel; COMMEFF_FA_HEAD=0: batched GEMMs + the loss kernel)
    _FUSED_HEAD = [os.environ.get("COMMEFF_FA_HEAD", "1") != "0"]

    def _fused_head_ok(self, n: int, F: int) -> bool:
        return self._FUSED_HEAD[0] and n <= 32 and n * (F + self.ncls) * 4 <= 96 * 1024

    # the stem's [64 x 27] weight updates on the TN GEMM too (COMMEFF_FA_STEM=blas: hipBLASLt)
    _STEM_TN = [os.environ.get("COMMEFF_FA_STEM", "tn") == "tn"]
    _BMM_INTO = [True]
    # (128-channel input gradients from the rows themselves: 29.72 vs 30.53 ms
    # per round with the per-step flipped images, same-box A/B)
    _DGRAD_BT = [True]
    # weight gradients / SGD updates on the native TN GEMM (gemm_tn.hip):
    # 128 x 128 tiles whose epilogue streams the updated rows and their bf16
    # mirror through LDS -- 32.4 ms per round vs 34.6 on hipBLASLt's baddbmm +
    # a cast pass (the MFMA-layout epilogue, 4-byte stores: 35.1)
    _TN = [True, 1]

    @classmethod
    def _bmm_rows(cls, sink, off, A, B, lane: bool = True):
        """fp32 A_g @ B_g (bf16 operands) into the sink's rows at ``off`` (they
        are in the product's order): the gradient itself, or -- the fused SGD
        step -- rows = beta rows + alpha A_g @ B_g in the GEMM's epilogue, then
        the bf16 mirror of the updated segment.  On the side lane
        (ops/lanes.py): the rows it updates were read by the layer's input
        gradient, enqueued before; the step joins the lane before it returns."""
        if not lane:
            cls._bmm_rows_impl(sink, off, A, B)
            return
        with _lanes.fork(A, B):
            cls._bmm_rows_impl(sink, off, A, B)

    @classmethod
    def _bmm_rows_impl(cls, sink, off, A, B):
        G, K, n = A.shape[0], A.shape[1], B.shape[2]
        # (the stem's 27 columns stay on hipBLASLt: its [64 x 27] products over
        # 5,120 pixels are 100 one-tile blocks of 80 K-steps on the TN GEMM --
        # 31.43 vs 31.15 ms per round, same-box A/B)
        if cls._TN[0] and (n % 8 == 0 or cls._STEM_TN[0]) and _ops().fa_bmm_rows(
                A, B, sink.dst, sink.ld, off, sink.beta, sink.alpha, sink.mirror,
                                             cls._TN[1], sink.src, sink.sld):
            return
        dst = sink.dst[:, off:off + K * n].view(G, K, n)
        if cls._BMM_INTO[0]:
            try:
                if sink.beta == 0.0 and sink.alpha == 1.0:
                    torch.bmm(A, B, out_dtype=torch.float32, out=dst)
                else:
                    torch.baddbmm(sink.src_rows(off, K, n), A, B, out_dtype=torch.float32, beta=sink.beta,
                                  alpha=sink.alpha, out=dst)
                cls._mirror(sink, off, K * n)
                return
            except (RuntimeError, TypeError):
                cls._BMM_INTO[0] = False
        part = torch.bmm(A, B, out_dtype=torch.float32)
        if sink.beta == 0.0 and sink.alpha == 1.0:
            _ops().wgrad_rsc_add(dst, part, 1, n, 1, False)
        else:
            if sink.src is not None:
                dst.copy_(sink.src_rows(off, K, n))
            dst.mul_(sink.beta).add_(part, alpha=sink.alpha)
        cls._mirror(sink, off, K * n)

    @staticmethod
    def _mirror(sink, off, n):
        if sink.mirror is not None:
            _ops().fa_cast_rows(sink.mirror, sink.dst, sink.ld, sink.dst.shape[0], off, n)

    def _conv3_wgrad(self, dy, x, G, sink, off, K, C):
        # (on the side lane, after the layer's input gradient: see _bmm_rows)
        with _lanes.fork(dy, x):
            self._conv3_wgrad_impl(dy, x, G, sink, off, K, C)

    def _conv3_wgrad_impl(self, dy, x, G, sink, off, K, C):
        # 32x32 maps on the grouped halo wgrad; 16x16 and smaller on the TN
        # GEMM over the implicit column image (27.59 vs 27.97 ms per round with
        # the halo kernel on 16x16 too, 27.88 with the TN GEMM on 32x32 too;
        # the wide wgrad kernel on 8x8 / 4x4 had measured 38.4 vs 36.5)
        if x.shape[3] >= 32 and _ops().conv3x3_wgrad_rows(dy, x, G, sink.dst, sink.ld, off, True, sink.beta,
                                                          sink.alpha, sink.mirror, sink.src, sink.sld):
            return
        A = _gview(dy, G).transpose(1, 2)
        if self._IMPLICIT[0]:
            # the TN GEMM reads the column image implicitly from x (no im2col)
            n, _, H, Wd = x.shape
            shape = torch.empty((1, 1, 1), device=x.device, dtype=torch.bfloat16).expand(G, n * H * Wd, 9 * C)
            if _ops().fa_bmm_rows(A, shape, sink.dst, sink.ld, off, sink.beta, sink.alpha, sink.mirror,
                                  self._TN[1], sink.src, sink.sld, x):
                return
        col = _ops().im2col_grouped(x, G, 3, 3, 1, 1, 9 * C, False)
        self._bmm_rows(sink, off, A, col.transpose(0, 1))

    # (8x8 / 4x4 weight updates reading the column image implicitly: 28.44 vs
    # 29.50 ms per round with im2col_grouped + the column-image TN GEMM, same-box A/B)
    _IMPLICIT = [True]
    # (the stride-2 convs + shortcuts forward and weight updates over the
    # implicit column image: 28.34 vs 28.60 ms per round with im2col, same-box A/B)
    _IMP_STRIDED = [True]

    # ------------------------------------------------------------- round
    def run(self, w0: torch.Tensor, x: torch.Tensor, y: torch.Tensor, G: int, n: int, bs: int,
            epochs: int, lr: float, decay: float, wd: float, clip: Optional[float],
            out: torch.Tensor, first_pass: bool):
        """Local SGD of G clients (client-major batch x [G*n, 3, H, W], labels
        y [G*n]); adds sum_g n (w0 - w_g) to ``out``.  Returns (per-client mean
        loss [G], per-client mean accuracy [G], per-layer sums of the clients'
        running statistics) over the local steps."""
        ops = _ops()
        dev = w0.device
        d = self.d
        ld = (d + 63) // 64 * 64
        perm = self._perm(dev)
        # the server weights in the rows' layout (+ bf16), read as a broadcast
        # row by the first local step
        w0i = torch.empty(ld, device=dev, dtype=torch.float32)
        w0b = torch.empty(ld, device=dev, dtype=torch.bfloat16)
        ops.fa_gather_rows(w0i, w0b, w0, perm)
        Wg = torch.empty((G, ld), device=dev, dtype=torch.float32)
        Wb = torch.empty((G, ld), device=dev, dtype=torch.bfloat16)
        # without clipping every weight-gradient producer applies the SGD step
        # to the client rows in place (no gradient rows, no separate update
        # pass); clipping needs each client's whole gradient norm first
        fused = not clip
        if fused:
            # (no broadcast of the server row into Wg: the first step's
            # producers read it as their source row)
            Gg = None
        else:
            Gg = torch.zeros((G, ld), device=dev, dtype=torch.float32)
        # per-client running statistics (the model keeps their mean): one
        # [4, G, C] buffer per block (mean 1, mean 2, var 1, var 2), each slice
        # a contiguous [G*C] copy per client -- one fill and one reduction per
        # block instead of four of each
        run, run_bufs = [], []
        for b in self.blocks:
            src = torch.stack([b.m1.running_mean, b.m2.running_mean, b.m1.running_var,
                               b.m2.running_var]).detach().float()
            buf = src.unsqueeze(1).expand(4, G, src.shape[1]).contiguous()
            run_bufs.append(buf)
            run.append(tuple(buf[i].view(-1) for i in range(4)))
        nbt = self.blocks[0].m1.num_batches_tracked if first_pass else None
        ls, cs = [], []  # per-step [G n] losses / correctness, reduced once at the end
        self._col_cache = None
        self._col_ok = bs >= n  # (full-batch steps: the same input every step)
        ones = torch.ones((G, max(n, bs), 1), device=dev)
        steps = 0
        xv = x.view(G, n, *x.shape[1:]) if bs < n else None
        for _ in range(epochs):
            for s0 in range(0, n, bs):
                s1 = min(n, s0 + bs)
                if bs < n:
                    xb = xv[:, s0:s1].reshape(G * (s1 - s0), *x.shape[1:]).contiguous(
                        memory_format=torch.channels_last)
                    yb = y.view(G, n)[:, s0:s1].reshape(-1).contiguous()
                else:
                    xb, yb = x, y
                if steps == 0:
                    W, Wbf, sld = w0i, w0b, 0
                else:
                    W, Wbf, sld = Wg, Wb, ld
                lr_t = float(lr * decay ** steps)
                # (the last step's updated weights are only uploaded from the
                # fp32 rows: no bf16 mirror writes)
                last = steps == epochs * ((n + bs - 1) // bs) - 1
                sink = (_Sink(Wg, ld, 1.0 - lr_t * wd, -lr_t, None if last else Wb, W, sld) if fused
                        else _Sink(Gg, ld, 0.0, 1.0, None))
                l, c = self._step(xb, yb, G, s1 - s0, W, Wbf, sld, sink, run, nbt, ones)
                ls.append(l.view(G, -1))
                cs.append(c.view(G, -1))
                if not fused:
                    _lanes.join()  # (the gradient rows)
                    ops.fa_row_sgd(Wg, ld, W, sld, Gg, ld, G, d, float(clip), lr_t, float(wd), Wb)
                steps += 1
        _lanes.join()
        ops.fa_upload(out, w0i, Wg, ld, G, float(n), perm)
        # running statistics: per-client copies summed for the caller's mean,
        # [4, C] fp64 per block (mean 1, mean 2, var 1, var 2)
        sums = [torch.sum(buf, dim=1, dtype=torch.float64) for buf in run_bufs]
        return _step_means(ls), _step_means(cs), sums

    def _step(self, x, y, G, n, W, Wb, ld, sink, run, nbt, ones):
        """One local step of every client (fp32 rows W, bf16 mirror Wb, both
        ld apart; ld 0 = the shared server row): forward, then backward into
        the sink (gradient rows, or the in-place SGD step)."""
        ops = _ops()
        # ---- stem: grouped column image of the client-major input (9 C0 = 27
        # columns zero-padded to 64: the forward is the native grouped GEMM
        # against a 64-column copy of the weight rows; the weight update reads
        # the first 27)
        C0, K0 = self.cin0, self.c0
        Kc0 = (9 * C0 + 63) // 64 * 64 if _NATIVE_GMM[0] else (9 * C0 + 7) // 8 * 8
        col0 = self._stem_col(x, G, Kc0)
        col0g = col0.transpose(0, 1)[:, :, :9 * C0]
        H, Wd = x.shape[2], x.shape[3]
        y0 = torch.empty((n, G * K0, H, Wd), device=x.device, dtype=torch.bfloat16,
                         memory_format=torch.channels_last)
        w0rows = self._rows(Wb, ld, G, self.prep, K0, 9 * C0)
        done = False
        if _NATIVE_GMM[0] and Kc0 % 64 == 0:
            pad = getattr(self, "_stem_img", None)
            if pad is None or pad.shape != (G, K0, Kc0) or pad.device != x.device:
                pad = self._stem_img = torch.zeros((G, K0, Kc0), device=x.device, dtype=torch.bfloat16)
            pad[:, :, :9 * C0].copy_(w0rows)  # (the padding columns stay zero)
            done = ops.fa_gemm(col0.transpose(0, 1), pad, _gview(y0, G), False, 0.0)
        if not done:
            torch.bmm(col0g, w0rows.transpose(1, 2), out=_gview(y0, G))
        a = ops.fa_ew(y0, None, 1)
        a0 = a
        saved = []
        _lanes.join()  # (the blocks read the rows the lane updated in the last step)
        for bi, b in enumerate(self.blocks):
            xin = a
            rm1, rm2, rv1, rv2 = run[bi]
            colx = None
            if b.stride == 1:
                h1 = self._conv3(xin, Wb, ld, G, b.conv1, b.cout, b.cin)
                sc = xin
            else:
                nn_, _, Hi, Wi = xin.shape
                Ho, Wo = (Hi - 1) // 2 + 1, (Wi - 1) // 2 + 1
                h1 = torch.empty((nn_, G * b.cout, Ho, Wo), device=x.device, dtype=torch.bfloat16,
                                 memory_format=torch.channels_last)
                sc = torch.empty_like(h1)
                w1 = self._rows(Wb, ld, G, b.conv1, b.cout, 9 * b.cin)
                wsc = self._rows(Wb, ld, G, b.sc, b.cout, b.cin)
                P1 = nn_ * Ho * Wo
                # the stride-2 conv and its 1x1 shortcut on the native GEMM over
                # the IMPLICIT column image of xin (no im2col)
                if not (self._IMP_STRIDED[0]
                        and ops.fa_gemm(_carrier(xin, G, P1, 9 * b.cin), w1, _gview(h1, G), False, 0.0, xin, 3, 2, 1)
                        and ops.fa_gemm(_carrier(xin, G, P1, b.cin), wsc, _gview(sc, G), False, 0.0, xin, 1, 2, 0)):
                    colx = ops.im2col_grouped(xin, G, 3, 3, 2, 1, 9 * b.cin, False)
                    cg = colx.transpose(0, 1)
                    _gmm(cg, w1, _gview(h1, G), False)
                    # the 1x1 stride-2 shortcut reads the centre tap of the column image
                    _gmm(cg[:, :, 4 * b.cin:5 * b.cin], wsc, _gview(sc, G), False)
            a1, st1, bits1 = ops.cs_bn_fwd(h1, W, ld, b.bn1w, b.bn1b, G, b.m1.eps, b.m1.momentum, rm1, rv1,
                                           nbt if bi == 0 else None)
            h2 = self._conv3(a1, Wb, ld, G, b.conv2, b.cout, b.cout)
            # relu(bn2) + shortcut in the BN's apply pass (the ReLU bits are the pre-add value's)
            a, st2, bits2 = ops.cs_bn_fwd(h2, W, ld, b.bn2w, b.bn2b, G, b.m2.eps, b.m2.momentum, rm2, rv2,
                                          None, sc)
            saved.append((xin, colx, h1, st1, bits1, a1, h2, st2, bits2))
        # ---- head: avg || max pool -> per-client linear -> cross entropy
        feat, codes = ops.fa_head_fwd(a, G)
        if self._fused_head_ok(n, self.feat):
            # classifier + loss + feature gradient + the rows' SGD step: logits
            # kernel, then the update kernel over (client, features, 32-class
            # chunks) whose partial feature gradients the pool backward sums
            S = -(-self.ncls // 32)
            dfeat = torch.empty((S * G, n, self.feat), device=feat.device, dtype=torch.float32)
            loss, correct = ops.fa_linear_ce(feat, n * self.feat, self.feat, G, n, W, ld, self.fc_w, self.fc_b,
                                             self.ncls, self.feat, 1.0, y, dfeat, n * self.feat, self.feat,
                                             sink.dst, sink.ld, sink.beta, sink.alpha, sink.src, sink.sld,
                                             None, 0,  # (the classifier reads the fp32 rows: no mirror)
                                             G * n * self.feat, 32)
        else:
            dfeat = torch.empty_like(feat)
            # classifier rows of every client (the first step: the server row, batch stride 0)
            Wfc = self._rows(W, ld, G, self.fc_w, self.ncls, self.feat)
            bfc = self._rows(W, ld, G, self.fc_b, 1, self.ncls)
            logits = torch.bmm(feat, Wfc.transpose(1, 2))
            logits.baddbmm_(ones[:, :n], bfc)
            loss, correct, gl = ops.ce_fwd(logits.view(G * n, self.ncls), y)
            gl = gl.view(G, n, self.ncls)
            inv = 1.0 / n
            # (the feature gradient first: the classifier rows may be updated in place next)
            torch.baddbmm(dfeat, gl, Wfc, beta=0.0, alpha=inv, out=dfeat)
            gW = sink.dst[:, self.fc_w:self.fc_w + self.ncls * self.feat].view(G, self.ncls, self.feat)
            torch.baddbmm(sink.src_rows(self.fc_w, self.ncls, self.feat), gl.transpose(1, 2), feat,
                          beta=sink.beta, alpha=sink.alpha * inv, out=gW)
            gb = sink.dst[:, self.fc_b:self.fc_b + self.ncls].view(G, 1, self.ncls)
            torch.baddbmm(sink.src_rows(self.fc_b, 1, self.ncls), ones[:, :n].transpose(1, 2), gl,
                          beta=sink.beta, alpha=sink.alpha * inv, out=gb)
        da = ops.fa_head_bwd(dfeat, codes, a.shape[2], a.shape[3])
        # ---- blocks, last to first
        for bi in range(len(self.blocks) - 1, -1, -1):
            b = self.blocks[bi]
            xin, colx, h1, st1, bits1, a1, h2, st2, bits2 = saved[bi]
            dh2 = ops.cs_bn_bwd(da, h2, st2, bits2, W, ld, b.bn2w, G, sink.dst, sink.ld, b.bn2w, b.bn2b,
                                sink.beta, sink.alpha, sink.src, sink.sld)
            # (each conv's input gradient reads its weights before the weight
            # gradient's producer may update them in place)
            da1 = self._conv3_dgrad(dh2, Wb, ld, G, b.conv2, b.cout, b.cout)
            self._conv3_wgrad(dh2, a1, G, sink, b.conv2, b.cout, b.cout)
            dh1 = ops.cs_bn_bwd(da1, h1, st1, bits1, W, ld, b.bn1w, G, sink.dst, sink.ld, b.bn1w, b.bn1b,
                                sink.beta, sink.alpha, sink.src, sink.sld)
            if b.stride == 1:
                # (+ the identity shortcut's gradient da, in the dgrad epilogue:
                # 31.94 vs 32.17 ms per round with a separate add)
                dx = self._conv3_dgrad(dh1, Wb, ld, G, b.conv1, b.cout, b.cin, da)
                self._conv3_wgrad(dh1, xin, G, sink, b.conv1, b.cout, b.cin)
                da = dx
            else:
                nn_, _, Hi, Wi = xin.shape
                P1 = nn_ * ((Hi - 1) // 2 + 1) * ((Wi - 1) // 2 + 1)
                dcol = torch.empty((P1, G, 9 * b.cin), device=x.device, dtype=torch.bfloat16)
                dcg = dcol.transpose(0, 1)
                _gmm(_gview(dh1, G), self._rows(Wb, ld, G, b.conv1, b.cout, 9 * b.cin), dcg, True)
                # the shortcut's input gradient joins the centre tap before the gather
                dctr = dcg[:, :, 4 * b.cin:5 * b.cin]
                _gmm(_gview(da, G), self._rows(Wb, ld, G, b.sc, b.cout, b.cin), dctr, True, 1.0)
                A1, Asc = _gview(dh1, G).transpose(1, 2), _gview(da, G).transpose(1, 2)
                if colx is None:
                    with _lanes.fork(A1, Asc, xin):
                        ok = (ops.fa_bmm_rows(A1, _carrier(xin, G, P1, 9 * b.cin), sink.dst, sink.ld, b.conv1,
                                              sink.beta, sink.alpha, sink.mirror, self._TN[1], sink.src, sink.sld,
                                              xin, 3, 2, 1)
                              and ops.fa_bmm_rows(Asc, _carrier(xin, G, P1, b.cin), sink.dst, sink.ld, b.sc,
                                                  sink.beta, sink.alpha, sink.mirror, self._TN[1], sink.src,
                                                  sink.sld, xin, 1, 2, 0))
                    if not ok:
                        raise RuntimeError("ResNet18FedAvg: implicit strided weight update refused after its forward")
                if colx is not None:
                    cg = colx.transpose(0, 1)
                    self._bmm_rows(sink, b.conv1, A1, cg)
                    self._bmm_rows(sink, b.sc, Asc, cg[:, :, 4 * b.cin:5 * b.cin])
                da = ops.col2im_grouped(dcol, G, nn_, Hi, Wi, b.cin, 3, 3, 2, 1)
        # ---- stem weight gradient (ReLU backward through its output)
        dy0 = ops.relu_mask(da, a0)
        # (the stem update on the main stream: it has nothing left to do while
        # the lane finishes the last blocks' updates)
        self._bmm_rows(sink, self.prep, _gview(dy0, G).transpose(1, 2), col0g, lane=False)
        # (no join here: the next step's stem runs beside the lane's last
        # updates; the step joins before its first block reads them)
        return loss, correct


class ResNet9FedAvg(ResNet18FedAvg):
    """Explicit G-client forward / backward / local SGD of models.resnet9.ResNet9
    (the headline model; BatchNorm off, as in the reference's FetchSGD / FedAvg
    CIFAR runs, cv_train.py:357): prep conv3x3 + ReLU, layer1 conv + ReLU +
    2x2 max-pool, res1 = x + relu(conv(relu(conv x))), layer2 / layer3 conv +
    ReLU + pool, res3, 4x4 max-pool, linear (no bias) x 0.125 -- reference
    /root/reference/CommEfficient/models/resnet9.py:32-148, local SGD
    fed_worker.py:61-113.  Same layout and kernels as ResNet18FedAvg: client
    rows (3x3 conv weights in the kernels' (k, r, s, c) order, bf16 mirror),
    channel-stacked activations, the grouped halo convs (forward, input
    gradient from the rows, weight gradient / fused SGD step), the grouped
    stem GEMM, the ReLU + max-pool kernels of csrc/pool.hip on the stacked
    channels, and a batched fp32 classifier on the weight rows."""

    # (conv offset key, input channels key, output channels key, pool after)
    _LAYERS = ("layer1", "res1.res1", "res1.res2", "layer2", "layer3", "res3.res1", "res3.res2")

    @staticmethod
    def supported(model, args) -> Tuple[bool, str]:
        from ..models.resnet9 import ResNet9
        if not isinstance(model, ResNet9):
            return False, "not the ResNet9 of models/resnet9.py"
        if getattr(args, "dtype", "bf16") != "bf16":
            return False, "bf16 compute only"
        if model.n.prep.do_batchnorm:
            return False, "ResNet9 with BatchNorm"
        n = model.n
        if not (isinstance(n.pool, torch.nn.MaxPool2d) and n.linear.bias is None
                and isinstance(n.layer1.pool, torch.nn.MaxPool2d)):
            return False, "ResNet9 head / pools of another form"
        ks = [n.layer1.pool.kernel_size, n.layer2.pool.kernel_size, n.layer3.pool.kernel_size, n.pool.kernel_size]
        if [k if isinstance(k, int) else k[0] for k in ks] != [2, 2, 2, 4]:
            return False, "ResNet9 pools must be 2, 2, 2 and 4"
        chans = [model.channels[c] for c in ("prep", "layer1", "layer2", "layer3")]
        if any(c % 64 for c in chans):
            return False, "channel counts must be multiples of 64"
        for p in model.parameters():
            if not p.requires_grad:
                return False, "frozen parameters"
        return True, ""

    def accepts(self, shape) -> Tuple[bool, str]:
        """NCHW client batches of the stem's channels whose 8x-pooled map is the
        4x4 the head pools whole (32 x 32 CIFAR images)."""
        if len(shape) != 4:
            return False, f"input of shape {tuple(shape)}: NCHW images expected"
        _, c, h, w = shape
        if c != self.cin0:
            return False, f"{c} input channels, the stem takes {self.cin0}"
        if h != 32 or w != 32:
            return False, f"{h}x{w} images: the 4x4 max-pool head needs 32 x 32"
        return True, ""

    def __init__(self, model, flat, names: List[str]):
        self.model = model
        off = self._aligned(names, flat)
        self.off = off
        n = model.n
        self.prep = off["n.prep.conv.weight"]
        self.c0 = n.prep.conv.out_channels
        self.cin0 = n.prep.conv.in_channels
        self.blocks = []  # (no BatchNorm)
        self.conv = {}
        for key in self._LAYERS:
            mod = n.get_submodule(key)
            self.conv[key] = (off[f"n.{key}.conv.weight"], mod.conv.in_channels, mod.conv.out_channels)
        self.fc_w = off["n.linear.weight"]
        self.ncls = n.linear.out_features
        self.feat = n.linear.in_features
        self.scale = float(n.classifier.weight)

    def _perm(self, device) -> torch.Tensor:
        return self._perm_convs(device, [(self.prep, self.c0, self.cin0)]
                                + [(o, K, C) for (o, C, K) in self.conv.values()])

    def run(self, w0, x, y, G, n, bs, epochs, lr, decay, wd, clip, out, first_pass):
        """As ResNet18FedAvg.run (no running statistics: returns an empty list)."""
        ops = _ops()
        dev = w0.device
        d = self.d
        ld = (d + 63) // 64 * 64
        perm = self._perm(dev)
        w0i = torch.empty(ld, device=dev, dtype=torch.float32)
        w0b = torch.empty(ld, device=dev, dtype=torch.bfloat16)
        ops.fa_gather_rows(w0i, w0b, w0, perm)
        Wg = torch.empty((G, ld), device=dev, dtype=torch.float32)
        Wb = torch.empty((G, ld), device=dev, dtype=torch.bfloat16)
        fused = not clip
        Gg = None if fused else torch.zeros((G, ld), device=dev, dtype=torch.float32)
        ls, cs = [], []
        self._col_cache = None
        self._col_ok = bs >= n
        steps = 0
        xv = x.view(G, n, *x.shape[1:]) if bs < n else None
        for _ in range(epochs):
            for s0 in range(0, n, bs):
                s1 = min(n, s0 + bs)
                if bs < n:
                    xb = xv[:, s0:s1].reshape(G * (s1 - s0), *x.shape[1:]).contiguous(
                        memory_format=torch.channels_last)
                    yb = y.view(G, n)[:, s0:s1].reshape(-1).contiguous()
                else:
                    xb, yb = x, y
                W, Wbf, sld = (w0i, w0b, 0) if steps == 0 else (Wg, Wb, ld)
                lr_t = float(lr * decay ** steps)
                # (the last step's updated weights are only uploaded from the
                # fp32 rows: no bf16 mirror writes)
                last = steps == epochs * ((n + bs - 1) // bs) - 1
                sink = (_Sink(Wg, ld, 1.0 - lr_t * wd, -lr_t, None if last else Wb, W, sld) if fused
                        else _Sink(Gg, ld, 0.0, 1.0, None))
                l, c = self._step9(xb, yb, G, s1 - s0, W, Wbf, sld, sink)
                ls.append(l.view(G, -1))
                cs.append(c.view(G, -1))
                if not fused:
                    _lanes.join()  # (the gradient rows)
                    ops.fa_row_sgd(Wg, ld, W, sld, Gg, ld, G, d, float(clip), lr_t, float(wd), Wb)
                steps += 1
        _lanes.join()
        ops.fa_upload(out, w0i, Wg, ld, G, float(n), perm)
        return _step_means(ls), _step_means(cs), []

    def _step9(self, x, y, G, n, W, Wb, ld, sink):
        ops = _ops()
        # ---- stem (as ResNet18FedAvg._step): grouped column image x weight rows
        C0, K0 = self.cin0, self.c0
        Kc0 = (9 * C0 + 63) // 64 * 64 if _NATIVE_GMM[0] else (9 * C0 + 7) // 8 * 8
        col0 = self._stem_col(x, G, Kc0)
        col0g = col0.transpose(0, 1)[:, :, :9 * C0]
        H, Wd = x.shape[2], x.shape[3]
        y0 = torch.empty((n, G * K0, H, Wd), device=x.device, dtype=torch.bfloat16,
                         memory_format=torch.channels_last)
        w0rows = self._rows(Wb, ld, G, self.prep, K0, 9 * C0)
        done = False
        if _NATIVE_GMM[0] and Kc0 % 64 == 0:
            pad = getattr(self, "_stem_img", None)
            if pad is None or pad.shape != (G, K0, Kc0) or pad.device != x.device:
                pad = self._stem_img = torch.zeros((G, K0, Kc0), device=x.device, dtype=torch.bfloat16)
            pad[:, :, :9 * C0].copy_(w0rows)
            done = ops.fa_gemm(col0.transpose(0, 1), pad, _gview(y0, G), False, 0.0)
        if not done:
            torch.bmm(col0g, w0rows.transpose(1, 2), out=_gview(y0, G))
        a0 = ops.fa_ew(y0, None, 1)
        cv = self.conv

        def conv(xin, key):
            off, C, K = cv[key]
            return self._conv3(xin, Wb, ld, G, off, K, C)

        # ---- forward (saving what the backward reads)
        _lanes.join()  # (the blocks read the rows the lane updated in the last step)
        p1, c1 = ops.relu_maxpool(conv(a0, "layer1"), 2)
        r1 = ops.fa_ew(conv(p1, "res1.res1"), None, 1)
        r2 = ops.fa_ew(conv(r1, "res1.res2"), None, 1)
        y1 = ops.fa_ew(p1, r2, 0)
        p2, c2 = ops.relu_maxpool(conv(y1, "layer2"), 2)
        p3, c3 = ops.relu_maxpool(conv(p2, "layer3"), 2)
        s1 = ops.fa_ew(conv(p3, "res3.res1"), None, 1)
        s2 = ops.fa_ew(conv(s1, "res3.res2"), None, 1)
        y3 = ops.fa_ew(p3, s2, 0)
        # ---- head: 4x4 max-pool (y3 >= 0: the ReLU is the identity) -> per-client
        # fp32 features -> logits = 0.125 feat Wl^T (batched on the weight rows)
        f16, c4 = ops.relu_maxpool(y3, 4)  # [n, G*512, 1, 1]: (example, client, feature)
        F_ = self.feat
        if self._fused_head_ok(n, F_):
            # classifier + loss + feature gradient + the rows' SGD step in one
            # kernel per client, the features read / their gradient written in
            # the channel-stacked bf16 layout (the classifier reads the fp32
            # rows: no mirror)
            df16 = torch.empty_like(f16)
            loss, correct = ops.fa_linear_ce(f16, F_, G * F_, G, n, W, ld, self.fc_w, -1, self.ncls, F_,
                                             self.scale, y, df16, F_, G * F_, sink.dst, sink.ld, sink.beta,
                                             sink.alpha, sink.src, sink.sld, None, 0)
            dy3 = ops.relu_maxpool_backward(df16, c4, 4)
        else:
            feat = f16.view(n, G, F_).transpose(0, 1).float()  # [G, n, F]
            Wl = self._rows(W, ld, G, self.fc_w, self.ncls, F_)
            logits = torch.bmm(feat, Wl.transpose(1, 2)).mul_(self.scale)
            loss, correct, gl = ops.ce_fwd(logits.reshape(G * n, self.ncls), y)
            gl = gl.view(G, n, self.ncls)
            a = self.scale / n
            dfeat = torch.bmm(gl, Wl).mul_(a)  # (read before the rows may be updated in place)
            gW = sink.dst[:, self.fc_w:self.fc_w + self.ncls * F_].view(G, self.ncls, F_)
            torch.baddbmm(sink.src_rows(self.fc_w, self.ncls, F_), gl.transpose(1, 2), feat, beta=sink.beta,
                          alpha=sink.alpha * a, out=gW)  # (the classifier reads the fp32 rows: no mirror)
            dy3 = ops.relu_maxpool_backward(
                dfeat.transpose(0, 1).reshape(n, G * F_, 1, 1).to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last), c4, 4)

        def back(dy, xin, key, addend=None):
            off, C, K = cv[key]
            dx = self._conv3_dgrad(dy, Wb, ld, G, off, K, C, addend)
            self._conv3_wgrad(dy, xin, G, sink, off, K, C)
            return dx

        # ---- res3: y3 = p3 + s2, s2 = relu(conv_b s1), s1 = relu(conv_a p3)
        ds1 = back(ops.relu_mask(dy3, s2), s1, "res3.res2")
        dp3 = back(ops.relu_mask(ds1, s1), p3, "res3.res1", dy3)
        # ---- layer3, layer2 (relu + pool backward, then the conv)
        dp2 = back(ops.relu_maxpool_backward(dp3, c3, 2), p2, "layer3")
        dy1 = back(ops.relu_maxpool_backward(dp2, c2, 2), y1, "layer2")
        # ---- res1
        dr1 = back(ops.relu_mask(dy1, r2), r1, "res1.res2")
        dp1 = back(ops.relu_mask(dr1, r1), p1, "res1.res1", dy1)
        da0 = back(ops.relu_maxpool_backward(dp1, c1, 2), a0, "layer1")
        # ---- stem weight gradient
        dy0 = ops.relu_mask(da0, a0)
        # (the stem update on the main stream: it has nothing left to do while
        # the lane finishes the last blocks' updates)
        self._bmm_rows(sink, self.prep, _gview(dy0, G).transpose(1, 2), col0g, lane=False)
        # (no join here: the next step's stem runs beside the lane's last
        # updates; the step joins before its first block reads them)
        return loss, correct


class FixupResNet9FedAvg(ResNet9FedAvg):
    """Explicit G-client forward / backward / local SGD of models.fixup.FixupResNet9
    (reference /root/reference/CommEfficient/models/fixup_resnet9.py:33-91):
    ResNet9FedAvg's convolutions, pools and classifier, plus the per-client
    Fixup scalars (``x + b`` before each conv, ``conv * s + b`` after) on the
    native affine kernels (fedavg.hip fa_affine / fa_affine_bwd): the
    scalars are read from the clients' fp32 rows, their gradients are
    fixed-order per-client sums written by ``fa_scalar_sgd`` with the step's
    SGD update.  The stem's input bias gradient is the sum of the stem's
    column-image gradient over the in-image taps (the im2col of ones)."""

    @staticmethod
    def supported(model, args) -> Tuple[bool, str]:
        from ..models.fixup import FixupResNet9
        if not isinstance(model, FixupResNet9):
            return False, "not the FixupResNet9 of models/fixup.py"
        if getattr(args, "dtype", "bf16") != "bf16":
            return False, "bf16 compute only"
        pools = [model.layer1.pool, model.layer2.pool, model.layer3.pool, model.pool]
        if not all(isinstance(q, torch.nn.MaxPool2d) for q in pools):
            return False, "FixupResNet9 pools of another form"
        ks = [q.kernel_size if isinstance(q.kernel_size, int) else q.kernel_size[0] for q in pools]
        if ks != [2, 2, 2, 4] or len(model.layer2.blocks) != 0 or len(model.layer1.blocks) != 1 \
                or len(model.layer3.blocks) != 1 or model.linear.bias is None:
            return False, "FixupResNet9 of another topology"
        if any(c % 64 for c in (model.channels[k] for k in ("prep", "layer1", "layer2", "layer3"))):
            return False, "channel counts must be multiples of 64"
        for p in model.parameters():
            if not p.requires_grad:
                return False, "frozen parameters"
        return True, ""

    def __init__(self, model, flat, names: List[str]):
        self.model = model
        off = self._aligned(names, flat)
        self.off = off
        self.prep = off["conv1.weight"]
        self.c0 = model.conv1.out_channels
        self.cin0 = model.conv1.in_channels
        self.blocks = []  # (no BatchNorm)
        self.conv = {}
        for key, mod in (("layer1", model.layer1.conv), ("layer1.b1", model.layer1.blocks[0].conv1),
                         ("layer1.b2", model.layer1.blocks[0].conv2), ("layer2", model.layer2.conv),
                         ("layer3", model.layer3.conv), ("layer3.b1", model.layer3.blocks[0].conv1),
                         ("layer3.b2", model.layer3.blocks[0].conv2)):
            wname = {"layer1": "layer1.conv.weight", "layer1.b1": "layer1.blocks.0.conv1.weight",
                     "layer1.b2": "layer1.blocks.0.conv2.weight", "layer2": "layer2.conv.weight",
                     "layer3": "layer3.conv.weight", "layer3.b1": "layer3.blocks.0.conv1.weight",
                     "layer3.b2": "layer3.blocks.0.conv2.weight"}[key]
            self.conv[key] = (off[wname], mod.in_channels, mod.out_channels)
        self.fc_w = off["linear.weight"]
        self.fc_b = off["linear.bias"]
        self.ncls = model.linear.out_features
        self.feat = model.linear.in_features
        self.scale = 1.0
        self.sc = {k: v for k, v in off.items() if k.endswith(("bias1a", "bias1b", "bias2a", "bias2b", "scale"))
                   or k == "bias2"}

    def _ones_col(self, x, G, Kc0):
        """im2col of an all-ones image of x's geometry: 1 at the in-image taps."""
        key = (tuple(x.shape), G, Kc0, x.device)
        if getattr(self, "_ones_key", None) != key:
            ones = torch.ones_like(x)
            c = _ops().im2col_grouped(ones, G, 3, 3, 1, 1, Kc0, True)
            n, H, Wd = x.shape[0] // G, x.shape[2], x.shape[3]
            self._ones = c.view(n, H, Wd, G * Kc0).permute(0, 3, 1, 2)  # channel-stacked view
            self._ones_key = key
        return self._ones

    def _step9(self, x, y, G, n, W, Wb, ld, sink):
        ops = _ops()
        S = self.sc

        def aff(t, s=None, b=None, add=None, relu=False, cm=False):
            return ops.fa_affine(t, G, cm, W, ld, -1 if s is None else S[s], -1 if b is None else S[b], add, relu)

        def sgd(part, b=None, s=None):
            # (b: the bias gets sum dpre; s: the scale -- or, without a scale
            # input, the unmasked sum -- gets the second sum)
            ops.fa_scalar_sgd(part, sink.dst, sink.ld, -1 if b is None else S[b], -1 if s is None else S[s],
                              sink.beta, sink.alpha, sink.src, sink.sld)

        def conv(xin, key):
            off, C, K = self.conv[key]
            return self._conv3(xin, Wb, ld, G, off, K, C)

        def back(dy, xin, key):
            off, C, K = self.conv[key]
            dx = self._conv3_dgrad(dy, Wb, ld, G, off, K, C)
            self._conv3_wgrad(dy, xin, G, sink, off, K, C)
            return dx

        # ---- stem: relu(conv1(x + b1a) * s + b1b) on the column image of x + b1a
        C0, K0 = self.cin0, self.c0
        Kc0 = (9 * C0 + 63) // 64 * 64
        N_, _, H, Wd = x.shape
        ps = x.stride(3)
        if x.stride(1) == 1 and ps >= C0 and x.stride(2) == ps * Wd and x.stride(0) == ps * H * Wd:
            # (the augmentation kernel's images: channels innermost in a wider
            # pixel -- the affine pass runs over the whole pixels, im2col reads C0)
            xr = torch.as_strided(x, (N_, ps, H, Wd), (x.stride(0), 1, x.stride(2), ps))
            xa = aff(xr, b="bias1a", cm=True)[:, :C0]
        else:
            xa = aff(x.contiguous(memory_format=torch.channels_last), b="bias1a", cm=True)
        col0 = ops.im2col_grouped(xa, G, 3, 3, 1, 1, Kc0, True)
        col0g = col0.transpose(0, 1)[:, :, :9 * C0]
        y0 = torch.empty((n, G * K0, H, Wd), device=x.device, dtype=torch.bfloat16,
                         memory_format=torch.channels_last)
        w0rows = self._rows(Wb, ld, G, self.prep, K0, 9 * C0)
        pad = getattr(self, "_stem_img", None)
        if pad is None or pad.shape != (G, K0, Kc0) or pad.device != x.device:
            pad = self._stem_img = torch.zeros((G, K0, Kc0), device=x.device, dtype=torch.bfloat16)
        pad[:, :, :9 * C0].copy_(w0rows)
        if not ops.fa_gemm(col0.transpose(0, 1), pad, _gview(y0, G), False, 0.0):
            torch.bmm(col0g, w0rows.transpose(1, 2), out=_gview(y0, G))
        a0 = aff(y0, s="scale", b="bias1b", relu=True)

        def layer(xin, name, key):  # pool(relu(conv(x + b1a) * s + b1b))
            xa_ = aff(xin, b=f"{name}.bias1a")
            h = conv(xa_, key)
            p, codes = ops.relu_maxpool(aff(h, s=f"{name}.scale", b=f"{name}.bias1b"), 2)
            return (xa_, h, codes), p

        def block(xin, name, k1, k2):  # relu(conv2(relu(conv1(x + b1a) + b1b) + b2a) * s + b2b + x)
            xa_ = aff(xin, b=f"{name}.bias1a")
            h1 = aff(conv(xa_, k1), b=f"{name}.bias1b", relu=True)
            h1a = aff(h1, b=f"{name}.bias2a")
            h2 = conv(h1a, k2)
            out = aff(h2, s=f"{name}.scale", b=f"{name}.bias2b", add=xin, relu=True)
            return (xa_, h1, h1a, h2, out), out

        _lanes.join()  # (the blocks read the rows the lane updated in the last step)
        sv1, p1 = layer(a0, "layer1", "layer1")
        sb1, y1 = block(p1, "layer1.blocks.0", "layer1.b1", "layer1.b2")
        sv2, p2 = layer(y1, "layer2", "layer2")
        sv3, p3 = layer(p2, "layer3", "layer3")
        sb3, y3 = block(p3, "layer3.blocks.0", "layer3.b1", "layer3.b2")
        # ---- head: 4x4 max-pool (y3 >= 0), + bias2, linear (+ bias) -> CE, one kernel pair
        f16, c4 = ops.relu_maxpool(y3, 4)
        F_ = self.feat
        feat = aff(f16, b="bias2")
        df16 = torch.empty_like(feat)
        loss, correct = ops.fa_linear_ce(feat, F_, G * F_, G, n, W, ld, self.fc_w, self.fc_b, self.ncls, F_,
                                         1.0, y, df16, F_, G * F_, sink.dst, sink.ld, sink.beta, sink.alpha,
                                         sink.src, sink.sld, None, 0)
        sgd(ops.fa_affine_bwd(df16, G, False, W, ld, -1, None, None, None, False, False)[2], b="bias2")
        dy3 = ops.relu_maxpool_backward(df16, c4, 4)

        def block_back(dy, saved, name, k1, k2):
            xa_, h1, h1a, h2, out = saved
            # relu(h2 s + b2b + x): dh2 = dpre s, the identity's gradient dpre
            dh2, dpre, part = ops.fa_affine_bwd(dy, G, False, W, ld, S[f"{name}.scale"], out, h2, None, True, True)
            sgd(part, b=f"{name}.bias2b", s=f"{name}.scale")
            dh1a = back(dh2, h1a, k2)
            # h1a = h1 + b2a (sum of dh1a), h1 = relu(c1 + b1b) (sum of the masked)
            dc1, _, part = ops.fa_affine_bwd(dh1a, G, False, W, ld, -1, h1, None, None, True, False)
            sgd(part, b=f"{name}.bias1b", s=f"{name}.bias2a")
            dxa = back(dc1, xa_, k1)
            # xa = x + b1a: sum of dxa; dx = dxa + the identity's gradient
            dx, _, part = ops.fa_affine_bwd(dxa, G, False, W, ld, -1, None, None, dpre, True, False)
            sgd(part, b=f"{name}.bias1a")
            return dx

        def layer_back(dp, xin, saved, name, key):
            xa_, h, codes = saved
            dhp = ops.relu_maxpool_backward(dp, codes, 2)  # (gradient of h s + b1b)
            dh, _, part = ops.fa_affine_bwd(dhp, G, False, W, ld, S[f"{name}.scale"], None, h, None, True, False)
            sgd(part, b=f"{name}.bias1b", s=f"{name}.scale")
            dxa = back(dh, xa_, key)
            sgd(ops.fa_affine_bwd(dxa, G, False, W, ld, -1, None, None, None, False, False)[2], b=f"{name}.bias1a")
            return dxa  # (xa = x + b1a: the input's gradient is dxa itself)

        dp3 = block_back(dy3, sb3, "layer3.blocks.0", "layer3.b1", "layer3.b2")
        dp2 = layer_back(dp3, p2, sv3, "layer3", "layer3")
        dy1 = layer_back(dp2, y1, sv2, "layer2", "layer2")
        dp1 = block_back(dy1, sb1, "layer1.blocks.0", "layer1.b1", "layer1.b2")
        da0 = layer_back(dp1, a0, sv1, "layer1", "layer1")
        # ---- stem: relu(y0 s + b1b)
        dy0, _, part = ops.fa_affine_bwd(da0, G, False, W, ld, S["scale"], a0, y0, None, True, False)
        sgd(part, b="bias1b", s="scale")
        # the input bias: sum of the stem's column-image gradient over the in-image taps
        dcol = torch.empty((n, G * Kc0, H, Wd), device=x.device, dtype=torch.bfloat16,
                           memory_format=torch.channels_last)
        if not ops.fa_gemm(_gview(dy0, G), pad, _gview(dcol, G), True, 0.0):
            torch.bmm(_gview(dy0, G), pad, out=_gview(dcol, G))
        part = ops.fa_affine_bwd(dcol, G, False, W, ld, -1, None, self._ones_col(x, G, Kc0), None, False, False)[2]
        sgd(part, s="bias1a")
        # (the stem update on the main stream: it has nothing left to do while
        # the lane finishes the last blocks' updates)
        self._bmm_rows(sink, self.prep, _gview(dy0, G).transpose(1, 2), col0g, lane=False)
        # (no join here: the next step's stem runs beside the lane's last
        # updates; the step joins before its first block reads them)
        return loss, correct


class FixupResNet18FedAvg(ResNet18FedAvg):
    """Explicit G-client forward / backward / local SGD of models.fixup.FixupResNet18
    (reference /root/reference/CommEfficient/models/fixup_resnet18.py:24-135):
    ResNet18FedAvg's stem, convolutions (stride-2 ones and their 1x1 shortcuts
    on implicit column images), avg || max head and fused classifier, with the
    blocks' BatchNorms replaced by the per-client Fixup scalars
    ``relu(conv2(relu(conv1(x + a1a) + a1b) + a2a) * m + a2b + shortcut(x))``
    on the affine kernels (see FixupResNet9FedAvg).  A strided block's input
    bias gradient is the sum of conv1's column-image gradient over the
    in-image taps, taken before the shortcut's gradient joins the centre tap."""

    run = ResNet9FedAvg.run  # (no running statistics)

    @staticmethod
    def supported(model, args) -> Tuple[bool, str]:
        from ..models.fixup import FixupResNet18
        if not isinstance(model, FixupResNet18):
            return False, "not the FixupResNet18 of models/fixup.py"
        if getattr(args, "dtype", "bf16") != "bf16":
            return False, "bf16 compute only"
        for layer in model.layers:
            for blk in layer:
                if blk.conv1.in_channels % 64 or blk.conv1.out_channels % 64:
                    return False, "channel counts must be multiples of 64"
        if model.prep.out_channels % 64:
            return False, "channel counts must be multiples of 64"
        for p in model.parameters():
            if not p.requires_grad:
                return False, "frozen parameters"
        return True, ""

    def __init__(self, model, flat, names: List[str]):
        self.model = model
        off = self._aligned(names, flat)
        self.off = off
        self.prep = off["prep.weight"]
        self.blocks: List[_Block] = []
        self.fx = []  # per block: scalar offsets
        for li, layer in enumerate(model.layers):
            for bi, blk in enumerate(layer):
                p = f"layers.{li}.{bi}."
                b = _Block()
                b.cin, b.cout = blk.conv1.in_channels, blk.conv1.out_channels
                b.stride = blk.conv1.stride[0]
                b.conv1, b.conv2 = off[p + "conv1.weight"], off[p + "conv2.weight"]
                b.sc = off.get(p + "shortcut.weight")
                if b.sc is None and (b.stride != 1 or b.cin != b.cout):
                    raise ValueError("FixupResNet18FedAvg: block without a shortcut changes shape")
                if b.sc is not None and b.stride != 2:
                    raise ValueError("FixupResNet18FedAvg: stride-1 projection shortcuts are not wired")
                self.blocks.append(b)
                self.fx.append({k: off[p + k + (".scale" if k == "mul" else ".bias")]
                                for k in ("add1a", "add1b", "add2a", "mul", "add2b")})
        self.fc_w, self.fc_b = off["classifier.weight"], off["classifier.bias"]
        self.ncls = model.classifier.out_features
        self.feat = model.classifier.in_features
        self.c0 = model.prep.out_channels
        self.cin0 = model.prep.in_channels

    def _ones_strided(self, xin, G, C):
        """channel-stacked im2col (3 x 3, stride 2, pad 1) of an all-ones xin: 1 at the in-image taps"""
        key = (tuple(xin.shape), G, C, xin.device)
        cache = getattr(self, "_ones_s", None)
        if cache is None:
            cache = self._ones_s = {}
        if key not in cache:
            c = _ops().im2col_grouped(torch.ones_like(xin), G, 3, 3, 2, 1, 9 * C, False)
            n_, _, Hi, Wi = xin.shape
            Ho, Wo = (Hi - 1) // 2 + 1, (Wi - 1) // 2 + 1
            cache[key] = c.view(n_, Ho, Wo, G * 9 * C).permute(0, 3, 1, 2)
        return cache[key]

    def _step9(self, x, y, G, n, W, Wb, ld, sink):
        ops = _ops()

        def aff(t, fx, s=None, b=None, add=None, relu=False):
            return ops.fa_affine(t, G, False, W, ld, -1 if s is None else fx[s], -1 if b is None else fx[b],
                                 add, relu)

        def sgd(part, fx, b=None, s=None):
            ops.fa_scalar_sgd(part, sink.dst, sink.ld, -1 if b is None else fx[b], -1 if s is None else fx[s],
                              sink.beta, sink.alpha, sink.src, sink.sld)

        # ---- stem (as ResNet18FedAvg._step): relu(conv(x))
        C0, K0 = self.cin0, self.c0
        Kc0 = (9 * C0 + 63) // 64 * 64
        col0 = self._stem_col(x, G, Kc0)
        col0g = col0.transpose(0, 1)[:, :, :9 * C0]
        H, Wd = x.shape[2], x.shape[3]
        y0 = torch.empty((n, G * K0, H, Wd), device=x.device, dtype=torch.bfloat16,
                         memory_format=torch.channels_last)
        w0rows = self._rows(Wb, ld, G, self.prep, K0, 9 * C0)
        pad = getattr(self, "_stem_img", None)
        if pad is None or pad.shape != (G, K0, Kc0) or pad.device != x.device:
            pad = self._stem_img = torch.zeros((G, K0, Kc0), device=x.device, dtype=torch.bfloat16)
        pad[:, :, :9 * C0].copy_(w0rows)
        if not ops.fa_gemm(col0.transpose(0, 1), pad, _gview(y0, G), False, 0.0):
            torch.bmm(col0g, w0rows.transpose(1, 2), out=_gview(y0, G))
        a = ops.fa_ew(y0, None, 1)
        a0 = a
        saved = []
        _lanes.join()  # (the blocks read the rows the lane updated in the last step)
        for b, fx in zip(self.blocks, self.fx):
            xin = a
            xa = aff(xin, fx, b="add1a")
            if b.stride == 1:
                c1 = self._conv3(xa, Wb, ld, G, b.conv1, b.cout, b.cin)
                sc = xin
            else:
                nn_, _, Hi, Wi = xin.shape
                Ho, Wo = (Hi - 1) // 2 + 1, (Wi - 1) // 2 + 1
                c1 = torch.empty((nn_, G * b.cout, Ho, Wo), device=x.device, dtype=torch.bfloat16,
                                 memory_format=torch.channels_last)
                sc = torch.empty_like(c1)
                P1 = nn_ * Ho * Wo
                # conv1 over the implicit column image of x + a1a, the shortcut of x
                if not (ops.fa_gemm(_carrier(xa, G, P1, 9 * b.cin), self._rows(Wb, ld, G, b.conv1, b.cout, 9 * b.cin),
                                    _gview(c1, G), False, 0.0, xa, 3, 2, 1)
                        and ops.fa_gemm(_carrier(xin, G, P1, b.cin), self._rows(Wb, ld, G, b.sc, b.cout, b.cin),
                                        _gview(sc, G), False, 0.0, xin, 1, 2, 0)):
                    raise RuntimeError("FixupResNet18FedAvg: implicit strided GEMM refused")
            h1 = aff(c1, fx, b="add1b", relu=True)
            h1a = aff(h1, fx, b="add2a")
            h2 = self._conv3(h1a, Wb, ld, G, b.conv2, b.cout, b.cout)
            a = aff(h2, fx, s="mul", b="add2b", add=sc, relu=True)
            saved.append((xin, xa, h1, h1a, h2, a))
        # ---- head: avg || max pool -> classifier (fused) -> cross entropy
        feat, codes = ops.fa_head_fwd(a, G)
        S_ = -(-self.ncls // 32)
        dfeat = torch.empty((S_ * G, n, self.feat), device=feat.device, dtype=torch.float32)
        loss, correct = ops.fa_linear_ce(feat, n * self.feat, self.feat, G, n, W, ld, self.fc_w, self.fc_b,
                                         self.ncls, self.feat, 1.0, y, dfeat, n * self.feat, self.feat,
                                         sink.dst, sink.ld, sink.beta, sink.alpha, sink.src, sink.sld,
                                         None, 0, G * n * self.feat, 32)
        da = ops.fa_head_bwd(dfeat, codes, a.shape[2], a.shape[3])
        # ---- blocks, last to first
        for bi in range(len(self.blocks) - 1, -1, -1):
            b, fx = self.blocks[bi], self.fx[bi]
            xin, xa, h1, h1a, h2, out = saved[bi]
            # relu(h2 m + a2b + sc): dh2 = dpre m, the shortcut's gradient dpre
            dh2, dpre, part = ops.fa_affine_bwd(da, G, False, W, ld, fx["mul"], out, h2, None, True, True)
            sgd(part, fx, b="add2b", s="mul")
            dh1a = self._conv3_dgrad(dh2, Wb, ld, G, b.conv2, b.cout, b.cout)
            self._conv3_wgrad(dh2, h1a, G, sink, b.conv2, b.cout, b.cout)
            # h1a = h1 + a2a (sum of dh1a), h1 = relu(c1 + a1b) (sum of the masked)
            dc1, _, part = ops.fa_affine_bwd(dh1a, G, False, W, ld, -1, h1, None, None, True, False)
            sgd(part, fx, b="add1b", s="add2a")
            if b.stride == 1:
                dxa = self._conv3_dgrad(dc1, Wb, ld, G, b.conv1, b.cout, b.cin)
                self._conv3_wgrad(dc1, xa, G, sink, b.conv1, b.cout, b.cin)
                # xa = x + a1a: sum of dxa; dx = dxa + the identity's gradient
                da, _, part = ops.fa_affine_bwd(dxa, G, False, W, ld, -1, None, None, dpre, True, False)
                sgd(part, fx, b="add1a")
            else:
                nn_, _, Hi, Wi = xin.shape
                Ho, Wo = (Hi - 1) // 2 + 1, (Wi - 1) // 2 + 1
                P1 = nn_ * Ho * Wo
                dcol = torch.empty((P1, G, 9 * b.cin), device=x.device, dtype=torch.bfloat16)
                dcg = dcol.transpose(0, 1)
                _gmm(_gview(dc1, G), self._rows(Wb, ld, G, b.conv1, b.cout, 9 * b.cin), dcg, True)
                # the input bias: conv1's column-image gradient over the in-image taps
                dcol4 = dcol.view(nn_, Ho, Wo, G * 9 * b.cin).permute(0, 3, 1, 2)
                sgd(ops.fa_affine_bwd(dcol4, G, False, W, ld, -1, None, self._ones_strided(xin, G, b.cin), None,
                                      False, False)[2], fx, s="add1a")
                # then the shortcut's input gradient joins the centre tap before the gather
                _gmm(_gview(dpre, G), self._rows(Wb, ld, G, b.sc, b.cout, b.cin), dcg[:, :, 4 * b.cin:5 * b.cin],
                     True, 1.0)
                A1, Asc = _gview(dc1, G).transpose(1, 2), _gview(dpre, G).transpose(1, 2)
                with _lanes.fork(A1, Asc, xa, xin):
                    ok = (ops.fa_bmm_rows(A1, _carrier(xa, G, P1, 9 * b.cin), sink.dst, sink.ld, b.conv1,
                                          sink.beta, sink.alpha, sink.mirror, self._TN[1], sink.src, sink.sld,
                                          xa, 3, 2, 1)
                          and ops.fa_bmm_rows(Asc, _carrier(xin, G, P1, b.cin), sink.dst, sink.ld, b.sc,
                                              sink.beta, sink.alpha, sink.mirror, self._TN[1], sink.src,
                                              sink.sld, xin, 1, 2, 0))
                if not ok:
                    raise RuntimeError("FixupResNet18FedAvg: implicit strided weight update refused")
                da = ops.col2im_grouped(dcol, G, nn_, Hi, Wi, b.cin, 3, 3, 2, 1)
        # ---- stem weight gradient (ReLU backward through its output)
        dy0 = ops.relu_mask(da, a0)
        # (the stem update on the main stream: it has nothing left to do while
        # the lane finishes the last blocks' updates)
        self._bmm_rows(sink, self.prep, _gview(dy0, G).transpose(1, 2), col0g, lane=False)
        # (no join here: the next step's stem runs beside the lane's last
        # updates; the step joins before its first block reads them)
        return loss, correct


def engine_for(model, args):
    """(engine class or None, why): the explicit G-client FedAvg program that
    covers this model / configuration."""
    why = []
    for cls in (ResNet18FedAvg, ResNet9FedAvg, FixupResNet9FedAvg, FixupResNet18FedAvg):
        ok, w = cls.supported(model, args)
        if ok:
            return cls, ""
        why.append(f"{cls.__name__}: {w}")
    return None, "; ".join(why)
