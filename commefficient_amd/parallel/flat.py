"""Flat parameter / gradient buffers.

The reference flattens every round: ``get_grad_vec`` is a ``torch.cat`` of all
``p.grad`` and ``set_param_vec`` a per-parameter ``zero_()`` + ``add_()``
(/root/reference/CommEfficient/utils.py:254-297).
Here trainable parameters and their gradients are *views* into two
contiguous fp32 buffers, so "flatten" and "load weights" are free and every
codec kernel streams one aligned vector.  The flat order is
``model.parameters()`` order restricted to ``requires_grad`` params, exactly
the reference's grad-vector order.
"""
from __future__ import annotations

from typing import List, Tuple

import torch
import torch.nn as nn

from .. import ops


def trainable_params(model: nn.Module) -> List[nn.Parameter]:
    return [p for p in model.parameters() if p.requires_grad]


def grad_size(model: nn.Module) -> int:
    return sum(p.numel() for p in trainable_params(model))


class FlatParams:
    """Re-homes a model's trainable params (and grads) into flat buffers."""

    def __init__(self, model: nn.Module, device):
        self.model = model
        self.params = trainable_params(model)
        self.shapes = [p.shape for p in self.params]
        self.numels = [p.numel() for p in self.params]
        # the codec kernels stream the whole (16-byte aligned) flat buffer,
        # so per-parameter alignment inside it does not matter
        self.offsets: List[int] = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += n
        self.d = off
        self.device = torch.device(device)
        self.w = torch.empty(self.d, dtype=torch.float32, device=self.device)
        self.g = torch.zeros(self.d, dtype=torch.float32, device=self.device)
        self.g_zeroed = False  # g already all-zero (cleared by the sketch encode)
        with torch.no_grad():
            for p, o, n in zip(self.params, self.offsets, self.numels):
                self.w[o:o + n].copy_(p.detach().reshape(-1).to(self.device, torch.float32))
        self.bind(self.w)
        self._bind_grads()
        # non-trainable tensors (BN buffers, frozen params) follow the device
        for m in model.modules():
            for name, b in list(m.named_buffers(recurse=False)):
                if b is not None:
                    setattr(m, name, b.to(self.device))
            for name, p in list(m.named_parameters(recurse=False)):
                if not p.requires_grad:
                    p.data = p.data.to(self.device)

    def bind(self, buf: torch.Tensor) -> None:
        """Make the model's params views of ``buf`` (a [d] fp32 tensor)."""
        assert buf.numel() == self.d and buf.dtype == torch.float32
        self.bound = buf
        for p, o, n, s in zip(self.params, self.offsets, self.numels, self.shapes):
            p.data = buf[o:o + n].view(s)

    def _bind_grads(self):
        for p, o, n, s in zip(self.params, self.offsets, self.numels, self.shapes):
            p.grad = self.g[o:o + n].view(s)

    def zero_grad(self):
        if self.g_zeroed:
            self.g_zeroed = False  # the sketch encode already cleared g (fed_model._encode_merged)
        elif self.g.is_cuda:
            ops.zero_(self.g)  # (a memset a recorded round can replay, parallel/tape.py)
        else:
            self.g.zero_()
        # autograd may have replaced .grad (e.g. set_to_none elsewhere); the
        # expected address is computed, not sliced (a view per parameter per
        # round was ~0.4 ms of host time on GPT-2)
        base, es = self.g.data_ptr(), self.g.element_size()
        for p, o, n in zip(self.params, self.offsets, self.numels):
            gr = p.grad
            if gr is None or gr.data_ptr() != base + o * es:
                p.grad = self.g[o:o + n].view(p.shape)

    # ----------------------------------------------------- bf16 compute copy
    def make_bf16_shadow(self) -> nn.Module:
        """A bf16 replica of the model for the forward/backward (``--weight_cast
        once``): its trainable params are views of ONE flat bf16 buffer ``wb``,
        refreshed from the fp32 master weights by a single cast kernel
        (``refresh_shadow``), and its gradients are gathered into the fp32 flat
        gradient by one concatenation + one add (``collect_shadow_grads``).
        Autocast instead casts every weight tensor on each forward and every
        weight gradient back to fp32 with its own cast + AccumulateGrad add
        (~3 launches per parameter: ~450 for GPT-2)."""
        import copy
        shadow = copy.deepcopy(self.model).to(torch.bfloat16)
        sp = trainable_params(shadow)
        assert [p.shape for p in sp] == list(self.shapes)
        self.wb = torch.empty(self.d, dtype=torch.bfloat16, device=self.device)
        self.gb = torch.empty(self.d, dtype=torch.bfloat16, device=self.device)
        for p, o, n, s in zip(sp, self.offsets, self.numels, self.shapes):
            p.data = self.wb[o:o + n].view(s)
            p.grad = None
        self.shadow_params = sp
        # the replica follows sparse server steps by a k-element patch instead
        # of a full cast (ops/nn.py weight-mirror protocol)
        self._wb_valid = None   # fp32 buffer the replica mirrors AFTER a patch (reusable)
        self._wb_synced = None  # fp32 buffer of the last full cast
        self._wb_sig = None     # write signature of the weights the replica matches
        if self.device.type == "cuda":
            from ..ops.nn import register_weight_mirror
            register_weight_mirror(self)
        return shadow

    def _write_sig(self) -> int:
        """Monotone signature of writes to the bound fp32 weights: in-place
        writes to the flat buffer bump its version counter, writes through the
        parameter views (``load_state_dict``, ``set_param_vec``) bump the
        parameters' own counters (views made by ``.data =`` do not share it)."""
        return self.bound._version + sum(p._version for p in self.params)

    def refresh_shadow(self) -> None:
        from ..ops.nn import mirrors_enabled
        ptr = self.bound.data_ptr()
        sig = self._write_sig()
        if self._wb_valid == ptr and self._wb_sig == sig and mirrors_enabled():
            return  # patched by the last (sparse) server step: already current
        self.wb.copy_(self.bound)
        self._wb_valid = None
        self._wb_synced = ptr
        self._wb_sig = sig

    # weight-mirror protocol (ops/nn.py weights_begin_update / weights_end_update)
    def begin(self, w_flat: torch.Tensor) -> bool:
        ptr = w_flat.data_ptr() if w_flat.numel() == self.d else None
        ok = (ptr is not None and ptr in (self._wb_valid, self._wb_synced)
              and ptr == self.bound.data_ptr() and self._wb_sig == self._write_sig())
        self._wb_valid = self._wb_synced = None
        return ok

    def patch(self, w_flat: torch.Tensor, idx: torch.Tensor) -> None:
        self.wb.index_copy_(0, idx, w_flat.index_select(0, idx).to(torch.bfloat16))
        self._wb_valid = w_flat.data_ptr()
        self._wb_sig = self._write_sig()

    def collect_shadow_grads(self) -> None:
        """g += the shadow's bf16 gradients (flat order); clears them.  When
        most parameters accumulated their gradient straight into ``g`` (no
        ``.grad``: ops/transformer.py ``grad_sinks``) only the others are
        added, one slice each."""
        have = [p.grad is not None for p in self.shadow_params]
        if sum(have) * 2 < len(have):
            dst, src = [], []
            for p, o, n in zip(self.shadow_params, self.offsets, self.numels):
                if p.grad is not None:
                    dst.append(self.g[o:o + n])
                    src.append(p.grad.reshape(-1))
                    p.grad = None
            if dst:
                torch._foreach_add_(dst, src)
            return
        gs = []
        for p, n in zip(self.shadow_params, self.numels):
            gs.append(p.grad.reshape(-1) if p.grad is not None
                      else torch.zeros(n, dtype=torch.bfloat16, device=self.device))
            p.grad = None
        torch.cat(gs, out=self.gb)
        self.g.add_(self.gb)

    def grad_sink_map(self):
        """{id(shadow param): its fp32 view of g} for ops/transformer.py grad_sinks."""
        if getattr(self, "_sink_map", None) is None:
            self._sink_map = {id(p): self.g[o:o + n].view(s) for p, o, n, s in
                              zip(self.shadow_params, self.offsets, self.numels, self.shapes)}
        return self._sink_map

    def ranges_of(self, params) -> List[Tuple[int, int]]:
        """Flat [start, end) ranges of the given parameters."""
        pos = {id(p): (o, o + n) for p, o, n in zip(self.params, self.offsets, self.numels)}
        return [pos[id(p)] for p in params if id(p) in pos]


# reference-compatible helpers (utils.py:254-297) for tools and tests
def get_param_vec(model: nn.Module) -> torch.Tensor:
    return torch.cat([p.data.reshape(-1).float() for p in trainable_params(model)])


def set_param_vec(model: nn.Module, vec: torch.Tensor) -> None:
    start = 0
    with torch.no_grad():
        for p in trainable_params(model):
            n = p.numel()
            # through the parameter (not ``p.data``): bumps its version counter,
            # which the derived weight copies (conv images, bf16 replica) watch
            p.copy_(vec[start:start + n].view_as(p))
            start += n


def get_grad_vec(model: nn.Module) -> torch.Tensor:
    out = []
    for p in trainable_params(model):
        out.append(torch.zeros(p.numel(), device=p.device) if p.grad is None
                   else p.grad.reshape(-1).float())
    return torch.cat(out)
