"""Server update, replicated on every rank.

Equivalent of ``FedOptimizer`` + ``get_server_update`` and the five
``_server_helper_*`` functions (/root/reference/CommEfficient/
fed_aggregator.py:383-613).

Every rank holds ``V`` (virtual momentum) and ``E`` (virtual error) --
``(r, c)`` in sketch mode, ``(d,)`` otherwise -- and, after the round's single
all-reduce, runs the identical, deterministic update below, so weights never
travel (no PS, no host round-trip).  All hot steps are native
kernels: ``momentum_ef`` (K6), ``cs_query`` + ``topk_abs`` (K7, K8),
``cs_zero_buckets`` (K10), ``zero_at`` (K11), ``sparse_apply`` /
``dense_apply`` (K12 + K13 change tracking).

Mode math (G = summed transmit / B):
  uncompressed  V = rho V + G (+ N(0, sigma^2) if dp_mode=server); w -= lr V
  true_topk     V = rho V + G; E += V; (i,v) = topk(E,k); E[i] = V[i] = 0;
                participating clients' local velocities zeroed at i; w[i] -= lr v
  local_topk    V = rho V + G; w -= lr V
  fedavg        V = rho V + G; w -= V           (lr folded into the clients)
  sketch        V = rho V + S; E += V (virtual) | E = V (local / none);
                (i,v) = topk(median-estimate(E), k); zero E (virtual) and V at
                the r buckets of every recovered coordinate; w[i] -= lr v

Documented divergences from the reference:
* sketch with ``--error_type none``: the reference never fills ``Verror`` and
  so un-sketches an all-zero table (no learning); here "none" un-sketches
  ``V`` directly (FetchSGD without error accumulation).
* heavy-hitter masking zeroes the buckets of the recovered coordinates
  directly instead of ``S(delta).nonzero()``; identical unless two recovered
  coordinates cancel exactly inside a bucket.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops.nn import weights_begin_update, weights_end_update
from .. import ops
from ..ops import CSVec
from . import dist


class FedOptimizer(torch.optim.Optimizer):
    """Wraps a torch optimizer only for its ``param_groups`` (LR schedule
    interface); ``step()`` performs the federated server update."""

    def __init__(self, optimizer: torch.optim.Optimizer, args, fed_model=None):
        # deliberately not calling Optimizer.__init__: we borrow param_groups
        self.args = args
        self.param_groups = optimizer.param_groups
        self.defaults = getattr(optimizer, "defaults", {})
        self.state = {}
        self._optimizer_step_pre_hooks = {}
        self._optimizer_step_post_hooks = {}
        self.fed_model = fed_model
        if fed_model is not None:
            fed_model.attach_optimizer(self)

    # ------------------------------------------------------------------ LR
    def get_lr(self):
        """Scalar when there is one param group, else a per-coordinate [d]
        vector on the device (fed_aggregator.py:411-427)."""
        if len(self.param_groups) == 1:
            return float(self.param_groups[0]["lr"])
        fm = self.fed_model
        lrs = tuple(float(g["lr"]) for g in self.param_groups)
        if getattr(self, "_lr_cache_key", None) == lrs:
            return self._lr_vec
        vec = torch.zeros(fm.d, device=fm.device)
        for g, lr in zip(self.param_groups, lrs):
            for (s, e) in fm.flat.ranges_of(g["params"]):
                vec[s:e] = lr
        self._lr_cache_key, self._lr_vec = lrs, vec
        return vec

    def step(self, closure=None):
        self.fed_model.server_step(self.get_lr())

    def zero_grad(self, set_to_none: bool = False):
        raise NotImplementedError("Please call zero_grad() on the model instead")


class ServerState:
    """Replicated server state + the mode-specific update."""

    def __init__(self, args, d: int, device, sketch: Optional[CSVec], shard=None):
        """``shard = (rank, world)``: the sharded FetchSGD server (region
        family on > 1 rank).  The round's sketch tables are reduce-scattered
        by region group (group-major layout, ``CSVec.set_group_layout``), and
        rank r keeps only its groups [r Gp, (r+1) Gp) of V and E: the momentum /
        error feedback, the median query and the top-k of its groups'
        coordinates run on 1/N of the table, the k-lists are all-gathered as
        packed words and merged in ascending coordinate order (csrc/shard.hip),
        so the global top-k -- ties to the lower index -- is bitwise the
        replicated one; each rank then zeroes the heavy hitters' buckets of
        its own groups and applies the (replicated) weight step."""
        self.args = args
        self.d = d
        self.device = device
        self.sketch = sketch
        self.shard = None
        mode = args.mode
        shape = (args.num_rows, args.num_cols) if mode == "sketch" else (d,)
        if shard is not None and mode == "sketch":
            rank, world = shard
            h = sketch.region
            Gp = h.shard_groups(world)
            self.shard = (int(rank), int(world), rank * Gp, Gp)
            shape = (Gp, args.num_rows, h.g * h.m)
        self.V = torch.zeros(shape, device=device)
        self.E = torch.zeros(shape, device=device)
        self.noise_round = 0

    def update(self, G: torch.Tensor, lr, w: torch.Tensor, last_mod: torch.Tensor, round_idx: int,
               client_state=None, participating=None, hist: Optional[torch.Tensor] = None,
               gscale: float = 1.0, step: Optional[torch.Tensor] = None):
        """Apply one server step.  ``gscale * G`` is the summed transmit / B
        (the scale is folded into the momentum kernel); ``hist`` is the
        accountant's change histogram, updated with the stamps.  ``step``
        (device int32 [2] = lr bits, round) replaces the scalar lr / round_idx
        in the apply kernels of a recorded round (parallel/tape.py).  Returns
        (idx, vals) for sparse modes (the un-scaled update), else None."""
        a = self.args
        rho = float(a.virtual_momentum)
        lr_s, lr_v = (lr, None) if not torch.is_tensor(lr) else (0.0, lr)
        mode = a.mode
        # kept derived weight copies (bf16 conv images, bf16 replica): stale from
        # here on, unless the step is sparse (then the k changed coordinates
        # are patched into them)
        img_sync = weights_begin_update(w)
        if mode == "sketch" and self.shard is not None:
            idx, vals = self._sketch_sharded(G, rho, gscale, w, lr_s, lr_v, last_mod, round_idx, hist, step)
            weights_end_update(img_sync, w, idx)
            return idx, vals
        if mode == "sketch":
            et = a.error_type
            virt = et == "virtual"
            src = self.E if virt else self.V  # local / none: un-sketch V itself (module docstring)
            # the momentum step (V = rho V + G/B; virtual: E += V) goes with the
            # unsketch: the region GPU query applies it while staging the table
            mom = (self.V, G, rho, gscale, "virtual" if virt else "none")
            sk = self.sketch.like(src)
            ctx = dist.ctx()
            if ctx.world_size > 1 and getattr(a, "shard_unsketch", "on") in ("on", "query"):
                # every rank estimates 1/N of the coordinates and the k-lists
                # are merged (bitwise the replicated result, ops/sketch.py)
                idx, vals = sk.unsketch_sparse_sharded(a.k, ctx.rank, ctx.world_size,
                                                       dist.all_gather_rows, mom=mom)
            else:
                idx, vals = sk.unsketch_sparse(a.k, mom=mom)
            # error feedback (virtual) + momentum-factor masking in sketch space,
            # and the weight step (one kernel for the region family)
            other = self.V if et == "virtual" else None
            # (region family: one fused kernel; csvec layout: zeroing, then the apply)
            if not sk.zero_heavy_hitters_apply(idx, vals, other, w, lr_s, lr_v, last_mod, round_idx, hist,
                                               step):
                sk.zero_heavy_hitters(idx, vals, other)
                ops.sparse_apply(w, idx, vals, lr_s, lr_v, last_mod, round_idx, step, hist)
            weights_end_update(img_sync, w, idx)
            return idx, vals
        if mode == "true_topk":
            ops.momentum_ef(self.V, self.E, G, rho, gscale, "virtual")
            idx, vals = ops.topk_abs(self.E, a.k, ops.topk_hint(("true_topk", self.d, a.k), self.E.device))
            if client_state is not None and participating is not None:
                client_state.zero_velocity_at(participating, idx)
            ops.zero_at(idx, self.E, self.V)
            ops.sparse_apply(w, idx, vals, lr_s, lr_v, last_mod, round_idx, step, hist)
            weights_end_update(img_sync, w, idx)
            return idx, vals
        if mode in ("local_topk", "uncompressed"):
            ops.momentum_ef(self.V, None, G, rho, gscale, "none")
            if mode == "uncompressed" and a.do_dp and a.dp_mode == "server":
                # the reference adds the noise to Vvelocity itself (``grad`` aliases
                # it, fed_aggregator.py:502-508), so it persists in the momentum;
                # same seed/offset on every rank keeps the replicas identical
                ops.clip_noise(self.V, None, 0.0, a.noise_multiplier, seed=a.seed * 7919 + 17,
                               offset=self.noise_round * self.d)
                self.noise_round += 1
            ops.dense_apply(w, self.V, lr_s, lr_v, last_mod, round_idx, step, hist)
            return None
        if mode == "fedavg":
            ops.momentum_ef(self.V, None, G, rho, gscale, "none")
            ops.dense_apply(w, self.V, 1.0, None, last_mod, round_idx, step, hist)
            return None
        raise ValueError(mode)

    def _sketch_sharded(self, G, rho, gscale, w, lr_s, lr_v, last_mod, round_idx, hist, step):
        from ..ops import sketch_region as _rg
        a = self.args
        rank, world, g0, Gp = self.shard
        k = int(a.k)
        h = self.sketch.region
        virt = a.error_type == "virtual"
        src = self.E if virt else self.V
        mom = (self.V, G.view(self.V.shape), rho, gscale, "virtual" if virt else "none")
        hint = ops.topk_hint(("unsketch_groups", self.d, k, rank, world), self.device)
        li, lv, cmap = _rg.topk(h, src, k, hint, mom=mom, g0=g0)
        pack = ops.pack_topk(li, lv, cmap, h.m)
        allp = dist.all_gather_rows(pack.view(1, k))
        vm, im = ops.merge_packed(allp.view(-1), world, k)
        pos, vals = ops.topk_abs(vm, k, ops.topk_hint(("merge_groups", self.d, k, world), self.device))
        idx = ops.gather_i64(im, pos)
        sk = self.sketch.like(src)
        other = self.V if virt else None
        if not sk.zero_heavy_hitters_apply(idx, vals, other, w, lr_s, lr_v, last_mod, round_idx, hist,
                                           step, g0=g0):
            _rg.zero_buckets(h, src, other, idx, vals, g0=g0)
            ops.sparse_apply(w, idx, vals, lr_s, lr_v, last_mod, round_idx, step, hist)
        return idx, vals

    def state_dict(self):
        if self.shard is not None:  # every rank's groups, in the row-major [r, c] format
            h = self.sketch.region
            rank, world, g0, Gp = self.shard
            V = h.row_major(dist.all_gather_rows(self.V.contiguous()))
            E = h.row_major(dist.all_gather_rows(self.E.contiguous()))
            return {"V": V.cpu(), "E": E.cpu(), "noise_round": self.noise_round}
        return {"V": self.V.cpu(), "E": self.E.cpu(), "noise_round": self.noise_round}

    def load_state_dict(self, sd):
        if self.shard is not None:
            h = self.sketch.region
            rank, world, g0, Gp = self.shard
            self.V.copy_(h.group_major(sd["V"].to(self.device), world)[g0:g0 + Gp])
            self.E.copy_(h.group_major(sd["E"].to(self.device), world)[g0:g0 + Gp])
        else:
            self.V.copy_(sd["V"])
            self.E.copy_(sd["E"])
        self.noise_round = int(sd.get("noise_round", 0))
