"""Independent float64 numpy simulation of one federated round for a linear
model ``y_hat = w . x`` with per-example loss ``(w.x - y)^2``, following the
reference's math (fed_worker.py:184-230, 249-335;
fed_aggregator.py:483-613).  Used to check the engine end to end.

Replaces the dead analytic oracle of /root/reference/CommEfficient/
unit_test.py:79-193 (whose values are internally inconsistent):
values here are derived, not copied.
"""
from __future__ import annotations

import numpy as np


def topk_mask(v, k):
    """lower index wins ties (same rule as the native radix select)"""
    key = np.abs(v.astype(np.float32)).astype(np.float64)
    order = sorted(range(len(v)), key=lambda i: (-key[i], i))[:k]
    m = np.zeros(len(v), bool)
    m[order] = True
    return m


class LinearFedOracle:
    def __init__(self, d, mode, k=1, rho=0.0, rho_l=0.0, error_type="none", wd=0.0,
                 num_workers=1, fedavg_lr=0.0, fedavg_epochs=1, fedavg_bs=-1, topk_down=False,
                 max_grad_norm=None, dp_clip=None):
        self.topk_down, self.max_grad_norm, self.dp_clip = topk_down, max_grad_norm, dp_clip
        self.wc = {}
        self.d, self.mode, self.k = d, mode, k
        self.rho, self.rho_l, self.et, self.wd, self.W = rho, rho_l, error_type, wd, num_workers
        self.w = np.zeros(d)
        self.V = np.zeros(d)
        self.E = np.zeros(d)
        self.u, self.e = {}, {}
        self.fedavg_lr = fedavg_lr
        self.fe, self.fbs = fedavg_epochs, fedavg_bs

    def mean_grad(self, w, X, y):
        r = X @ w - y
        g = (2 * X * r[:, None]).mean(0)
        if self.max_grad_norm is not None and self.mode != "sketch_exact":
            nrm = np.linalg.norm(g)
            if nrm > self.max_grad_norm:
                g = g * (self.max_grad_norm / nrm)
        g = g + self.wd / self.W * w
        if self.dp_clip is not None:  # utils.clip_grad, noise_multiplier 0
            nrm = np.linalg.norm(g)
            if nrm > self.dp_clip:
                g = g * (self.dp_clip / nrm)
        return g

    def round(self, clients, lr):
        """clients: list of (client_id, X[n,d], y[n])"""
        B = sum(len(y) for _, _, y in clients)
        tot = np.zeros(self.d)
        for c, X, y in clients:
            n = len(y)
            if self.mode == "fedavg":
                wl = self.w.copy()
                bs = n if self.fbs == -1 else self.fbs
                step = 0
                for _ in range(self.fe):
                    for s in range(0, n, bs):
                        g = self.mean_grad(wl, X[s:s + bs], y[s:s + bs])
                        wl -= g * self.fedavg_lr
                        step += 1
                tot += (self.w - wl) * n
                continue
            wloc = self.w
            if self.topk_down:  # fed_worker.py:232-247, state written back
                wc = self.wc.setdefault(c, np.zeros(self.d))
                diff = self.w - wc
                wc[:] = wc + np.where(topk_mask(diff, self.k), diff, 0.0)
                wloc = wc.copy()
            g = self.mean_grad(wloc, X, y) * n
            t = g
            if self.rho_l > 0:
                u = self.u.setdefault(c, np.zeros(self.d))
                u[:] = self.rho_l * u + g
                t = u
            if self.et == "local":
                e = self.e.setdefault(c, np.zeros(self.d))
                e += t
                t = e
            if self.mode == "local_topk":
                m = topk_mask(t, self.k)
                sent = np.where(m, t, 0.0)
                if self.et == "local":
                    self.e[c][m] = 0
                if self.rho_l > 0:
                    self.u[c][m] = 0
                t = sent
            tot += t
        G = tot / B
        if self.mode in ("uncompressed", "local_topk"):
            self.V = self.rho * self.V + G
            self.w -= lr * self.V
        elif self.mode == "fedavg":
            self.V = self.rho * self.V + G
            self.w -= self.V
            self.fedavg_lr = lr
        elif self.mode in ("true_topk", "sketch_exact"):
            # with a collision-free sketch, FetchSGD == true top-k with error
            # feedback and momentum masking
            self.V = self.rho * self.V + G
            self.E += self.V
            m = topk_mask(self.E, self.k)
            upd = np.where(m, self.E, 0.0)
            nz = m & (upd != 0)
            if self.rho_l > 0:
                for c, _, _ in clients:
                    if c in self.u:
                        self.u[c][nz] = 0
            self.E[nz] = 0
            self.V[nz] = 0
            self.w -= lr * upd
        return self.w.copy()
