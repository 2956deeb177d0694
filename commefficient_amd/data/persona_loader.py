"""Round loaders for the PersonaChat datasets: the host builds token records
only for the rows this rank computes, pads them to the selection's max length
and ships the round's int64 tensors in ONE pinned H2D copy (non_blocking),
split into views on the device."""
from __future__ import annotations

import os

import numpy as np
import torch

from ..parallel.fed_model import RoundBatch
from .fed_dataset import FedSampler
from .fed_persona import collate, label_positions


def _to_dev(ts, device):
    """Host tensors -> device tensors of the same shapes: one packed H2D copy
    when they are all int64 on a GPU (a copy per tensor cost a pinned-ring
    round trip each at the start of every GPT-2 round, where the GPU waits)."""
    from ..parallel.dist import h2d
    if torch.device(device).type != "cuda":
        return list(ts)
    if not all(t.dtype == torch.int64 for t in ts) or os.environ.get("COMMEFF_PERSONA_PACK") == "0":
        return [h2d(t, device) for t in ts]
    flat = h2d(np.concatenate([t.numpy().reshape(-1) for t in ts]), device)
    out, o = [], 0
    for t in ts:
        out.append(flat[o:o + t.numel()].view(t.shape))
        o += t.numel()
    return out


class PersonaFedLoader:
    def __init__(self, dataset, num_workers, local_batch_size, device, seed):
        self.dataset = dataset
        self.sampler = FedSampler(dataset, num_workers, local_batch_size, seed=seed)
        self.device = device

    def __len__(self):
        return len(self.dataset)

    def __iter__(self):
        self.epoch = getattr(self, "epoch", 0) + 1
        for r in self.sampler:
            yield self.make_batch(r)

    def state_dict(self, pos=None):
        """Sampler position (resume mid-epoch) -- the records themselves are a
        pure function of the item index."""
        return {"sampler": self.sampler.state_dict(pos), "epoch": max(0, getattr(self, "epoch", 0) - 1)}

    def load_state_dict(self, sd):
        self.sampler.load_state_dict(sd["sampler"])
        self.epoch = int(sd.get("epoch", 0))

    def make_batch(self, r):
        ds, dev = self.dataset, self.device
        cids = ds.client_of(r)

        def take(pos, r=r):
            recs = [ds[int(i)][1] for i in r[pos]]
            host = collate(recs)
            ids, mc, lab, mcl, tt, lp = _to_dev(list(host) + [label_positions(host[2])], dev)
            # sequence lengths stay on the host (mc token = last real token):
            # the transformer runs its token-wise ops on the real tokens only
            lens = host[1] + 1
            return ids, mc, lab, tt, lp, lens, mcl

        return RoundBatch(cids, take, n_inputs=6)


class PersonaValLoader:
    def __init__(self, dataset, batch_size, device):
        self.dataset, self.batch_size, self.device = dataset, batch_size, device

    def __len__(self):
        return (len(self.dataset) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        n = len(self.dataset)
        for s in range(0, n, self.batch_size):
            rows = np.arange(s, min(n, s + self.batch_size))
            ds, dev = self.dataset, self.device

            def take(pos, rows=rows):
                recs = [ds[int(i)][1] for i in rows[pos]]
                ids, mc, lab, mcl, tt = _to_dev(collate(recs), dev)
                return ids, mc, lab, tt, mcl

            yield RoundBatch(np.full(len(rows), -1, dtype=np.int64), take, n_inputs=4)
