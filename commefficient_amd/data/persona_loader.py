"""Round loaders for the PersonaChat datasets: the host builds token records
only for the rows this rank computes, pads them to the selection's max length
and ships the round's int64 tensors in ONE pinned H2D copy (non_blocking),
split into views on the device."""
from __future__ import annotations


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
    if not all(t.dtype == torch.int64 for t in ts):
        return [h2d(t, device) for t in ts]
    flat = h2d(np.concatenate([t.numpy().reshape(-1) for t in ts]), device)
    out, o = [], 0
    for t in ts:
        out.append(flat[o:o + t.numel()].view(t.shape))
        o += t.numel()
    return out


# --train_dataloader_workers: the records of the next rounds are built in
# worker processes while the current round runs (the reference's DataLoader
# workers, gpt2_train.py:155-166).  Forked, not spawned: the children inherit
# the dataset and never touch the GPU (as PyTorch DataLoader workers), and no
# process that initialised the GPU execs another program.
_WORKER_DS = None


def _build_records(idx):
    """Worker: the records of dataset items ``idx``, token lists as int32
    arrays (pickled compactly; collate pads them like lists)."""
    out = []
    for i in idx:
        rec = _WORKER_DS[int(i)][1]
        out.append({"input_ids": [np.asarray(x, dtype=np.int32) for x in rec["input_ids"]],
                    "token_type_ids": [np.asarray(x, dtype=np.int32) for x in rec["token_type_ids"]],
                    "lm_labels": [np.asarray(x, dtype=np.int32) for x in rec["lm_labels"]],
                    "mc_token_ids": list(rec["mc_token_ids"]), "mc_labels": rec["mc_labels"]})
    return out


class PersonaFedLoader:
    def __init__(self, dataset, num_workers, local_batch_size, device, seed, workers=0, prefetch=2):
        self.dataset = dataset
        self.sampler = FedSampler(dataset, num_workers, local_batch_size, seed=seed)
        self.device = device
        self.workers = int(workers)
        self.prefetch = max(1, int(prefetch))
        self._pool = None

    def _executor(self):
        if self._pool is None:
            import multiprocessing as mp
            from concurrent.futures import ProcessPoolExecutor
            global _WORKER_DS
            _WORKER_DS = self.dataset
            self._pool = ProcessPoolExecutor(max_workers=self.workers, mp_context=mp.get_context("fork"))
        return self._pool

    def close(self):
        if self._pool is not None:
            self._pool.shutdown(wait=False, cancel_futures=True)
            self._pool = None

    def __len__(self):
        return len(self.dataset)

    def __iter__(self):
        self.epoch = getattr(self, "epoch", 0) + 1
        if self.workers <= 0:
            for r in self.sampler:
                yield self.make_batch(r)
            return
        # the next ``prefetch`` rounds' records are built in the workers while
        # this one is consumed (each round's items split across the workers)
        from collections import deque
        ex = self._executor()
        ahead = deque()

        def submit(r):
            parts = np.array_split(np.asarray(r), min(self.workers, len(r)))
            return r, [ex.submit(_build_records, p) for p in parts if len(p)]

        it = iter(self.sampler)
        for r in it:
            ahead.append(submit(r))
            if len(ahead) > self.prefetch:
                break
        while ahead:
            r, futs = ahead.popleft()
            nxt = next(it, None)
            if nxt is not None:
                ahead.append(submit(nxt))
            yield self.make_batch(r, futs)

    def state_dict(self, pos=None):
        """Sampler position (resume mid-epoch) -- the records themselves are a
        pure function of the item index."""
        return {"sampler": self.sampler.state_dict(pos), "epoch": max(0, getattr(self, "epoch", 0) - 1)}

    def load_state_dict(self, sd):
        self.sampler.load_state_dict(sd["sampler"])
        self.epoch = int(sd.get("epoch", 0))

    def make_batch(self, r, futures=None):
        ds, dev = self.dataset, self.device
        cids = ds.client_of(r)
        built = []

        def take(pos, r=r):
            if futures is not None:
                if not built:
                    for f in futures:
                        built.extend(f.result())
                recs = [built[int(i)] for i in np.asarray(pos).reshape(-1)]
            else:
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
