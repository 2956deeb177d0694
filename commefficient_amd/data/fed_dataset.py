"""Federated index space and client sampler.

``FedDataset`` / ``FedSampler`` follow the reference semantics
(/root/reference/CommEfficient/data_utils/fed_dataset.py:9-98,
fed_sampler.py:5-71):

* non-iid: each *natural* client (e.g. one CIFAR class) is split into
  ``num_clients / num_natural`` equal clients (remainder to the last);
* iid: a random permutation of the examples, clients get equal contiguous
  shares (the last ``extra`` clients get one more);
* ``__getitem__`` returns ``(client_id, *inputs, target)``; validation items
  have ``client_id = -1``;
* the sampler shuffles within each client; each batch picks
  ``min(W, #non-exhausted)`` clients without replacement and takes up to
  ``local_batch_size`` items from each (all remaining if -1).

Additions for the device-resident path: ``client_of(indices)`` and
``data_index(indices)`` map sampler indices to (client id, storage row)
vectorised, so a batch can be gathered on the GPU without per-item Python.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import numpy as np
import torch


class FedDataset(torch.utils.data.Dataset):
    def __init__(self, dataset_dir, dataset_name, transform=None, do_iid=False, num_clients=None,
                 train=True, download=False, seed: Optional[int] = None):
        self.dataset_dir = dataset_dir
        self.dataset_name = dataset_name
        self.transform = transform
        self.do_iid = do_iid
        self._num_clients = num_clients
        self.type = "train" if train else "val"
        if not do_iid and num_clients == 1:
            raise ValueError("can't have 1 client when non-iid")
        if not self._meta_ready():
            self.prepare_datasets(download=download)
        self._load_meta(train)
        if self.do_iid:
            rng = np.random.RandomState(seed) if seed is not None else np.random
            self.iid_shuffle = rng.permutation(len(self))
        self._dpc_cache = None

    # ---- metadata -------------------------------------------------------------
    def _meta_ready(self) -> bool:
        return os.path.exists(self.stats_fn())

    def stats_fn(self):
        return os.path.join(self.dataset_dir, "stats.json")

    def _load_meta(self, train):
        with open(self.stats_fn(), "r") as f:
            stats = json.load(f)
        self.images_per_client = np.array(stats["images_per_client"])
        self.num_val_images = stats["num_val_images"]

    def prepare_datasets(self, download=False):
        raise NotImplementedError

    @property
    def num_clients(self):
        return self._num_clients if self._num_clients is not None else len(self.images_per_client)

    @property
    def data_per_client(self):
        if self._dpc_cache is not None:
            return self._dpc_cache
        if self.do_iid:
            num_data = len(self)
            ipc = np.ones(self.num_clients, dtype=int) * num_data // self.num_clients
            extra = num_data % self.num_clients
            if extra:
                ipc[self.num_clients - extra:] += 1
            out = ipc
        else:
            new_ipc = []
            n_nat = len(self.images_per_client)
            per = self.num_clients // n_nat
            if per < 1:
                raise ValueError("num_clients must be >= number of natural clients when non-iid")
            for num_images in self.images_per_client:
                extra = num_images % per
                split = [num_images // per for _ in range(per)]
                split[-1] += extra
                new_ipc.extend(split)
            out = np.array(new_ipc)
        self._dpc_cache = out
        return out

    def __len__(self):
        if self.type == "train":
            return int(sum(self.images_per_client))
        return int(self.num_val_images)

    # ---- vectorised index maps ---------------------------------------------
    def client_of(self, indices: np.ndarray) -> np.ndarray:
        cumsum = np.cumsum(self.data_per_client)
        return np.searchsorted(cumsum, indices, side="right")

    def data_index(self, indices: np.ndarray) -> np.ndarray:
        """Flat storage row (natural-client-major order) of sampler indices."""
        return self.iid_shuffle[indices] if self.do_iid else indices

    def natural_client_of_row(self, rows: np.ndarray) -> np.ndarray:
        cumsum = np.cumsum(self.images_per_client)
        return np.searchsorted(cumsum, rows, side="right")

    # ---- item access (host path) -----------------------------------------------
    def __getitem__(self, idx):
        if self.type == "train":
            orig_idx = idx
            row = int(self.data_index(np.array([idx]))[0])
            nat = int(self.natural_client_of_row(np.array([row]))[0])
            offs = getattr(self, "_client_offsets", None)
            if offs is None or len(offs) != len(self.images_per_client) + 1:
                offs = self._client_offsets = np.concatenate([[0], np.cumsum(self.images_per_client)])
            start = int(offs[nat])
            inputs = self._get_train_item(nat, row - start)
            client_id = int(self.client_of(np.array([orig_idx]))[0])
        else:
            inputs = self._get_val_item(idx)
            client_id = -1
        if not isinstance(inputs, tuple):
            inputs = (inputs,)
        if self.transform is not None:
            inputs = (self.transform(inputs[0]),) + tuple(inputs[1:])
        return (client_id,) + tuple(inputs)

    def _get_train_item(self, client_id, idx_within_client):
        raise NotImplementedError

    def _get_val_item(self, idx):
        raise NotImplementedError


class FedSampler:
    """batch_sampler yielding index arrays, one federated round per batch
    (/root/reference/CommEfficient/data_utils/fed_sampler.py:5-71).

    Resumable: ``state_dict()`` holds the RNG state at the start of the
    current epoch and ``pos`` (rounds drawn so far in it); after
    ``load_state_dict`` the next epoch replays the same draws and skips the
    first ``pos`` rounds, so a resumed run sees exactly the rounds it would
    have seen."""

    def __init__(self, dataset: FedDataset, num_workers: int, local_batch_size: int,
                 shuffle_clients: bool = True, seed: Optional[int] = None):
        self.dataset = dataset
        self.num_workers = num_workers
        self.local_batch_size = local_batch_size
        self.shuffle_clients = shuffle_clients
        # an explicit RandomState makes every rank draw the same client sets
        self.rng = np.random.RandomState(seed) if seed is not None else np.random
        self.pos = 0  # rounds drawn in the current epoch
        self._epoch_state = None
        self._skip = 0

    def __iter__(self):
        rng = self.rng
        self._epoch_state = rng.get_state()
        self.pos = 0
        skip, self._skip = self._skip, 0
        dpc = self.dataset.data_per_client
        cumsum = np.hstack([[0], np.cumsum(dpc)])
        permuted = np.hstack([s + rng.permutation(u) for s, u in zip(cumsum, dpc)]).astype(np.int64)
        cur = np.zeros(self.dataset.num_clients, dtype=np.int64)
        while True:
            nonexhausted = np.where(cur < dpc)[0]
            if len(nonexhausted) == 0:
                break
            nw = min(self.num_workers, len(nonexhausted))
            workers = rng.choice(nonexhausted, nw, replace=False)
            remaining = dpc[workers] - cur[workers]
            if self.local_batch_size == -1:
                sizes = remaining
            else:
                sizes = np.clip(remaining, 0, self.local_batch_size)
            starts = cumsum[workers] + cur[workers]
            self.pos += 1
            if self.pos > skip:
                r = np.concatenate([permuted[s:s + n] for s, n in zip(starts, sizes)])
                yield r
            cur[workers] += sizes

    def state_dict(self, pos: Optional[int] = None):
        """RNG state at the start of the current epoch + rounds consumed
        (``pos``: override, e.g. the rounds the driver actually processed)."""
        pos = self.pos if pos is None else pos
        # pos 0 = between epochs: the next epoch starts from the current state
        st = self._epoch_state if (pos > 0 and self._epoch_state is not None) \
            else self.rng.get_state()
        return {"keys": torch.from_numpy(np.asarray(st[1], dtype=np.int64)),
                "rng_pos": int(st[2]), "has_gauss": int(st[3]), "gauss": float(st[4]),
                "pos": int(pos)}

    def load_state_dict(self, sd):
        keys = sd["keys"].numpy().astype(np.uint32)
        self.rng.set_state(("MT19937", keys, int(sd["rng_pos"]), int(sd["has_gauss"]),
                            float(sd["gauss"])))
        self._skip = int(sd["pos"])

    def __len__(self):
        return len(self.dataset)
