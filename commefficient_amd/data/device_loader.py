"""Device-resident federated data loading.

The reference builds every batch on the host (PIL decode + torchvision
transforms per item in a DataLoader) and pickles it to the workers through
queues (/root/reference/CommEfficient/cv_train.py:254-287,
fed_aggregator.py:303-307).  On MI355X the whole uint8 image set sits in HBM
(CIFAR-10: 150 MB of 288 GB) and a round is materialised by ONE kernel that
gathers the round's rows and applies crop/flip/normalise, writing bf16 NHWC
(``ops.augment_u8_nhwc``).  Only the rows of the clients assigned to this
rank are materialised.  The sampler (``FedSampler`` semantics, seeded
identically on every rank) runs on the host and costs microseconds.
"""
from __future__ import annotations

from typing import Iterator, Optional

import numpy as np
import torch

from .. import ops
from ..parallel.dist import h2d
from ..parallel.fed_model import RoundBatch
from .fed_dataset import FedSampler


_GOLDEN = 0x9E3779B97F4A7C15
_MASK64 = (1 << 64) - 1


class DeviceImageSource:
    def __init__(self, dataset, device, augment: bool, pad: int = 4, flip: bool = True,
                 out_bf16: bool = True):
        images, targets = dataset.arrays()
        self.device = torch.device(device)
        self.data = torch.from_numpy(np.ascontiguousarray(images)).to(self.device)
        self.targets = torch.from_numpy(np.asarray(targets, dtype=np.int64)).to(self.device)
        mean = torch.tensor(dataset.mean, dtype=torch.float32)
        std = torch.tensor(dataset.std, dtype=torch.float32)
        self.mean = mean.to(self.device)
        self.inv_std = (1.0 / std).to(self.device)
        self.augment = augment
        self.pad = pad if augment else 0
        self.flip = flip if augment else False
        self.out_bf16 = out_bf16 and self.device.type == "cuda"

    def gather(self, rows: np.ndarray, seed: int, keys: Optional[np.ndarray] = None):
        """Batch of ``rows``; ``keys`` (default: slot index) key the per-example
        random crop/flip, so an example's augmentation does not depend on
        which rank materialises it."""
        host = np.asarray(rows, dtype=np.int64)
        if keys is not None:
            host = np.stack([host, np.asarray(keys, dtype=np.int64)])
        t = torch.from_numpy(host)
        if self.device.type == "cuda":
            t = h2d(t, self.device)
        idx, kt = (t[0], t[1]) if keys is not None else (t, None)
        if self.device.type == "cuda":  # labels gathered by the same kernel
            return ops.augment_u8_nhwc_y(self.data, idx, self.pad, self.flip, self.mean,
                                         self.inv_std, seed, self.out_bf16, kt, self.targets)
        x = ops.augment_u8_nhwc(self.data, idx, self.pad, self.flip, self.mean, self.inv_std,
                                seed, self.out_bf16, kt)
        y = self.targets[idx]
        return x, y

    def gather_device(self, idx2: torch.Tensor):
        """Batch from a device int64 [2, B] = (rows, pre-mixed keys) with seed
        0 -- the same pixels as ``gather(rows, seed, keys)`` when
        ``keys' = seed * 0x9E3779B97F4A7C15 + keys`` (mod 2^64), so the rows and
        keys ride in the round's one packed H2D copy."""
        if self.device.type == "cuda":  # labels gathered by the same kernel
            return ops.augment_u8_nhwc_y(self.data, idx2[0], self.pad, self.flip, self.mean,
                                         self.inv_std, 0, self.out_bf16, idx2[1], self.targets)
        x = ops.augment_u8_nhwc(self.data, idx2[0], self.pad, self.flip, self.mean,
                                self.inv_std, 0, self.out_bf16, idx2[1])
        return x, self.targets[idx2[0]]


class DeviceFedLoader:
    """Iterates federated training rounds as ``RoundBatch``es."""

    def __init__(self, dataset, num_workers: int, local_batch_size: int, device, seed: int,
                 augment: bool = True, out_bf16: bool = True, pad: int = 4, flip: bool = True):
        self.dataset = dataset
        self.sampler = FedSampler(dataset, num_workers, local_batch_size, seed=seed)
        self.source = DeviceImageSource(dataset, device, augment, pad=pad, flip=flip,
                                        out_bf16=out_bf16)
        self.seed = seed
        self._round = 0
        self.epoch = 0  # epochs started (the next __iter__ runs epoch ``self.epoch``)

    def __len__(self):
        return len(self.dataset)

    def __iter__(self) -> Iterator[RoundBatch]:
        ep = self.epoch
        self.epoch += 1
        for r in self.sampler:
            cids = self.dataset.client_of(r)
            rows = self.dataset.data_index(r)
            # augmentation keyed by (epoch, round in epoch): a resumed run
            # (FedSampler skip) reproduces the same pixels
            yield self.make_batch(cids, rows, key=(ep << 24) + self.sampler.pos - 1)

    def state_dict(self, pos=None):
        return {"sampler": self.sampler.state_dict(pos), "epoch": max(0, self.epoch - 1)}

    def load_state_dict(self, sd):
        self.sampler.load_state_dict(sd["sampler"])
        self.epoch = int(sd["epoch"])

    def make_batch(self, cids, rows, key=None) -> RoundBatch:
        if key is None:
            key = self._round
            self._round += 1
        rnd_seed = (self.seed * 1000003 + key) & 0x7FFFFFFFFFFF
        src = self.source

        def take(pos, rows=rows, seed=rnd_seed):
            # seed by round, key by the example's position in the round
            return src.gather(rows[pos], seed, keys=pos)

        rb = RoundBatch(cids, take, n_inputs=1)
        if src.device.type == "cuda":
            mix = np.array([(rnd_seed * _GOLDEN) & _MASK64], dtype=np.uint64)

            def index(pos, rows=rows, mix=mix):
                pos = np.asarray(pos, dtype=np.int64)
                keys = (pos.astype(np.uint64) + mix).view(np.int64)  # wraps mod 2^64
                return np.stack([np.asarray(rows, dtype=np.int64)[pos], keys])

            rb.device_index = index
            rb.device_gather = src.gather_device
        return rb


class DeviceValLoader:
    """Sequential validation batches of ``batch_size`` (client id -1)."""

    def __init__(self, dataset, batch_size: int, device, out_bf16: bool = True):
        self.dataset = dataset
        self.batch_size = batch_size
        self.source = DeviceImageSource(dataset, device, augment=False, out_bf16=out_bf16)

    def __len__(self):
        return (len(self.dataset) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        n = len(self.dataset)
        for s in range(0, n, self.batch_size):
            rows = np.arange(s, min(n, s + self.batch_size))
            cids = np.full(len(rows), -1, dtype=np.int64)
            src = self.source

            def take(pos, rows=rows):
                return src.gather(rows[pos], 0)

            yield RoundBatch(cids, take, n_inputs=1)
