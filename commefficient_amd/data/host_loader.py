"""Host-decoded loaders (PIL folder datasets such as ImageNet) with the
reference's DataLoader wiring (cv_train.py:254-287): FedSampler as
``batch_sampler`` for train, sequential ``valid_batch_size * W`` batches for
val.  Batches are ``(client_ids, images, targets)`` tuples."""
from __future__ import annotations

import torch

from .fed_dataset import FedSampler


def _collate(items):
    cids = torch.tensor([it[0] for it in items], dtype=torch.int64)
    x = torch.stack([it[1] for it in items])
    y = torch.tensor([it[2] for it in items], dtype=torch.int64)
    return cids, x, y


def host_fed_loaders(args, train_ds, test_ds, transforms):
    train_ds.transform, test_ds.transform = transforms
    sampler = FedSampler(train_ds, args.num_workers, args.local_batch_size, seed=args.seed)
    train = torch.utils.data.DataLoader(train_ds, batch_sampler=sampler, collate_fn=_collate,
                                        num_workers=args.train_dataloader_workers,
                                        pin_memory=args.device == "cuda")
    test = torch.utils.data.DataLoader(test_ds, batch_size=args.valid_batch_size * args.num_workers,
                                       shuffle=False, collate_fn=_collate,
                                       num_workers=args.val_dataloader_workers)
    return train, test
