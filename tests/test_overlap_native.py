"""Dense-mode overlap on the native GPU path (parallel/overlap.py): the native
weight-gradient kernels accumulate into the flat gradient and hand autograd
None, so no post-accumulate hook fires for those parameters -- they announce
the write (``ops.nn._grad_written``) instead.  This records, on ONE GPU, when
each gradient bucket would be issued during a native ResNet-9 backward (the
collective itself is replaced by a recorder: no process group is needed)."""
import numpy as np
import pytest
import torch


def _engine_and_batch(bucket_mb: float):
    from commefficient_amd import models
    from commefficient_amd.data import make_synthetic
    from commefficient_amd.data.device_loader import DeviceFedLoader
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.overlap import OverlapReducer
    from commefficient_amd.train.losses import cv_loss
    from commefficient_amd.utils.args import parse_args
    dist.init("cuda")
    args = parse_args(argv=["--dataset_name", "CIFAR10", "--synthetic", "--synthetic_size", "400",
                            "--mode", "uncompressed", "--local_momentum", "0",
                            "--virtual_momentum", "0.9", "--num_clients", "40", "--num_workers", "8",
                            "--local_batch_size", "-1", "--device", "cuda", "--dtype", "bf16"],
                      probe_port=False)
    torch.manual_seed(0)
    model = models.build_model(args, 10)
    fed = FedModel(model, cv_loss, args, num_clients=40)
    ds = make_synthetic("CIFAR10", train=True, num_clients=40, size=400, seed=0)
    loader = DeviceFedLoader(ds, 8, -1, "cuda", seed=0, augment=True, out_bf16=True)
    ovl = OverlapReducer(fed.flat, fed.flat.params, int(bucket_mb * 2 ** 20))
    return fed, ovl, next(iter(loader)), cv_loss, args


@pytest.mark.gpu
def test_native_backward_marks_buckets_ready():
    fed, ovl, batch, cv_loss, args = _engine_and_batch(1.0)
    log = []
    in_backward = [False]

    def record(b):  # stands in for the async RCCL all-reduce of bucket b
        log.append((b, in_backward[0]))
        ovl.works[b] = torch.futures.Future()
        ovl.works[b].set_result(None)
    ovl._issue = record
    assert len(ovl.buckets) >= 4, len(ovl.buckets)
    fed.flat.zero_grad()
    x, y = batch.take(np.arange(len(batch)))
    ovl.arm()
    with fed._autocast(cache=False):
        per_ex, _ = cv_loss(fed.model, fed._prep((x,)), y, args)
    in_backward[0] = True
    per_ex.float().sum().backward()
    in_backward[0] = False
    early = ovl.issued_early
    ovl.finish()
    torch.cuda.synchronize()
    n = len(ovl.buckets)
    during = sum(1 for _, inb in log if inb)
    # every parameter of ResNet-9 is written natively (convs, head) or through
    # autograd: all buckets complete inside the backward, in backward order
    assert early == during == n, (early, during, n, log)
    assert [b for b, _ in log] == list(range(n))
    ovl.remove()


@pytest.mark.gpu
def test_native_backward_grad_ready_follows_backward_order():
    """Buckets are issued while the backward still runs: the first bucket
    (the head) goes out before the last conv's gradient exists."""
    from commefficient_amd.ops import nn as nnops
    fed, ovl, batch, cv_loss, args = _engine_and_batch(0.5)
    order = []
    names = {id(p): i for i, p in enumerate(fed.flat.params)}
    listener = lambda p: order.append(names.get(id(p)))  # noqa: E731
    nnops.add_grad_ready_listener(listener)
    try:
        issued_at = []
        ovl._issue = lambda b: issued_at.append((b, len(order)))
        ovl.works = [None] * len(ovl.buckets)
        fed.flat.zero_grad()
        x, y = batch.take(np.arange(len(batch)))
        ovl.arm()
        with fed._autocast(cache=False):
            per_ex, _ = cv_loss(fed.model, fed._prep((x,)), y, args)
        per_ex.float().sum().backward()
        torch.cuda.synchronize()
    finally:
        nnops.remove_grad_ready_listener(listener)
        ovl.armed = False
        ovl.remove()
    native = [i for i in order if i is not None]
    assert len(native) >= 6, order  # the 8 native convs + head announce their writes
    # parameter indices are announced in (roughly) reverse flat order
    assert native[0] > native[-1], native
    # the first bucket was issued before the last native write
    assert issued_at and issued_at[0][1] < len(order), issued_at
