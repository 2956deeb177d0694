"""Deterministic replay: the whole GPU FetchSGD round at the
headline sketch geometry (5 x 500,000) -- native convs with fixed-order split-K
reductions, the region sketch (default; no atomics, any geometry incl. GPT-2's:
tests/test_sketch_region.py) or the planned csvec-layout sketch, radix-select
top-k, fused head/loss -- is a pure function of its inputs: two runs from the
same seed end with bit-identical weights and server state.  (The csvec
layout's binned fallback uses LDS float atomics and is not bitwise
reproducible run to run; ranks still agree, since every rank applies the same
all-reduced table.)"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(rounds: int, encode: str):
    from commefficient_amd import models
    from commefficient_amd.data import make_synthetic
    from commefficient_amd.data.device_loader import DeviceFedLoader
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.server import FedOptimizer
    from commefficient_amd.train.losses import cv_loss
    from commefficient_amd.utils.args import parse_args
    dist.init("cuda")
    args = parse_args(argv=["--dataset_name", "CIFAR10", "--synthetic", "--synthetic_size", "800",
                            "--mode", "sketch", "--error_type", "virtual", "--local_momentum", "0",
                            "--virtual_momentum", "0.9", "--k", "50000", "--num_rows", "5",
                            "--num_cols", "500000", "--num_clients", "80", "--num_workers", "16",
                            "--local_batch_size", "-1", "--weight_decay", "5e-4",
                            "--device", "cuda", "--encode", encode], probe_port=False)
    torch.manual_seed(0)
    ds = make_synthetic("CIFAR10", train=True, num_clients=80, size=800, seed=1)
    loader = DeviceFedLoader(ds, 16, -1, "cuda", seed=2, augment=True, out_bf16=True)
    model = models.build_model(args, 10)
    fed = FedModel(model, cv_loss, args, num_clients=80)
    opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.05), args, fed)
    it = iter(loader)
    for _ in range(rounds):
        fed(next(it))
        opt.step()
    torch.cuda.synchronize()
    if encode == "region":
        assert fed.sketch.region is not None, "expected the region sketch kernels"
    else:
        assert fed.sketch._use_plan(), "expected the planned (atomic-free) sketch kernels"
    return fed.w.clone(), fed.server.V.clone(), fed.server.E.clone()


@pytest.mark.parametrize("encode", ["region", "planned"])
def test_fetchsgd_rounds_replay_bitwise(encode):
    a = _run(3, encode)
    b = _run(3, encode)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert torch.isfinite(a[0]).all()
