"""Batched FedAvg local SGD (parallel/fed_model.py ``_fedavg_batched``): the
clients' multi-step local SGD (fed_worker.py:61-113) in lockstep under
torch.func.vmap must equal the one-client-at-a-time path."""
import copy

import pytest
import torch
import torch.nn.functional as F

from commefficient_amd import models
from commefficient_amd.models.resnets import BasicBlock, ResNet
from commefficient_amd.parallel import dist
from commefficient_amd.parallel.fed_model import FedModel
from commefficient_amd.parallel.server import FedOptimizer
from commefficient_amd.train.losses import cv_loss
from commefficient_amd.utils.args import parse_args


def _engine(batched, extra, model):
    dist.init("cpu")
    args = parse_args(argv=["--dataset_name", "CIFAR10", "--mode", "fedavg", "--error_type", "none",
                            "--local_momentum", "0", "--virtual_momentum", "0.5",
                            "--num_workers", "4", "--num_clients", "4", "--local_batch_size", "-1",
                            "--device", "cpu", "--dtype", "fp32", "--fedavg_batched", batched]
                      + extra, probe_port=False)
    fed = FedModel(model, cv_loss, args, num_clients=4)
    opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1), args, fed)
    return fed, opt


@pytest.mark.parametrize("extra", [
    ["--fedavg_batch_size", "3"],
    ["--fedavg_batch_size", "2", "--num_fedavg_epochs", "2", "--fedavg_lr_decay", "0.9"],
    ["--fedavg_batch_size", "3", "--weight_decay", "5e-3", "--max_grad_norm", "0.05"],
])
def test_batched_local_sgd_equals_sequential(extra):
    """ResNet-9 (no BatchNorm): three rounds, weights and per-client losses."""
    torch.manual_seed(0)
    base = models.ResNet9(channels={"prep": 4, "layer1": 8, "layer2": 8, "layer3": 16})
    res = {}
    for b in ("on", "off"):
        fed, opt = _engine(b, extra, copy.deepcopy(base))
        g = torch.Generator().manual_seed(3)
        losses = []
        for _ in range(3):
            x = torch.randn(24, 3, 32, 32, generator=g)
            y = torch.randint(0, 10, (24,), generator=g)
            out = fed((torch.arange(4).repeat_interleave(6), x, y))
            opt.param_groups[0]["lr"] = 0.1
            opt.step()
            losses.append(out[0].clone())
        res[b] = (fed.w.clone(), torch.stack(losses))
    torch.testing.assert_close(res["on"][0], res["off"][0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(res["on"][1], res["off"][1], rtol=1e-4, atol=1e-5)


def test_vmapped_batchnorm_steps_exact_in_fp64():
    """The vmapped step itself (per-client weights AND BatchNorm buffers as
    batched inputs) equals per-client autograd exactly in float64 -- in
    fp32 a random-init BN ResNet on 8-image steps amplifies rounding by
    ~1e4, so the engine-level comparison with BN is done in fp64 here."""
    from torch.func import grad, vmap
    from torch.nn.utils.stateless import _reparametrize_module
    torch.manual_seed(1)
    m = ResNet(BasicBlock, [1, 1, 1, 1], num_classes=10, input_hw=32).double().train()
    G, n = 3, 8
    g = torch.Generator().manual_seed(3)
    x = torch.randn(G, n, 3, 32, 32, generator=g, dtype=torch.float64)
    y = torch.randint(0, 10, (G, n), generator=g)
    P = {k: v.detach().unsqueeze(0).repeat((G,) + (1,) * v.dim()) for k, v in m.named_parameters()}
    B = {k: v.detach().unsqueeze(0).repeat((G,) + (1,) * v.dim()).clone()
         for k, v in m.named_buffers()}

    def loss(p, b, xx, yy):
        with _reparametrize_module(m, {**p, **b}):
            return F.cross_entropy(m(xx), yy)

    gf = vmap(grad(loss))
    for s in (0, 4):
        gr = gf(P, B, x[:, s:s + 4], y[:, s:s + 4])
        P = {k: P[k] - 0.05 * gr[k] for k in P}
    for c in range(G):
        mc = copy.deepcopy(m)
        for s in (0, 4):
            mc.zero_grad()
            F.cross_entropy(mc(x[c, s:s + 4]), y[c, s:s + 4]).backward()
            with torch.no_grad():
                for p in mc.parameters():
                    p -= 0.05 * p.grad
        for k, p in mc.named_parameters():
            torch.testing.assert_close(P[k][c], p.detach(), rtol=1e-10, atol=1e-12)
        # each client's own running statistics
        torch.testing.assert_close(B["bn1.running_mean"][c], mc.bn1.running_mean,
                                   rtol=1e-10, atol=1e-12)


def test_batched_path_runs_with_batchnorm_and_updates_running_stats():
    torch.manual_seed(0)
    model = ResNet(BasicBlock, [1, 1, 1, 1], num_classes=10, input_hw=16)
    rm0 = model.bn1.running_mean.clone()
    fed, opt = _engine("on", ["--fedavg_batch_size", "3"], model)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(24, 3, 16, 16, generator=g)
    y = torch.randint(0, 10, (24,), generator=g)
    fed.fedavg_lr = 0.01
    out = fed((torch.arange(4).repeat_interleave(6), x, y))
    assert torch.isfinite(out[0]).all() and out[0].shape == (4,)
    assert not torch.equal(model.bn1.running_mean, rm0)
    assert fed._payload[:fed.d].abs().max() > 0


def _gpu_round(base, dtype, batched, steps, extra=()):
    dist.init("cuda")
    args = parse_args(argv=["--dataset_name", "CIFAR10", "--mode", "fedavg", "--error_type", "none",
                            "--local_momentum", "0", "--virtual_momentum", "0.5", "--num_workers",
                            "8", "--num_clients", "8", "--local_batch_size", "-1", "--device", "cuda",
                            "--dtype", dtype, "--fedavg_batched", batched]
                      + (["--fedavg_batch_size", "4", "--num_fedavg_epochs", "2"] if steps == 4
                         else ["--fedavg_batch_size", "8"]) + list(extra), probe_port=False)
    model = copy.deepcopy(base).cuda()
    if dtype == "bf16":
        model = model.to(memory_format=torch.channels_last)
    fed = FedModel(model, cv_loss, args, num_clients=8)
    fed.fedavg_lr = 0.05
    g = torch.Generator().manual_seed(3)
    x = torch.randn(64, 3, 32, 32, generator=g).cuda()
    if dtype == "bf16":
        x = x.to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (64,), generator=g).cuda()
    out = fed((torch.arange(8).repeat_interleave(8), x, y))
    torch.cuda.synchronize()
    return fed._payload[:fed.d].clone(), out[0].clone()


@pytest.mark.gpu
def test_batched_local_sgd_gpu_fp32():
    """fp32 on the GPU: 4 local steps, MIOpen grouped convolutions under vmap
    vs the sequential path (MIOpen picks different algorithms for the two:
    measured 2.4e-4 relative)."""
    torch.manual_seed(0)
    base = models.ResNet9(channels={"prep": 64, "layer1": 128, "layer2": 128, "layer3": 256})
    up_a, l_a = _gpu_round(base, "fp32", "on", 4)
    up_b, l_b = _gpu_round(base, "fp32", "off", 4)
    assert ((up_a - up_b).norm() / up_b.norm()).item() < 1e-3
    torch.testing.assert_close(l_a, l_b, rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
def test_batched_local_sgd_gpu_fp32_clip_weight_decay():
    """The vmap path's client tail on the row kernel (fa_row_sgd: per-client
    clip + weight decay + SGD) vs the sequential path's stock tail"""
    torch.manual_seed(0)
    base = models.ResNet9(channels={"prep": 64, "layer1": 128, "layer2": 128, "layer3": 256})
    extra = ["--max_grad_norm", "0.5", "--weight_decay", "5e-2", "--fedavg_lr_decay", "0.8"]
    up_a, l_a = _gpu_round(base, "fp32", "on", 4, extra)
    up_b, l_b = _gpu_round(base, "fp32", "off", 4, extra)
    assert ((up_a - up_b).norm() / up_b.norm()).item() < 1e-3
    torch.testing.assert_close(l_a, l_b, rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
def test_batched_local_sgd_gpu_bf16():
    """bf16 (autocast inside the vmap): one local step.  Two bf16 paths of
    different kernels differ by bf16 rounding amplified through the net, so
    the bound is relative to how far the sequential bf16 step is from the
    fp32 one: the batched step must be as close to it as bf16 is to fp32."""
    torch.manual_seed(0)
    base = models.ResNet9(channels={"prep": 64, "layer1": 128, "layer2": 128, "layer3": 256})
    up_a, l_a = _gpu_round(base, "bf16", "on", 1)
    up_b, l_b = _gpu_round(base, "bf16", "off", 1)
    up_f, _ = _gpu_round(base, "fp32", "off", 1)
    bf_noise = ((up_b - up_f).norm() / up_f.norm()).item()
    rel = ((up_a - up_b).norm() / up_b.norm()).item()
    assert rel < 2 * bf_noise + 1e-2, (rel, bf_noise)
    assert ((up_a - up_f).norm() / up_f.norm()).item() < 2 * bf_noise + 1e-2
    torch.testing.assert_close(l_a, l_b, rtol=2e-2, atol=2e-2)


def test_batched_running_stats_do_not_depend_on_pass_size():
    """BatchNorm running statistics after a batched FedAvg round are the mean
    over ALL clients, each client starting from the round's buffers: splitting
    the clients over several vmap passes (a small --grouped_gb) gives the same
    buffers and upload as one pass."""
    torch.manual_seed(0)
    base = ResNet(BasicBlock, [1, 1, 1, 1], num_classes=10, input_hw=16)
    res = {}
    for gb in ("4", "1e-9"):  # one pass of 4 clients / two passes of 2
        model = copy.deepcopy(base)
        fed, opt = _engine("on", ["--fedavg_batch_size", "3", "--grouped_gb", gb], model)
        g = torch.Generator().manual_seed(3)
        x = torch.randn(24, 3, 16, 16, generator=g)
        y = torch.randint(0, 10, (24,), generator=g)
        # lr 0: the clients' weights stay put, so their statistics differ only
        # by conv rounding across vmap widths (a random-init BN net amplifies
        # any weight difference ~1e4-fold, test_vmapped_batchnorm_steps_exact_in_fp64)
        fed.fedavg_lr = 0.0
        fed((torch.arange(4).repeat_interleave(6), x, y))
        res[gb] = {k: b.clone() for k, b in model.named_buffers()}
    for k, b in res["4"].items():
        # rounding: ~1e-6; the old pass-order dependence (pass 2 started from
        # pass 1's mean and overwrote it) moved them by ~1e-2
        torch.testing.assert_close(res["1e-9"][k], b, rtol=1e-5, atol=1e-5)


def test_bn_stock_cumulative_average_when_momentum_none():
    """momentum=None: PyTorch's cumulative moving average (factor
    1/num_batches_tracked), also in the vmap-friendly stock composition."""
    from commefficient_amd.models.common import GhostBatchNorm2d
    from commefficient_amd.ops.nn import stock_ops
    torch.manual_seed(0)
    ref = torch.nn.BatchNorm2d(5, momentum=None)
    ours = GhostBatchNorm2d(5, momentum=None)
    for _ in range(3):
        x = torch.randn(6, 5, 4, 4)
        ref(x)
        with stock_ops():
            ours(x)
    torch.testing.assert_close(ours.running_mean, ref.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ours.running_var, ref.running_var, rtol=1e-5, atol=1e-6)
