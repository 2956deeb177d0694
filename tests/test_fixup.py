"""Fixup scalar affine maps (ops/fixup.py) and the Fixup models' merged-batch
path: the native bf16 pass vs an fp32 PyTorch reference of the same op, and
whole-model bf16 runs vs fp32 runs (reference models/fixup_resnet9.py,
fixup_resnet18.py, fixup_resnet.py)."""
import itertools

import pytest
import torch
import torch.nn.functional as F

from commefficient_amd.ops.fixup import scalar_affine


def _ref(x, s, b, add, relu):
    y = x.float()
    if s is not None:
        y = y * s
    if b is not None:
        y = y + b
    if add is not None:
        y = y + add.float()
    return F.relu(y) if relu else y


def test_scalar_affine_cpu_composition():
    torch.manual_seed(0)
    x = torch.randn(2, 8, 3, 3)
    s, b = torch.tensor([1.5]), torch.tensor([-0.25])
    add = torch.randn_like(x)
    torch.testing.assert_close(scalar_affine(x, s, b, add, True), _ref(x, s, b, add, True))
    torch.testing.assert_close(scalar_affine(x, b=b), x + b)


@pytest.mark.parametrize("name", ["FixupResNet9", "FixupResNet18", "FixupResNet50"])
def test_fixup_models_cpu_forward_backward(name):
    from commefficient_amd import models
    torch.manual_seed(0)
    m = _perturbed(getattr(models, name)(num_classes=10))
    x = torch.randn(2, 3, 32, 32)
    loss = F.cross_entropy(m(x), torch.tensor([1, 7]))
    loss.backward()
    assert torch.isfinite(loss)
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())


@pytest.mark.gpu
@pytest.mark.parametrize("has_s,has_b,has_add,relu", list(itertools.product([0, 1], repeat=4)))
def test_scalar_affine_native_matches_fp32(has_s, has_b, has_add, relu):
    from commefficient_amd.ops import fixup as fx
    g = torch.Generator(device="cuda").manual_seed(3)
    shape = (6, 64, 9, 11)
    x = torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    s = (torch.rand(1, device="cuda", generator=g) + 0.5).requires_grad_(True) if has_s else None
    b = (torch.randn(1, device="cuda", generator=g) * 0.3).requires_grad_(True) if has_b else None
    add = None
    if has_add:
        add = torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16)
        add = add.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    assert fx.native_ok(x, s, b, add)
    y = scalar_affine(x, s, b, add, bool(relu))
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    w = torch.randn(shape, device="cuda", generator=g)  # dy, fp32 -> the contiguous bf16 layout path
    (y.float() * w).sum().backward()
    leaves = [t for t in (x, s, b, add) if t is not None]
    refs = [t.detach().float().clone().requires_grad_(True) for t in leaves]
    it = iter(refs)
    xr = next(it)
    sr = next(it) if has_s else None
    br = next(it) if has_b else None
    ar = next(it) if has_add else None
    yr = _ref(xr, sr, br, ar, bool(relu))
    (yr * w.to(torch.bfloat16).float()).sum().backward()
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2)
    for t, r in zip(leaves, refs):
        a, e = t.grad.float(), r.grad
        err = ((a - e).norm() / e.norm().clamp_min(1e-6)).item()
        assert err < 1e-2, (err, tuple(t.shape))


@pytest.mark.gpu
@pytest.mark.parametrize("has_b", [0, 1])
def test_scalar_affine_post_bias_matches_fp32(has_b):
    """relu(x + b) + post: one pass each way, the relu mask recomputed from x"""
    g = torch.Generator(device="cuda").manual_seed(4)
    shape = (5, 128, 7, 9)
    x = torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    b = (torch.randn(1, device="cuda", generator=g) * 0.3).requires_grad_(True) if has_b else None
    p = (torch.randn(1, device="cuda", generator=g) * 0.3).requires_grad_(True)
    y = scalar_affine(x, b=b, relu=True, post=p)
    w = torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16)
    (y.float() * w.float()).sum().backward()
    xr = x.detach().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if has_b else None
    pr = p.detach().clone().requires_grad_(True)
    yr = F.relu(xr + br if has_b else xr) + pr
    (yr * w.float()).sum().backward()
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2)
    for a, e in [(x.grad, xr.grad), (p.grad, pr.grad)] + ([(b.grad, br.grad)] if has_b else []):
        err = ((a.float() - e).norm() / e.norm().clamp_min(1e-6)).item()
        assert err < 1e-2, err


@pytest.mark.gpu
def test_fork_bias_sums_both_gradients():
    """(x + b, x) with dx = dxa + didentity and db = sum dxa in one pass"""
    from commefficient_amd.ops.fixup import fork_bias
    g = torch.Generator(device="cuda").manual_seed(6)
    shape = (4, 128, 6, 10)
    x = torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    b = (torch.randn(1, device="cuda", generator=g) * 0.3).requires_grad_(True)
    w1 = torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16)
    w2 = torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16)
    xa, idt = fork_bias(x, b)
    assert xa.dtype == torch.bfloat16
    ((xa.float() * w1.float()).sum() + (idt.float() * w2.float()).sum()).backward()
    torch.testing.assert_close(xa.float(), x.detach().float() + b.detach(), rtol=1e-2, atol=1e-2)
    ref_dx = w1.float() + w2.float()
    err = ((x.grad.float() - ref_dx).norm() / ref_dx.norm()).item()
    assert err < 1e-2, err
    torch.testing.assert_close(b.grad, w1.float().sum().view(1), rtol=1e-3, atol=1e-1)


@pytest.mark.gpu
def test_scalar_affine_sums_deterministic_large():
    """many chunks (the two-level fold) and bit-identical reruns"""
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(40, 256, 28, 28, device="cuda", generator=g).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    s = torch.ones(1, device="cuda").requires_grad_(True)
    b = torch.zeros(1, device="cuda").requires_grad_(True)
    dy = torch.randn(x.shape, device="cuda", generator=g).to(torch.bfloat16)
    dy = dy.contiguous(memory_format=torch.channels_last)
    grads = []
    for _ in range(2):
        s.grad = b.grad = None
        scalar_affine(x, s, b, relu=True).backward(dy)
        grads.append((s.grad.clone(), b.grad.clone()))
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])
    m = (x.float() > 0).float()
    torch.testing.assert_close(b.grad, (dy.float() * m).sum().view(1), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s.grad, (dy.float() * m * x.float()).sum().view(1), rtol=1e-4, atol=1e-2)


def _perturbed(model):
    """Fixup zero-inits the last conv of each branch and the classifier (all
    gradients but a few vanish): give every parameter a small random value."""
    g = torch.Generator().manual_seed(7)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if p.dim() > 1:
                fan = p[0].numel()
                p.copy_(torch.randn(p.shape, generator=g) * (1.0 / fan) ** 0.5)
            else:
                p.add_(torch.randn(p.shape, generator=g) * 0.1)
    return model


@pytest.mark.gpu
@pytest.mark.parametrize("name,hw,ncls", [("FixupResNet9", 32, 10), ("FixupResNet18", 32, 10),
                                          ("FixupResNet50", 64, 100)])
def test_fixup_model_native_bf16_close_to_fp32(name, hw, ncls):
    """The merged-batch path of a Fixup model: activations stay bf16 (the
    scalars on the native affine kernels, the convs on the native kernels),
    loss and gradients close to an fp32 run of the same weights."""
    from commefficient_amd import models
    torch.manual_seed(0)
    m = _perturbed(getattr(models, name)(num_classes=ncls)).cuda()
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(8, 3, hw, hw, device="cuda", generator=g)
    t = torch.randint(0, ncls, (8,), device="cuda", generator=g)
    from commefficient_amd.ops.nn import stock_ops
    out = {}
    for mode in ("fp32", "stock", "bf16"):
        m.zero_grad(set_to_none=True)
        if mode == "fp32":
            loss = F.cross_entropy(m(x), t)
        elif mode == "stock":  # autocast bf16 on the PyTorch composition (fp32-promoted scalars)
            with stock_ops(), torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x.to(torch.bfloat16)).float(), t)
        else:
            seen = []
            hooks = [mod.register_forward_hook(lambda _m, i, _o: seen.append(i[0].dtype))
                     for mod in m.modules() if isinstance(mod, torch.nn.Conv2d)]
            with torch.autocast("cuda", dtype=torch.bfloat16):
                xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
                loss = F.cross_entropy(m(xb).float(), t)
            for h in hooks:
                h.remove()
            assert seen and all(d == torch.bfloat16 for d in seen), seen
        loss.backward()
        out[mode] = (loss.item(), [p.grad.float().clone() for p in m.parameters()])
    (lr, gr), (ls, gs), (lb, gb) = out["fp32"], out["stock"], out["bf16"]

    def err(g):
        num = sum(((a - b) ** 2).sum() for a, b in zip(g, gr)) ** 0.5
        return (num / sum((b ** 2).sum() for b in gr) ** 0.5).item()

    print(name, "loss", lr, ls, lb, "grad err stock", err(gs), "native", err(gb))
    assert abs(lb - lr) < 2e-2 * max(1.0, abs(lr)), (lb, lr)
    # bf16 activations throughout: as close as the bf16 composition, within bf16 noise
    assert err(gb) < 1.5 * err(gs) + 2e-2, (err(gb), err(gs))
