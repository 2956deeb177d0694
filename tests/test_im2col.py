"""Column-image convolutions and the overlapping max-pool (csrc/im2col.hip,
ops/nn.py ``_ConvCol`` / ``_Conv1x1`` / ``_MaxPool``) vs fp32 PyTorch
references of the same ops on the same bf16 values: forward, input gradient,
weight gradient (returned, accumulated into an existing ``.grad``, and per
group under ``grouped_grads``).  The ImageNet ResNet shapes -- 7x7/s2 stem on
the augmentation kernel's 4-channel-stride input, strided 3x3, strided 1x1,
3x3/s2/p1 max-pool -- at small batch, plus odd sizes."""
import pytest
import torch
import torch.nn.functional as F

from commefficient_amd.ops import nn as cnn
from commefficient_amd.ops.grouped import GroupedGrads, grouped_grads

pytestmark = pytest.mark.gpu


def _close(a, b, rel=2e-2):
    a, b = a.float(), b.float()
    scale = b.abs().max().clamp_min(1e-6)
    err = (a - b).abs().max() / scale
    assert err < rel, f"max rel err {err.item():.3e}"


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


CASES = [  # N, C, H, W, K, R, stride, pad, data_input
    (2, 3, 32, 32, 64, 7, 2, 3, True),     # ImageNet stem, 4-channel pixel stride
    (2, 3, 29, 31, 64, 7, 2, 3, True),     # odd sizes
    (2, 3, 16, 16, 64, 3, 1, 1, True),     # CIFAR ResNet stem
    (2, 128, 14, 14, 128, 3, 2, 1, False),  # layer2 strided 3x3
    (3, 64, 15, 13, 64, 3, 2, 1, False),   # odd sizes, K = 64
    (2, 256, 7, 7, 256, 3, 2, 1, False),   # layer3/4-like
    (2, 16, 9, 11, 24, 5, 1, 2, False),    # 5x5, C % 64 != 0
]


def _case_inputs(N, C, H, W, K, R, data_input, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    if data_input:  # [N, H, W, 4] storage, 3 channels used: strides (4HW, 1, 4W, 4)
        store = torch.randn(N, H, W, 4, device="cuda", generator=g).to(torch.bfloat16)
        x = store.permute(0, 3, 1, 2)[:, :C]
        assert x.stride() == (4 * H * W, 1, 4 * W, 4)
    else:
        x = _nhwc(torch.randn(N, C, H, W, device="cuda", generator=g).to(torch.bfloat16))
    w = torch.randn(K, C, R, R, device="cuda", generator=g) * (2.0 / (R * R * C)) ** 0.5
    return x, w


@pytest.mark.parametrize("N,C,H,W,K,R,stride,pad,data_input", CASES)
def test_col_conv_matches_fp32(N, C, H, W, K, R, stride, pad, data_input):
    x, w = _case_inputs(N, C, H, W, K, R, data_input)
    x = x if data_input else x.requires_grad_()
    w = w.requires_grad_()
    assert cnn.conv2d_native_kind(x, w, stride, pad, 1, 1) == "col"
    y = cnn.conv2d_native(x, w, "col", stride, None, pad)
    xr = x.detach().float().requires_grad_(not data_input)
    wr = w.detach().to(torch.bfloat16).float().requires_grad_()
    ref = F.conv2d(xr, wr, stride=stride, padding=pad)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    _close(y, ref)
    gy = torch.randn_like(ref)
    y.backward(gy.to(torch.bfloat16))
    ref.backward(gy.to(torch.bfloat16).float())
    _close(w.grad, wr.grad)
    if not data_input:
        assert x.grad.is_contiguous(memory_format=torch.channels_last)
        _close(x.grad, xr.grad)


@pytest.mark.parametrize("N,C,H,W,K,bnstats", [(2, 128, 14, 14, 128, False), (3, 64, 15, 13, 64, False),
                                                (2, 64, 32, 32, 128, True), (2, 128, 24, 23, 64, True)])
def test_implicit_col_conv_matches_materialised(N, C, H, W, K, bnstats):
    """The strided 3x3 on the implicit column image (conv_nt_imp forward,
    gemm_tn_parts_imp weight gradient) == the im2col path bitwise: output,
    epilogue BN moments, both gradients."""
    x0, w0 = _case_inputs(N, C, H, W, K, 3, False, seed=3)
    gy = None
    outs = []
    for imp in (True, False):
        cnn._IMP_COL[0] = imp
        saved = dict(cnn._EPI)
        try:
            cnn._EPI.update(on=bnstats, G=N if bnstats else 0)
            x = x0.detach().clone().requires_grad_()
            w = w0.detach().clone().requires_grad_()
            y = cnn.conv2d_native(x, w, "col", 2, None, 1)
            st = getattr(y, "_commeff_bnstats", None)
            if gy is None:
                gy = torch.randn(y.shape, device="cuda").to(torch.bfloat16)
            y.backward(gy)
            outs.append((y.detach(), None if st is None else st[0], x.grad, w.grad))
        finally:
            cnn._IMP_COL[0] = True
            cnn._EPI.clear()
            cnn._EPI.update(saved)
    (yi, si, xi, wi), (ym, sm, xm, wm) = outs
    assert torch.equal(yi, ym) and torch.equal(xi, xm) and torch.equal(wi, wm)
    assert (si is None) == (sm is None) == (not bnstats)
    if bnstats:
        assert torch.equal(si, sm)


@pytest.mark.parametrize("grouped", [False, True])
def test_narrow_3x3_wgrad_implicit_matches_materialised(grouped):
    """The K = 64 stride-1 3x3 (ImageNet layer 1) weight gradient on the TN
    GEMM over the implicit column image == the im2col path bitwise (returned
    and per group)."""
    G, n, C, H, K = 2, 2, 64, 20, 64
    g = torch.Generator(device="cuda").manual_seed(5)
    x0 = _nhwc(torch.randn(G * n, C, H, H, device="cuda", generator=g).to(torch.bfloat16))
    w0 = torch.randn(K, C, 3, 3, device="cuda", generator=g) * 0.05
    assert cnn.conv2d_native_kind(x0, w0, 1, 1, 1, 1) == "3x3"
    gy = torch.randn(G * n, K, H, H, device="cuda", generator=g).to(torch.bfloat16)
    gy = _nhwc(gy)
    outs = []
    for imp in (True, False):
        cnn._IMP_COL[0] = imp
        try:
            w = w0.detach().clone().requires_grad_()
            if grouped:
                buf = torch.zeros(G, w.numel() + 8, device="cuda")
                gg = GroupedGrads(G, buf, {id(w): (8, w.shape)})
                with grouped_grads(gg):
                    y = cnn.conv2d_native(x0, w, "3x3", 1, gg, 1)
                y.backward(gy)
                outs.append(buf.clone())
            else:
                y = cnn.conv2d_native(x0, w, "3x3", 1, None, 1)
                y.backward(gy)
                outs.append(w.grad.clone())
        finally:
            cnn._IMP_COL[0] = True
    assert torch.equal(outs[0], outs[1])


def test_col_conv_wgrad_accumulates_into_existing_grad():
    x, w = _case_inputs(2, 128, 14, 14, 128, 3, False)
    w.grad = torch.full_like(w, 0.5)
    w.requires_grad_()
    y = cnn.conv2d_native(x, w, "col", 2, None, 1)
    gy = torch.randn(y.shape, device="cuda").to(torch.bfloat16)
    y.backward(gy)
    wr = w.detach().to(torch.bfloat16).float().requires_grad_()
    F.conv2d(x.float(), wr, stride=2, padding=1).backward(gy.float())
    _close(w.grad - 0.5, wr.grad)


@pytest.mark.parametrize("kind,R,stride,pad", [("col", 3, 2, 1), ("3x3", 3, 1, 1), ("1x1", 1, 2, 0)])
def test_per_group_weight_grads(kind, R, stride, pad):
    """Per-group weight gradients == each group's slice of the batch alone
    (the 3x3 case: K = 64, the column-image wgrad of _Conv3x3)."""
    G, n, C, H, K = 4, 2, 64, 12, 64
    g = torch.Generator(device="cuda").manual_seed(1)
    x = _nhwc(torch.randn(G * n, C, H, H, device="cuda", generator=g).to(torch.bfloat16))
    w = (torch.randn(K, C, R, R, device="cuda", generator=g) * 0.05).requires_grad_()
    assert cnn.conv2d_native_kind(x, w, stride, pad, 1, 1) == kind
    d = w.numel() + 8
    buf = torch.zeros(G, d, device="cuda")
    gg = GroupedGrads(G, buf, {id(w): (8, w.shape)})
    with grouped_grads(gg):
        y = cnn.conv2d_native(x, w, kind, stride, gg, pad)
    gy = torch.randn(y.shape, device="cuda", generator=g).to(torch.bfloat16)
    y.backward(gy)
    assert w.grad is None
    wr = w.detach().to(torch.bfloat16).float()
    for j in range(G):
        wj = wr.clone().requires_grad_()
        F.conv2d(x[j * n:(j + 1) * n].float(), wj, stride=stride, padding=pad).backward(
            gy[j * n:(j + 1) * n].float())
        _close(gg.view(w)[j], wj.grad)
    assert torch.equal(buf[:, :8], torch.zeros(G, 8, device="cuda"))


@pytest.mark.parametrize("N,C,H,W,K", [(2, 64, 14, 14, 128), (2, 64, 7, 9, 64)])
def test_strided_1x1_native_subsample(N, C, H, W, K):
    g = torch.Generator(device="cuda").manual_seed(2)
    x = _nhwc(torch.randn(N, C, H, W, device="cuda", generator=g).to(torch.bfloat16)).requires_grad_()
    w = (torch.randn(K, C, 1, 1, device="cuda", generator=g) * 0.1).requires_grad_()
    y = cnn.conv2d_native(x, w, "1x1", 2)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().to(torch.bfloat16).float().requires_grad_()
    ref = F.conv2d(xr, wr, stride=2)
    _close(y, ref)
    gy = torch.randn_like(ref).to(torch.bfloat16)
    y.backward(gy)
    ref.backward(gy.float())
    _close(x.grad, xr.grad)
    _close(w.grad, wr.grad)
    # off the stride grid the input gradient is exactly zero
    assert torch.equal(x.grad[:, :, 1::2, :].float().abs().sum(), torch.tensor(0.0, device="cuda"))


@pytest.mark.parametrize("H,W,data_input", [(11, 10, True), (150, 141, True), (37, 140, False)])
def test_im2col_layout(H, W, data_input):
    """col[p][(r*S + s)*C + c] = x[n][c][oh*s - p + r][ow*s - p + s] (zero outside
    and in the padding columns) -- against F.unfold (4-channel and 3-channel
    pixel strides, wide rows)."""
    x, _ = _case_inputs(2, 3, H, W, 8, 7, data_input)
    col = cnn._ops().im2col(x, 7, 7, 2, 3, 152)
    u = F.unfold(x.float(), 7, padding=3, stride=2)  # [N, C*49, L] (c, r, s) order
    N, L = x.shape[0], u.shape[2]
    ref = u.view(N, 3, 49, L).permute(0, 3, 2, 1).reshape(N * L, 147)
    assert torch.equal(col[:, :147].float(), ref)
    assert torch.equal(col[:, 147:], torch.zeros_like(col[:, 147:]))


def _distinct_planes(N, C, H, W, seed=3):
    """bf16 NHWC values distinct inside every (n, c) plane (no max ties)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    v = torch.argsort(torch.rand(N * C, H * W, device="cuda", generator=g), dim=1).float()
    v = v - H * W // 2  # integers of magnitude <= 128: exact in bf16 (H * W <= 256)
    return _nhwc(v.view(N, C, H, W).to(torch.bfloat16))


@pytest.mark.parametrize("N,C,H,W,k,s,p", [(2, 64, 16, 16, 3, 2, 1),
                                            (2, 64, 15, 17, 3, 2, 1),
                                            (3, 16, 8, 8, 2, 2, 0),
                                            (2, 8, 9, 9, 3, 1, 1)])
def test_maxpool_matches_reference(N, C, H, W, k, s, p):
    assert H * W <= 256
    x = _distinct_planes(N, C, H, W).requires_grad_()
    assert cnn.maxpool_native_ok(x, k, s, p)
    y = cnn.max_pool2d(x, k, s, p)
    xr = x.detach().float().requires_grad_()
    ref = F.max_pool2d(xr, k, s, p)
    assert y.shape == ref.shape and torch.equal(y.float(), ref)
    gy = torch.randn(ref.shape, device="cuda").to(torch.bfloat16)
    y.backward(gy)
    ref.backward(gy.float())
    # each input sums <= 4 bf16 gradients: fp32 sum then one rounding
    assert torch.allclose(x.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)


def test_maxpool_nan_propagates():
    x = _distinct_planes(1, 8, 6, 6)
    x[0, 3, 2, 2] = float("nan")
    y = cnn.max_pool2d(x, 3, 2, 1)
    ref = F.max_pool2d(x.float(), 3, 2, 1)
    assert torch.equal(torch.isnan(y), torch.isnan(ref))


def test_resnet101_round_has_no_library_convs():
    """The ImageNet ResNet-101 forward/backward dispatches every conv and the
    max-pool to native paths (no MIOpen conv, no at::native max-pool)."""
    from commefficient_amd.models.resnets import ResNet
    from commefficient_amd.models.resnets import Bottleneck
    torch.manual_seed(0)
    m = ResNet(Bottleneck, (1, 1, 1, 1), num_classes=10, input_hw=64).cuda()
    m = m.to(memory_format=torch.channels_last)
    store = torch.randn(2, 64, 64, 4, device="cuda").to(torch.bfloat16)
    x = store.permute(0, 3, 1, 2)[:, :3]
    with torch.autocast("cuda", dtype=torch.bfloat16), torch.profiler.profile(
            activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        loss = m(x).float().sum()
        loss.backward()
    names = {e.name for e in prof.events()}
    assert not any("convolution" in n and "aten::" in n for n in names), sorted(
        n for n in names if "conv" in n)
    assert not any("max_pool" in n for n in names), sorted(n for n in names if "pool" in n)


@pytest.mark.gpu
@pytest.mark.parametrize("k,s,p,H", [(3, 2, 1, 15), (3, 2, 1, 16), (2, 2, 0, 14), (3, 1, 1, 9)])
def test_maxpool_fwd_bwd_match_torch(k, s, p, H):
    """Native max-pool (k = 3 window loads all in flight; the runtime-k loop
    otherwise) vs F.max_pool2d: values, and the gradient routed to the first
    maximum of each window (PyTorch's rule)"""
    ops = torch.ops.commeff
    torch.manual_seed(0)
    x = torch.randn(3, 64, H, H + 1, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y, codes = ops.maxpool_fwd(x, k, s, p)
    xr = x.float().requires_grad_(True)
    yr = torch.nn.functional.max_pool2d(xr, k, s, p)
    torch.testing.assert_close(y.float(), yr.detach(), rtol=0, atol=0)
    gy = torch.randn_like(yr).bfloat16()
    yr.backward(gy.float())
    gx = ops.maxpool_bwd(gy.contiguous(memory_format=torch.channels_last), codes, H, H + 1, k, s, p)
    torch.testing.assert_close(gx.float(), xr.grad, rtol=1e-2, atol=1e-2)
