"""Native batched FedAvg (parallel/fedavg_native.py): every kernel of the
explicit G-client ResNet-18 program against a plain PyTorch fp32 reference of
the same op, and the whole local-SGD round against the vmap composition and
the fp32 sequential path (fed_worker.py:61-113 semantics)."""
import copy

import pytest
import torch
import torch.nn.functional as F

from commefficient_amd import _ext
from commefficient_amd.models.fixup import ResNet18
from commefficient_amd.parallel.fedavg_native import ResNet18FedAvg, _gview
from commefficient_amd.utils.args import parse_args


def _ops():
    return _ext.ops()


def _args(extra=()):
    return parse_args(argv=["--dataset_name", "CIFAR100", "--mode", "fedavg", "--batchnorm",
                            "--local_batch_size", "-1", "--local_momentum", "0", "--error_type", "none"]
                      + list(extra), probe_port=False)


def test_supported_models():
    ok, _ = ResNet18FedAvg.supported(ResNet18(num_classes=100), _args())
    assert ok
    from commefficient_amd import models
    from commefficient_amd.parallel.fedavg_native import ResNet9FedAvg, engine_for
    assert not ResNet18FedAvg.supported(models.ResNet9(), _args())[0]
    assert ResNet9FedAvg.supported(models.ResNet9(), _args())[0]
    assert not ResNet9FedAvg.supported(models.ResNet9(do_batchnorm=True), _args())[0]
    assert engine_for(models.ResNet9(), _args())[0] is ResNet9FedAvg
    assert engine_for(ResNet18(num_classes=100), _args())[0] is ResNet18FedAvg
    from commefficient_amd.models.fixup import FixupResNet9
    from commefficient_amd.parallel.fedavg_native import FixupResNet9FedAvg
    assert engine_for(FixupResNet9(num_classes=10), _args())[0] is FixupResNet9FedAvg
    assert not FixupResNet9FedAvg.supported(models.ResNet9(), _args())[0]
    from commefficient_amd.models.fixup import FixupResNet18
    from commefficient_amd.parallel.fedavg_native import FixupResNet18FedAvg
    assert engine_for(FixupResNet18(num_classes=10), _args())[0] is FixupResNet18FedAvg
    assert not ResNet18FedAvg.supported(ResNet18(num_classes=10), _args(["--dtype", "fp32"]))[0]


def test_engine_layout_matches_parameter_order():
    """Offsets of every parameter the program reads come from the flat layout
    (FedModel's named_parameters order)."""
    m = ResNet18(num_classes=100)
    names = [nm for nm, p in m.named_parameters()]

    class _Flat:
        offsets, numels = [], []
    o = 0
    for p in m.parameters():
        _Flat.offsets.append(o)
        _Flat.numels.append(p.numel())
        o += p.numel()
    eng = ResNet18FedAvg(m, _Flat, names)
    # rows: every parameter on a 16-byte boundary, padding between (perm -1)
    assert o <= eng.d < o + 8 * len(names)
    assert all(v % 8 == 0 for v in eng.off.values())
    perm = eng._perm("cpu")
    real = perm[perm >= 0]
    assert real.numel() == o and torch.equal(real.sort().values, torch.arange(o, dtype=real.dtype))
    assert [b.stride for b in eng.blocks] == [1, 1, 2, 1, 2, 1, 2, 1]
    assert sum(b.sc is not None for b in eng.blocks) == 3
    assert eng.feat == 512 and eng.ncls == 100


def test_engine_accepts_only_covered_geometry():
    """auto mode must fall back to vmap (not fail mid-round) for inputs the
    engine's kernels do not cover: the fused pooling head takes final maps of
    <= 256 pixels, and the stem its own input channel count."""
    m = ResNet18(num_classes=100)
    names = [nm for nm, p in m.named_parameters()]

    class _Flat:
        offsets, numels = [], []
    o = 0
    for p in m.parameters():
        _Flat.offsets.append(o)
        _Flat.numels.append(p.numel())
        o += p.numel()
    eng = ResNet18FedAvg(m, _Flat, names)
    assert eng.accepts((5, 3, 32, 32))[0]
    assert eng.accepts((5, 3, 128, 128))[0]  # 16 x 16 final map
    ok, why = eng.accepts((5, 3, 224, 224))
    assert not ok and "256" in why
    assert not eng.accepts((5, 1, 28, 28))[0]  # a 3-channel stem


# ----------------------------------------------------------------- kernels
def _cs(t, G):
    """[G, n, C, H, W] fp32 -> channel-stacked bf16 [n, G*C, H, W] channels_last"""
    Gq, n, C, H, W = t.shape
    return (t.permute(1, 0, 2, 3, 4).reshape(n, G * C, H, W).to(torch.bfloat16)
            .contiguous(memory_format=torch.channels_last))


@pytest.mark.gpu
@pytest.mark.parametrize("R", [3, 1])
def test_weight_images(R):
    torch.manual_seed(0)
    G, K, C, off, ld = 3, 64, 16, 40, 64 * 16 * R * R + 104
    W = torch.randn(G, ld, device="cuda")
    w = W[:, off:off + K * C * R * R].view(G, K, C, R, R)
    Kc = (R * R * C + 7) // 8 * 8
    ops = _ops()
    if R == 3:
        i0 = ops.fa_weight_image(W, ld, G, off, K, C, R, Kc, 0)
        torch.testing.assert_close(i0.float(), w.permute(0, 1, 3, 4, 2).reshape(G * K, R, R, C).bfloat16().float())
        i1 = ops.fa_weight_image(W, ld, G, off, K, C, R, Kc, 1)
        ref = w.flip(3, 4).permute(0, 2, 3, 4, 1).reshape(G * C, R, R, K)
        torch.testing.assert_close(i1.float(), ref.bfloat16().float())
    i2 = ops.fa_weight_image(W, ld, G, off, K, C, R, Kc, 2)
    ref = torch.zeros(G, K, Kc, device="cuda")
    ref[:, :, :R * R * C] = w.permute(0, 1, 3, 4, 2).reshape(G, K, R * R * C)
    torch.testing.assert_close(i2.float(), ref.bfloat16().float())
    # ld 0: one broadcast row
    b = ops.fa_weight_image(W[0].contiguous(), 0, G, off, K, C, R, Kc, 2)
    torch.testing.assert_close(b.float(), ref[:1].expand(G, -1, -1).bfloat16().float())


@pytest.mark.gpu
@pytest.mark.parametrize("stride,C", [(1, 64), (2, 64), (2, 16)])
def test_im2col_col2im_grouped_match_per_client(stride, C):
    torch.manual_seed(0)
    G, n, H = 3, 2, 8
    X = torch.randn(G, n, C, H, H, device="cuda")
    x = _cs(X, G)
    ops = _ops()
    col = ops.im2col_grouped(x, G, 3, 3, stride, 1, 9 * C, False)
    gcol = torch.randn_like(col, dtype=torch.float32).bfloat16()
    gx = ops.col2im_grouped(gcol, G, n, H, H, C, 3, 3, stride, 1)
    for g in range(G):
        xg = X[g].bfloat16().contiguous(memory_format=torch.channels_last)
        torch.testing.assert_close(col[:, g], ops.im2col(xg, 3, 3, stride, 1, 9 * C), rtol=0, atol=0)
        ref = ops.col2im(gcol[:, g].contiguous(), n, H, H, C, 3, 3, stride, 1)
        torch.testing.assert_close(gx[:, g * C:(g + 1) * C].float(), ref.float(), rtol=0, atol=0)
    # client-major input (the data loader's [G*n, C, H, W] batch)
    xc = X.reshape(G * n, C, H, H).bfloat16().contiguous(memory_format=torch.channels_last)
    colc = ops.im2col_grouped(xc, G, 3, 3, stride, 1, 9 * C, True)
    torch.testing.assert_close(colc, col, rtol=0, atol=0)


@pytest.mark.gpu
def test_im2col_grouped_three_channel_stem():
    torch.manual_seed(0)
    G, n = 4, 3
    X = torch.randn(G * n, 3, 32, 32, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    col = _ops().im2col_grouped(X, G, 3, 3, 1, 1, 32, True)
    for g in range(G):
        ref = _ops().im2col(X[g * n:(g + 1) * n], 3, 3, 1, 1, 32)
        torch.testing.assert_close(col[:, g], ref, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("G,C,H,n", [(4, 64, 8, 5), (100, 64, 4, 5), (3, 256, 4, 5), (100, 64, 32, 5),
                                     (6, 512, 4, 2), (6, 512, 4, 1)])
def test_cs_bn_forward_backward(G, C, H, n):
    torch.manual_seed(0)
    X = torch.randn(G, n, C, H, H, device="cuda") * 2 + 0.5
    x = _cs(X, G)
    ld, woff, boff = 2 * C + 32, 8, C + 16
    P = torch.randn(G, ld, device="cuda")
    rm = torch.randn(G * C, device="cuda")
    rv = torch.rand(G * C, device="cuda") + 0.5
    rm0, rv0 = rm.clone(), rv.clone()
    nbt = torch.zeros((), dtype=torch.long, device="cuda")
    ops = _ops()
    y, stat, bits = ops.cs_bn_fwd(x, P, ld, woff, boff, G, 1e-5, 0.1, rm, rv, nbt)
    xf = x.float().view(n, G, C, H, H).transpose(0, 1)  # [G, n, C, H, W]
    w = P[:, woff:woff + C].view(G, 1, C, 1, 1)
    b = P[:, boff:boff + C].view(G, 1, C, 1, 1)
    xr = xf.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    mean = xr.mean(dim=(1, 3, 4), keepdim=True)
    var = xr.var(dim=(1, 3, 4), unbiased=False, keepdim=True)
    yr = F.relu((xr - mean) * torch.rsqrt(var + 1e-5) * wr + br)
    torch.testing.assert_close(y.float().view(n, G, C, H, H).transpose(0, 1), yr.detach(), rtol=2e-2, atol=2e-2)
    M = n * H * H
    torch.testing.assert_close(rm.view(G, C), 0.9 * rm0.view(G, C) + 0.1 * mean.view(G, C), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rv.view(G, C), 0.9 * rv0.view(G, C) + 0.1 * var.view(G, C) * M / (M - 1),
                               rtol=1e-3, atol=1e-3)
    assert int(nbt) == 1
    # the residual add after the ReLU (PreActBlock tail): same bits, y + r
    r = torch.randn_like(y, dtype=torch.float32).bfloat16().contiguous(memory_format=torch.channels_last)
    y2, _, bits2 = ops.cs_bn_fwd(x, P, ld, woff, boff, G, 1e-5, 0.1, rm.clone(), rv.clone(), None, r)
    assert torch.equal(bits2, bits)
    torch.testing.assert_close(y2.float(), (y.float() + r.float()).bfloat16().float(), rtol=0, atol=0)
    DY = torch.randn(G, n, C, H, H, device="cuda")
    dy = _cs(DY, G)
    yr.backward(dy.float().view(n, G, C, H, H).transpose(0, 1))
    Gg = torch.zeros(G, ld, device="cuda")
    dx = ops.cs_bn_bwd(dy, x, stat, bits, P, ld, woff, G, Gg, ld, woff, boff)
    scale = xr.grad.abs().max()
    torch.testing.assert_close(dx.float().view(n, G, C, H, H).transpose(0, 1) / scale, xr.grad / scale,
                               rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(Gg[:, woff:woff + C], wr.grad.view(G, C), rtol=2e-2, atol=2e-2 * M ** 0.5)
    torch.testing.assert_close(Gg[:, boff:boff + C], br.grad.view(G, C), rtol=2e-2, atol=2e-2 * M ** 0.5)


@pytest.mark.gpu
def test_head_pool_forward_backward():
    torch.manual_seed(0)
    G, n, C = 5, 3, 256
    X = torch.randn(G, n, C, 4, 4, device="cuda")
    x = _cs(X, G)
    feat, codes = _ops().fa_head_fwd(x, G)
    xf = x.float().view(n, G, C, 4, 4).transpose(0, 1).requires_grad_(True)
    # (adaptive max-pool routes a tied maximum's gradient to one position, as the kernel does)
    mx = F.adaptive_max_pool2d(xf.reshape(G * n, C, 4, 4), 1).view(G, n, C)
    ref = torch.cat([xf.mean(dim=(3, 4)), mx], dim=2)  # [G, n, 2C]
    torch.testing.assert_close(feat, ref.detach(), rtol=1e-5, atol=1e-5)
    df = torch.randn_like(feat)
    ref.backward(df)
    dx = _ops().fa_head_bwd(df, codes, 4, 4)
    torch.testing.assert_close(dx.float().view(n, G, C, 4, 4).transpose(0, 1), xf.grad, rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("clip,G", [(0.0, 5), (0.5, 5), (0.5, 13)])
def test_row_sgd_and_upload(clip, G):
    torch.manual_seed(0)
    d = 1003
    ld = 1024
    W = torch.randn(G, ld, device="cuda")
    Gr = torch.zeros(G, ld, device="cuda")
    Gr[:, :d] = torch.randn(G, d, device="cuda")
    w0 = torch.randn(d, device="cuda")
    w0p = torch.zeros(ld, device="cuda")
    w0p[:d] = w0
    ops = _ops()
    # first step: the broadcast server row
    out = torch.zeros(G, ld, device="cuda")
    ops.fa_row_sgd(out, ld, w0p, 0, Gr, ld, G, d, clip, 0.1, 0.01)
    g = Gr[:, :d]
    nrm = g.norm(dim=1, keepdim=True)
    sc = torch.where(nrm > clip, clip / nrm, torch.ones_like(nrm)) if clip > 0 else torch.ones_like(nrm)
    ref = w0 - 0.1 * (sc * g + 0.01 * w0)
    torch.testing.assert_close(out[:, :d], ref, rtol=1e-5, atol=1e-6)
    # in place
    W2 = W.clone()
    ops.fa_row_sgd(W2, ld, W2, ld, Gr, ld, G, d, clip, 0.1, 0.01)
    torch.testing.assert_close(W2[:, :d], W[:, :d] - 0.1 * (sc * g + 0.01 * W[:, :d]), rtol=1e-5, atol=1e-6)
    up = torch.ones(d, device="cuda")
    ops.fa_upload(up, w0, W, ld, G, 5.0)
    torch.testing.assert_close(up, 1 + 5 * (w0 - W[:, :d]).sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_conv3x3_wgrad_rows_matches_grouped_conv():
    torch.manual_seed(0)
    G, n, C, K, H = 3, 5, 128, 128, 16
    x = _cs(torch.randn(G, n, C, H, H, device="cuda"), G)
    dy = _cs(torch.randn(G, n, K, H, H, device="cuda"), G)
    ld, off = K * C * 9 + 64, 32
    dst = torch.zeros(G, ld, device="cuda")
    assert _ops().conv3x3_wgrad_rows(dy, x, G, dst, ld, off)
    ref = torch.nn.grad.conv2d_weight(x.float(), (G * K, C, 3, 3), dy.float(), padding=1, groups=G)
    got = dst[:, off:off + K * C * 9].reshape(G * K, C, 3, 3)
    scale = ref.abs().max()
    torch.testing.assert_close(got / scale, ref / scale, rtol=1e-2, atol=1e-2)
    assert dst[:, :off].abs().max() == 0 and dst[:, off + K * C * 9:].abs().max() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("H,K,C", [(16, 128, 128), (8, 256, 128), (32, 64, 64)])
def test_conv_rows_forward_and_dgrad_image(H, K, C):
    """Grouped halo conv reading every client's bf16 (k, r, s, c) weight rows in
    place (row stride ld, or one shared row), and the flipped / transposed
    dgrad image built from those rows."""
    torch.manual_seed(0)
    G, n, off = 3, 2, 64
    ld = off + K * 9 * C + 64
    x = _cs(torch.randn(G, n, C, H, H, device="cuda"), G)
    w = torch.randn(G, K, C, 3, 3, device="cuda") / (3 * C ** 0.5)  # PyTorch layout
    Wb = torch.zeros(G, ld, device="cuda", dtype=torch.bfloat16)
    Wb[:, off:off + K * 9 * C] = w.permute(0, 1, 3, 4, 2).reshape(G, -1).bfloat16()
    ops = _ops()
    y = ops.conv3x3_fwd_rows(x, Wb, G, off, ld, K)
    ref = F.conv2d(x.float(), w.reshape(G * K, C, 3, 3).bfloat16().float(), padding=1, groups=G)
    scale = ref.abs().max()
    torch.testing.assert_close(y.float() / scale, ref / scale, rtol=2e-2, atol=2e-2)
    # one shared row (the first local step)
    y0 = ops.conv3x3_fwd_rows(x, Wb[0].contiguous(), G, off, 0, K)
    ref0 = F.conv2d(x.float(), w[:1].expand(G, -1, -1, -1, -1).reshape(G * K, C, 3, 3).bfloat16().float(),
                    padding=1, groups=G)
    torch.testing.assert_close(y0.float() / scale, ref0 / scale, rtol=2e-2, atol=2e-2)
    # the residual addend epilogue: y + r (the shortcut gradient of the backward)
    r = torch.randn_like(y, dtype=torch.float32).bfloat16().contiguous(memory_format=torch.channels_last)
    ya = ops.conv3x3_fwd_rows(x, Wb, G, off, ld, K, r)
    torch.testing.assert_close(ya.float(), (y.float() + r.float()).bfloat16().float(), rtol=1e-2, atol=2e-2)
    img = ops.fa_dgrad_image(Wb, ld, G, off, K, C)
    refi = w.flip(3, 4).permute(0, 2, 3, 4, 1).reshape(G * C, 3, 3, K).bfloat16()
    torch.testing.assert_close(img, refi, rtol=0, atol=0)
    assert ops.fa_dgrad_image(Wb[1].contiguous(), 0, G, off, K, C).shape == (C, 3, 3, K)
    # the input gradient: through the image, and (C % 128 == 0) straight from
    # the rows with the transposed B tiles -- vs the fp32 grouped dgrad
    dy = _cs(torch.randn(G, n, K, H, H, device="cuda"), G)
    gref = torch.nn.grad.conv2d_input(x.shape, w.reshape(G * K, C, 3, 3).bfloat16().float(), dy.float(),
                                      padding=1, groups=G)
    gs = gref.abs().max()
    dx_img = ops.conv3x3_fwd_rows(dy, img, G, 0, C * 9 * K, C)
    torch.testing.assert_close(dx_img.float() / gs, gref / gs, rtol=2e-2, atol=2e-2)
    dx_bt = ops.conv3x3_fwd_rows(dy, Wb, G, off, ld, C, None, True)
    if C % 64 == 0:
        torch.testing.assert_close(dx_bt.float() / gs, gref / gs, rtol=2e-2, atol=2e-2)
        assert torch.equal(dx_bt, dx_img)  # same products in the same order
        # the first local step's shared row
        dx0 = ops.conv3x3_fwd_rows(dy, Wb[0].contiguous(), G, off, 0, C, None, True)
        g0 = torch.nn.grad.conv2d_input(x.shape, w[:1].expand(G, -1, -1, -1, -1).reshape(G * K, C, 3, 3)
                                        .bfloat16().float(), dy.float(), padding=1, groups=G)
        torch.testing.assert_close(dx0.float() / gs, g0 / gs, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("G,C,K,H", [(2, 128, 128, 16), (4, 64, 64, 32), (2, 256, 256, 8), (3, 256, 256, 4)])
def test_conv3x3_wgrad_rows_rsc_order(G, C, K, H):
    """(64-channel clients: computed in pairs as 128-channel groups, the
    diagonal blocks kept; 8x8 / 4x4 images: the wide wgrad kernel with
    channel-stacked groups)"""
    torch.manual_seed(0)
    n = 5
    x = _cs(torch.randn(G, n, C, H, H, device="cuda"), G)
    dy = _cs(torch.randn(G, n, K, H, H, device="cuda"), G)
    ld, off = K * C * 9 + 64, 32
    dst = torch.zeros(G, ld, device="cuda")
    assert _ops().conv3x3_wgrad_rows(dy, x, G, dst, ld, off, True)
    ref = torch.nn.grad.conv2d_weight(x.float(), (G * K, C, 3, 3), dy.float(), padding=1, groups=G)
    got = dst[:, off:off + K * C * 9].reshape(G * K, 3, 3, C).permute(0, 3, 1, 2)
    scale = ref.abs().max()
    torch.testing.assert_close(got / scale, ref / scale, rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("K,N,Nfull,o,P,small", [(256, 2304, 2304, 0, 80, -1), (64, 64, 576, 256, 320, -1),
                                                 (512, 2304, 2304, 0, 17, 1), (128, 1152, 1152, 0, 200, 0),
                                                 (72, 136, 136, 0, 50, 1), (64, 27, 32, 0, 300, 1),
                                                 # split-K (few tiles over long K) + the reduction's SGD step
                                                 (64, 27, 32, 0, 5120, 1), (128, 1152, 1152, 0, 2048, 0)])
def test_fa_bmm_rows_sgd_and_mirror(K, N, Nfull, o, P, small):
    """TN GEMM over channel-stacked operands into client rows: rows = beta rows
    + alpha A_g B_g with the bf16 mirror from the epilogue (fp32 reference)"""
    torch.manual_seed(0)
    G, ld, off = 5, K * N + 96, 32
    At = torch.randn(P, G, K, device="cuda").bfloat16()
    col = torch.randn(P, G, Nfull, device="cuda").bfloat16()
    A = At.permute(1, 2, 0)
    B = col.transpose(0, 1)[:, :, o:o + N]
    W = torch.randn(G, ld, device="cuda")
    W0 = W.clone()
    Wb = torch.zeros(G, ld, device="cuda", dtype=torch.bfloat16)
    assert _ops().fa_bmm_rows(A, B, W, ld, off, 0.99, -0.1, Wb, small)
    ref = 0.99 * W0[:, off:off + K * N].view(G, K, N) - 0.1 * torch.bmm(A.float(), B.float())
    got = W[:, off:off + K * N].view(G, K, N)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(Wb[:, off:off + K * N].view(G, K, N), got.bfloat16(), rtol=0, atol=0)
    # the rest of the rows untouched
    assert torch.equal(W[:, :off], W0[:, :off]) and torch.equal(W[:, off + K * N:], W0[:, off + K * N:])
    assert not Wb[:, :off].any() and not Wb[:, off + K * N:].any()
    # the first local step: beta scales the shared server row (sld 0), not dst
    w0 = torch.randn(ld, device="cuda")
    W3 = torch.full((G, ld), float("nan"), device="cuda")
    assert _ops().fa_bmm_rows(A, B, W3, ld, off, 0.99, -0.1, Wb, small, w0, 0)
    ref3 = 0.99 * w0[off:off + K * N].view(1, K, N) - 0.1 * torch.bmm(A.float(), B.float())
    torch.testing.assert_close(W3[:, off:off + K * N].view(G, K, N), ref3, rtol=1e-4, atol=1e-3)
    # plain accumulation (beta 1, alpha 1), no mirror
    W2 = W0.clone()
    assert _ops().fa_bmm_rows(A, B, W2, ld, off, 1.0, 1.0, None, small)
    torch.testing.assert_close(W2[:, off:off + K * N].view(G, K, N),
                               W0[:, off:off + K * N].view(G, K, N) + torch.bmm(A.float(), B.float()),
                               rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("nn,M,N,K,shared", [(False, 320, 256, 1152, False), (False, 80, 128, 64, True),
                                             (True, 1280, 576, 128, False), (True, 80, 2304, 256, True)])
def test_fa_gemm_grouped(nn, M, N, K, shared):
    """Grouped native GEMM over channel-stacked operands (strided views) vs
    fp32 bmm, with beta accumulation and a shared (broadcast) weight row"""
    torch.manual_seed(0)
    G = 5
    At = torch.randn(M, G, K, device="cuda").bfloat16()
    A = At.transpose(0, 1)  # [G, M, K], strides (K, G K, 1)
    shape = (G, K, N) if nn else (G, N, K)
    B = torch.randn(1 if shared else G, *shape[1:], device="cuda").bfloat16()
    B = B.expand(G, -1, -1) if shared else B
    out_t = torch.randn(M, G, N, device="cuda").bfloat16()
    out = out_t.transpose(0, 1)
    old = out.float().clone()
    assert _ops().fa_gemm(A, B, out, nn, 1.0)
    ref = old + torch.bmm(A.float(), B.float() if nn else B.float().transpose(1, 2))
    scale = ref.abs().max()
    torch.testing.assert_close(out.float() / scale, ref / scale, rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("C,K,H,n", [(256, 256, 8, 5), (256, 256, 4, 5), (128, 256, 4, 2)])
def test_fa_bmm_rows_implicit_column_image(C, K, H, n):
    """The TN GEMM reading the 3x3 column image implicitly from the
    channel-stacked x == the same update from the materialised im2col_grouped"""
    torch.manual_seed(0)
    G = 3
    x = _cs(torch.randn(G, n, C, H, H, device="cuda"), G)
    dy = _cs(torch.randn(G, n, K, H, H, device="cuda"), G)
    ld, off = K * 9 * C + 64, 32
    W0 = torch.randn(G, ld, device="cuda")
    Wa, Wb_ = W0.clone(), W0.clone()
    Ma = torch.zeros(G, ld, device="cuda", dtype=torch.bfloat16)
    Mb = torch.zeros_like(Ma)
    ops = _ops()
    A = _gview(dy, G).transpose(1, 2)
    col = ops.im2col_grouped(x, G, 3, 3, 1, 1, 9 * C, False)
    assert ops.fa_bmm_rows(A, col.transpose(0, 1), Wa, ld, off, 0.99, -0.1, Ma, 1)
    shape = torch.empty((1, 1, 1), device="cuda", dtype=torch.bfloat16).expand(G, n * H * H, 9 * C)
    assert ops.fa_bmm_rows(A, shape, Wb_, ld, off, 0.99, -0.1, Mb, 1, None, 0, x)
    torch.testing.assert_close(Wb_, Wa, rtol=1e-5, atol=1e-5)
    assert torch.equal(Mb, Ma) or (Mb.float() - Ma.float()).abs().max() < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("C,K,H,n", [(64, 128, 32, 2), (128, 256, 16, 3), (256, 256, 8, 5)])
def test_implicit_strided_column_image(C, K, H, n):
    """Stride-2 3x3 conv and its 1x1 stride-2 shortcut: forward on the native
    GEMM over the implicit column image, and the TN weight update over it, ==
    the same products over the materialised im2col_grouped image"""
    torch.manual_seed(0)
    G = 3
    ops = _ops()
    x = _cs(torch.randn(G, n, C, H, H, device="cuda"), G)
    Ho = (H - 1) // 2 + 1
    P = n * Ho * Ho
    col = ops.im2col_grouped(x, G, 3, 3, 2, 1, 9 * C, False)
    cg = col.transpose(0, 1)
    w1 = torch.randn(G, K, 9 * C, device="cuda").bfloat16()
    wsc = torch.randn(G, K, C, device="cuda").bfloat16()
    carrier = torch.empty((1, 1, 1), device="cuda", dtype=torch.bfloat16)
    for R, pad, N, w, ref_a in ((3, 1, 9 * C, w1, cg), (1, 0, C, wsc, cg[:, :, 4 * C:5 * C])):
        out = torch.empty(P, G, K, device="cuda", dtype=torch.bfloat16)
        ref = torch.empty_like(out)
        assert ops.fa_gemm(ref_a, w, ref.transpose(0, 1), False, 0.0)
        assert ops.fa_gemm(carrier.expand(G, P, N), w, out.transpose(0, 1), False, 0.0, x, R, 2, pad)
        assert torch.equal(out, ref)
        # the weight update over the same implicit image
        dy = torch.randn(P, G, K, device="cuda").bfloat16()
        A = dy.permute(1, 2, 0)  # [G, K, P]
        ld, off = K * N + 64, 32
        Wr = torch.randn(G, ld, device="cuda")
        Wi = Wr.clone()
        assert ops.fa_bmm_rows(A, ref_a, Wr, ld, off, 0.99, -0.1, None, 1)
        assert ops.fa_bmm_rows(A, carrier.expand(G, P, N), Wi, ld, off, 0.99, -0.1, None, 1, None, 0, x, R, 2, pad)
        torch.testing.assert_close(Wi, Wr, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("layout,bias,shared,n,C", [("client", True, False, 5, 100), ("client", True, True, 7, 10),
                                                    ("stacked", False, False, 5, 10), ("stacked", False, True, 32, 100)])
def test_fa_linear_ce_matches_fp32(layout, bias, shared, n, C):
    """The per-client classifier step in one kernel (fedavg.hip fa_linear_ce):
    per-example loss / top-1, the feature gradient with the step's weights and
    the SGD-updated classifier rows (+ bias) vs an fp32 reference; features
    client-major fp32 ([G, n, F]) or channel-stacked bf16 ([n, G F]), weights
    per client or the shared server row (ld 0) updated into client rows."""
    torch.manual_seed(3)
    G, F = 6, 512
    scale = 1.0 if bias else 0.125
    per = C * F + C
    ld = per + 40
    boff = C * F + 3 if bias else -1
    woff = 3 if bias else 0
    Wsrc = torch.randn(ld if shared else G * ld, device="cuda") * 0.05
    wld = 0 if shared else ld
    if layout == "client":
        feat = torch.randn(G, n, F, device="cuda").relu()
        fsg, fsn = n * F, F
        ff = feat
    else:
        feat = torch.randn(n, G * F, device="cuda").relu().to(torch.bfloat16)
        fsg, fsn = F, G * F
        ff = feat.float().view(n, G, F).transpose(0, 1)
    y = torch.randint(0, C, (G * n,), device="cuda")
    dst = torch.full((G, ld), float("nan"), device="cuda")
    beta, alpha = 1.0 - 0.05 * 5e-4, -0.05
    # client-major fp32 features: 32-class chunks with partial feature-gradient slabs
    S = -(-C // 32) if layout == "client" else 1
    dfeat = torch.empty((S * feat.shape[0],) + tuple(feat.shape[1:]), device="cuda", dtype=feat.dtype)
    loss, correct = _ops().fa_linear_ce(feat, fsg, fsn, G, n, Wsrc, wld, woff, boff, C, F, scale, y, dfeat,
                                        fsg, fsn, dst, ld, beta, alpha, Wsrc, wld, None, 0,
                                        feat.numel() if S > 1 else 0, 32 if S > 1 else 0)
    dfeat = dfeat.view(S, *feat.shape).sum(0)
    rows = Wsrc.view(1, ld).expand(G, ld) if shared else Wsrc.view(G, ld)
    Wg = rows[:, woff:woff + C * F].view(G, C, F)
    bg = rows[:, boff:boff + C] if bias else torch.zeros(G, C, device="cuda")
    logits = scale * torch.bmm(ff, Wg.transpose(1, 2)) + bg[:, None, :]
    ref_loss = torch.nn.functional.cross_entropy(logits.reshape(G * n, C), y, reduction="none")
    torch.testing.assert_close(loss, ref_loss, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(correct, (logits.reshape(G * n, C).argmax(1) == y).float())
    gl = torch.softmax(logits, -1) - torch.nn.functional.one_hot(y.view(G, n), C).float()
    ref_df = torch.bmm(gl, Wg) * (scale / n)
    got_df = dfeat.float() if layout == "client" else dfeat.float().view(n, G, F).transpose(0, 1)
    tol = 1e-4 if layout == "client" else 1e-2
    torch.testing.assert_close(got_df, ref_df, rtol=tol, atol=tol * ref_df.abs().max().item())
    ref_w = beta * Wg + alpha * (scale / n) * torch.bmm(gl.transpose(1, 2), ff)
    torch.testing.assert_close(dst[:, woff:woff + C * F].view(G, C, F), ref_w, rtol=1e-5, atol=1e-6)
    if bias:
        ref_b = beta * bg + alpha / n * gl.sum(1)
        torch.testing.assert_close(dst[:, boff:boff + C], ref_b, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_ew_add_relu():
    a = torch.randn(2, 64, 4, 4, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    b = torch.randn_like(a)
    torch.testing.assert_close(_ops().fa_ew(a, b, 0).float(), (a.float() + b.float()).bfloat16().float())
    torch.testing.assert_close(_ops().fa_ew(a, None, 1).float(), a.float().clamp_min(0))


# ---------------------------------------------------------------- engine
def _round(base, engine, dtype, G, n, extra, lr=0.05):
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.train.losses import cv_loss
    dist.init("cuda")
    args = parse_args(argv=["--dataset_name", "CIFAR100", "--mode", "fedavg", "--error_type", "none",
                            "--local_momentum", "0", "--virtual_momentum", "0", "--num_workers", str(G),
                            "--num_clients", str(G), "--local_batch_size", "-1", "--device", "cuda",
                            "--dtype", dtype, "--batchnorm", "--fedavg_engine", engine] + extra,
                      probe_port=False)
    model = copy.deepcopy(base).cuda()
    if dtype == "bf16":
        model = model.to(memory_format=torch.channels_last)
    fed = FedModel(model, cv_loss, args, num_clients=G)
    fed.fedavg_lr = lr
    g = torch.Generator().manual_seed(3)
    x = torch.randn(G * n, 3, 32, 32, generator=g).cuda()
    if dtype == "bf16":
        x = x.bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 100, (G * n,), generator=g).cuda()
    out = fed((torch.arange(G).repeat_interleave(n), x, y))
    torch.cuda.synchronize()
    bufs = {k: b.detach().float().clone() for k, b in model.named_buffers()}
    return fed._payload[:fed.d].clone(), out[0].clone(), bufs, fed


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [
    ["--fedavg_batch_size", "-1", "--num_fedavg_epochs", "2"],
    ["--fedavg_batch_size", "-1", "--num_fedavg_epochs", "3", "--weight_decay", "5e-4",
     "--max_grad_norm", "2.0", "--fedavg_lr_decay", "0.9"],
    ["--fedavg_batch_size", "2", "--num_fedavg_epochs", "1"],
])
def test_native_round_matches_vmap_and_fp32(extra):
    """Upload and per-client losses of the native program vs the vmap
    composition (bf16) and the fp32 sequential path: the native round must be
    as close to fp32 as the bf16 vmap round is."""
    _check_native_round(extra, 6, 5)


@pytest.mark.gpu
def test_native_round_multi_pass_uneven(monkeypatch):
    """A --grouped_gb small enough for 3 clients per pass splits 7 clients
    into passes of 3, 3 and 1: the running-statistic sums accumulate across
    passes, num_batches_tracked advances once (first pass only), the stem's
    padded weight image is re-made for the smaller last pass -- and the round
    still matches the vmap and fp32 rounds."""
    from commefficient_amd.parallel import fedavg_native as fa
    d = sum(p.numel() for p in ResNet18(num_classes=100).parameters())
    gb = 3.5 * 12 * d / 2 ** 30  # per pass: int(gb 2^30) // (12 d) = 3 clients
    passes = []
    orig = fa.ResNet18FedAvg.run

    def run(self, *a, **kw):
        passes.append(a[3])  # G of the pass
        return orig(self, *a, **kw)

    monkeypatch.setattr(fa.ResNet18FedAvg, "run", run)
    _check_native_round(["--fedavg_batch_size", "-1", "--num_fedavg_epochs", "2", "--grouped_gb", str(gb)],
                        7, 5, passes)


def _check_native_round(extra, G, n, passes=None):
    torch.manual_seed(0)
    base = ResNet18(num_classes=100)
    up_n, l_n, b_n, fed = _round(base, "native", "bf16", G, n, extra)
    assert fed._fa_native, "native engine did not run"
    if passes is not None:
        assert passes == [3, 3, 1], passes
    up_v, l_v, b_v, _ = _round(base, "vmap", "bf16", G, n, extra)
    up_f, l_f, b_f, _ = _round(base, "vmap", "fp32", G, n, extra + ["--fedavg_batched", "off"])
    noise = ((up_v - up_f).norm() / up_f.norm()).item()
    rel = ((up_n - up_f).norm() / up_f.norm()).item()
    assert rel < 2 * noise + 2e-2, (rel, noise)
    lnoise = (l_v - l_f).abs().max().item()
    assert (l_n - l_f).abs().max().item() <= 2 * lnoise + 3e-2 * l_f.abs().max().item(), (l_n, l_v, l_f)
    # running statistics: the clients' mean (the batched semantics -- the
    # sequential path accumulates them client after client on one model), so
    # against the fp32 vmap round, within twice the bf16 vmap round's distance
    # (as norms: with 1-image batches (extra2: 16 values per channel at 4x4) a
    # single channel's variance follows the bf16 rounding of the steps before
    # it chaotically -- max-abs distances of 0.6 (vmap) to 1.3 between two
    # summation orders of the same BN kernel)
    _, _, b_vf, _ = _round(base, "vmap", "fp32", G, n, extra)
    for k in b_v:
        if "running" in k:
            ref = b_vf[k].norm().item()
            bn_noise = (b_v[k] - b_vf[k]).norm().item() / ref
            err = (b_n[k] - b_vf[k]).norm().item() / ref
            assert err <= 2 * bn_noise + 1e-2, (k, err, bn_noise)
        elif "num_batches" in k:
            assert b_n[k] == b_v[k], k


# ------------------------------------------------------------ ResNet-9 engine
def _round9(base, engine, dtype, G, n, extra, lr=0.05):
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.train.losses import cv_loss
    dist.init("cuda")
    args = parse_args(argv=["--dataset_name", "CIFAR10", "--mode", "fedavg", "--error_type", "none",
                            "--local_momentum", "0", "--virtual_momentum", "0", "--num_workers", str(G),
                            "--num_clients", str(G), "--local_batch_size", "-1", "--device", "cuda",
                            "--dtype", dtype, "--fedavg_engine", engine] + extra, probe_port=False)
    model = copy.deepcopy(base).cuda()
    if dtype == "bf16":
        model = model.to(memory_format=torch.channels_last)
    fed = FedModel(model, cv_loss, args, num_clients=G)
    fed.fedavg_lr = lr
    g = torch.Generator().manual_seed(4)
    x = torch.randn(G * n, 3, 32, 32, generator=g).cuda()
    if dtype == "bf16":
        x = x.bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (G * n,), generator=g).cuda()
    out = fed((torch.arange(G).repeat_interleave(n), x, y))
    torch.cuda.synchronize()
    return fed._payload[:fed.d].clone(), out[0].clone(), fed


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [
    ["--fedavg_batch_size", "-1", "--num_fedavg_epochs", "2"],
    ["--fedavg_batch_size", "2", "--num_fedavg_epochs", "1", "--weight_decay", "5e-4",
     "--max_grad_norm", "2.0", "--fedavg_lr_decay", "0.9"],
])
def test_resnet9_native_round_matches_vmap_and_fp32(extra):
    """The headline model's FedAvg round on the native G-client program
    (ResNet9FedAvg: grouped halo convs, ReLU + max-pool kernels on the stacked
    channels, batched classifier) vs the vmap composition (bf16) and the fp32
    sequential path (fed_worker.py:61-113): as close to fp32 as bf16 vmap is."""
    from commefficient_amd import models
    torch.manual_seed(0)
    base = models.ResNet9()
    G, n = 5, 4
    up_n, l_n, fed = _round9(base, "native", "bf16", G, n, extra)
    assert fed._fa_native and type(fed._fa_native).__name__ == "ResNet9FedAvg"
    up_v, l_v, _ = _round9(base, "vmap", "bf16", G, n, extra)
    up_f, l_f, _ = _round9(base, "vmap", "fp32", G, n, extra + ["--fedavg_batched", "off"])
    noise = ((up_v - up_f).norm() / up_f.norm()).item()
    rel = ((up_n - up_f).norm() / up_f.norm()).item()
    assert rel < 2 * noise + 2e-2, (rel, noise)
    lnoise = (l_v - l_f).abs().max().item()
    assert (l_n - l_f).abs().max().item() <= 2 * lnoise + 3e-2 * l_f.abs().max().item(), (l_n, l_v, l_f)


def _fixup9_perturbed(cls_name="FixupResNet9"):
    """A Fixup model whose zero-initialised parts (last convs, classifier,
    scalars) are perturbed, so every gradient path is exercised."""
    from commefficient_amd.models import fixup
    torch.manual_seed(0)
    m = getattr(fixup, cls_name)(num_classes=10)
    g = torch.Generator().manual_seed(11)
    with torch.no_grad():
        for name, p in m.named_parameters():
            if p.numel() == 1:
                base = 1.0 if name.endswith("scale") else 0.0
                p.fill_(base + 0.2 * torch.randn((), generator=g).item())
            elif p.dim() == 4:
                # (He init, damped in the deep model: 18 un-normalised layers
                # would otherwise blow the logits up to losses of ~200, where
                # bf16 rounding alone moves them by tens)
                gain = 0.5 if cls_name == "FixupResNet18" else 1.0
                p.copy_(torch.randn(p.shape, generator=g) * gain * (2.0 / (p.shape[1] * p.shape[2] * p.shape[3])) ** 0.5)
            else:
                p.copy_(torch.randn(p.shape, generator=g) * 0.05)
    return m


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["stacked", "client"])
def test_fa_affine_forward_backward_and_scalar_sgd(layout):
    """Per-client Fixup scalars (fedavg.hip fa_affine / fa_affine_bwd /
    fa_scalar_sgd) vs torch on the same bf16 values: y = relu(x s_g + b_g +
    add), dx = dpre s_g + add2, the per-client sums of dpre and dpre x (or of
    dy unmasked), and the scalars' SGD step from a shared source row."""
    torch.manual_seed(2)
    G, n, C, H = 6, 3, 64, 8
    ld, soff, boff = 40, 7, 13
    W = torch.randn(G, ld, device="cuda")
    if layout == "stacked":
        x = torch.randn(n, G * C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        grp = lambda t: t.float().permute(0, 2, 3, 1).reshape(-1, G, C).transpose(0, 1).reshape(G, -1)  # noqa: E731
        sv = lambda v: v.view(1, G, 1, 1, 1).expand(n, G, C, H, H).reshape(n, G * C, H, H)  # noqa: E731
        cm = False
    else:
        x = torch.randn(G * n, 4, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        grp = lambda t: t.float().reshape(G, -1)  # noqa: E731
        sv = lambda v: v.view(G, 1, 1, 1, 1).expand(G, n, 4, H, H).reshape(G * n, 4, H, H)  # noqa: E731
        cm = True
    add = torch.randn_like(x)
    s_, b_ = W[:, soff], W[:, boff]
    y = _ops().fa_affine(x, G, cm, W, ld, soff, boff, add, True)
    ref = torch.relu(x.float() * sv(s_) + sv(b_) + add.float())
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)
    dy, add2 = torch.randn_like(x), torch.randn_like(x)
    out1, out2, part = _ops().fa_affine_bwd(dy, G, cm, W, ld, soff, y, x, add2, True, True)
    dpre = dy.float() * (y.float() > 0)
    torch.testing.assert_close(out2.float(), dpre, rtol=0, atol=0)
    torch.testing.assert_close(out1.float(), dpre * sv(s_) + add2.float(), rtol=1e-2, atol=2e-2)
    sums = part.sum(0)
    torch.testing.assert_close(sums[:, 0], grp(dpre).sum(1), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(sums[:, 1], (grp(dpre) * grp(x)).sum(1), rtol=1e-4, atol=1e-3)
    # without the scale input the second sum is of dy unmasked
    _, _, part2 = _ops().fa_affine_bwd(dy, G, cm, W, ld, -1, y, None, None, False, False)
    torch.testing.assert_close(part2.sum(0)[:, 1], grp(dy).sum(1), rtol=1e-4, atol=1e-3)
    # the SGD step into client rows from the shared server row
    src = torch.randn(ld, device="cuda")
    dst = torch.full((G, ld), float("nan"), device="cuda")
    _ops().fa_scalar_sgd(part, dst, ld, boff, soff, 0.99, -0.1, src, 0)
    torch.testing.assert_close(dst[:, boff], 0.99 * src[boff] - 0.1 * sums[:, 0], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dst[:, soff], 0.99 * src[soff] - 0.1 * sums[:, 1], rtol=1e-5, atol=1e-5)
    assert torch.isnan(dst[:, 0]).all()  # the rest of the rows untouched


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [
    ["--fedavg_batch_size", "-1", "--num_fedavg_epochs", "2"],
    ["--fedavg_batch_size", "2", "--num_fedavg_epochs", "1", "--weight_decay", "5e-4",
     "--max_grad_norm", "2.0", "--fedavg_lr_decay", "0.9"],
])
@pytest.mark.parametrize("model", ["FixupResNet9", "FixupResNet18"])
def test_fixup_native_round_matches_vmap_and_fp32(extra, model):
    """A Fixup model's FedAvg round on the native G-client program
    (FixupResNet9FedAvg / FixupResNet18FedAvg: the ResNet-9 / ResNet-18
    kernels + per-client Fixup scalars) vs the vmap composition (bf16) and the
    fp32 sequential path: as close to fp32 as bf16 vmap is (reference
    models/fixup_resnet9.py, fixup_resnet18.py, fed_worker.py:61-113)."""
    base = _fixup9_perturbed(model)
    G, n = 5, 4
    up_n, l_n, fed = _round9(base, "native", "bf16", G, n, extra, lr=0.02)
    assert fed._fa_native and type(fed._fa_native).__name__ == model + "FedAvg"
    up_v, l_v, _ = _round9(base, "vmap", "bf16", G, n, extra, lr=0.02)
    up_f, l_f, _ = _round9(base, "vmap", "fp32", G, n, extra + ["--fedavg_batched", "off"], lr=0.02)
    noise = ((up_v - up_f).norm() / up_f.norm()).item()
    rel = ((up_n - up_f).norm() / up_f.norm()).item()
    assert rel < 2 * noise + 2e-2, (rel, noise)
    lnoise = (l_v - l_f).abs().max().item()
    assert (l_n - l_f).abs().max().item() <= 2 * lnoise + 3e-2 * l_f.abs().max().item(), (l_n, l_v, l_f)
    # the scalars moved like the fp32 path's (their own slice of the upload)
    names = [nm for nm, _ in base.named_parameters()]
    offs = dict(zip(names, fed.flat.offsets))
    idx = torch.tensor([offs[nm] for nm, p in base.named_parameters() if p.numel() == 1], device="cuda")
    torch.testing.assert_close(up_n[idx], up_f[idx], rtol=0.1, atol=0.1 * up_f[idx].abs().max().item())

