"""Ghost-BN statistics written by the producing GEMM's epilogue
(csrc/gemm.hip GemmArgs::stats -> csrc/bn.hip bn_fwd_finalize_tiles_kernel,
ops/nn.py _mm_nt_conv / take_bnstats): per-128-row-tile moments vs an fp32
reference of the stored output, the norm with tile moments vs its own
statistics pass, and a ResNet forward/backward with the fusion on vs off."""
import pytest
import torch

from commefficient_amd import _ext


def _ops():
    return _ext.ops()


def _tile_moments(y: torch.Tensor, Mg: int):
    """Reference [T, 4, N]: per 128-row tile and group slot, mean and M2."""
    M, N = y.shape
    T = (M + 127) // 128
    out = torch.zeros(T, 4, N, dtype=torch.float64)
    yf = y.double().cpu()
    for t in range(T):
        r0, r1 = t * 128, min(M, t * 128 + 128)
        rb = min(r1, (r0 // Mg + 1) * Mg)
        for slot, (a, b) in enumerate(((r0, rb), (rb, r1))):
            if b > a:
                blk = yf[a:b]
                m = blk.mean(0)
                out[t, 2 * slot] = m
                out[t, 2 * slot + 1] = ((blk - m) ** 2).sum(0)
    return out


def test_mm_nt_bnstats_cpu_semantics():
    g = torch.Generator().manual_seed(0)
    a = torch.randn(3 * 200, 64, generator=g).to(torch.bfloat16)
    b = torch.randn(64, 64, generator=g).to(torch.bfloat16)
    y, st = _ops().mm_nt_bnstats(a, b, 3)
    torch.testing.assert_close(y, _ops().mm_nt(a, b))
    ref = _tile_moments(y, 200)
    torch.testing.assert_close(st.double(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("G,Mg,N,K", [(8, 1568, 256, 512), (2, 6272, 64, 256), (1, 1000, 128, 64),
                                      (4, 200, 512, 128)])
def test_mm_nt_bnstats_moments_gpu(G, Mg, N, K):
    """Output bitwise the plain GEMM's; tile moments (split at group
    boundaries that fall inside tiles: 1568 % 128 = 32) vs fp64 of the output."""
    g = torch.Generator().manual_seed(G * Mg + N)
    a = (torch.randn(G * Mg, K, generator=g) + 0.5).to(torch.bfloat16).cuda()
    b = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).cuda()
    y, st = _ops().mm_nt_bnstats(a, b, G)
    assert torch.equal(y, _ops().mm_nt(a, b))
    ref = _tile_moments(y, Mg)
    got = st.double().cpu()
    torch.testing.assert_close(got[:, 0::2], ref[:, 0::2], rtol=1e-4, atol=1e-4)  # means
    torch.testing.assert_close(got[:, 1::2], ref[:, 1::2], rtol=1e-4, atol=1e-3)  # M2


@pytest.mark.gpu
@pytest.mark.parametrize("G,Mg,C", [(8, 1568, 256), (2, 6272, 64), (4, 200, 512)])
@pytest.mark.parametrize("relu", [False, True])
def test_ghost_bn_tile_moments_match_own_pass_gpu(G, Mg, C, relu):
    """ghost_bn_fwd with the GEMM's tile moments == with its own statistics
    pass: batch mean / rstd to fp32 rounding, outputs to one bf16 rounding,
    running statistics alike."""
    g = torch.Generator().manual_seed(Mg + C)
    K = 128
    a = (torch.randn(G * Mg, K, generator=g) + 1.0).to(torch.bfloat16).cuda()
    b = (torch.randn(C, K, generator=g) * K ** -0.5).to(torch.bfloat16).cuda()
    y2d, st = _ops().mm_nt_bnstats(a, b, G)
    # [N, C, H, W] channels_last view of the rows (H*W = Mg / n per group)
    n, hw = Mg // 8 if Mg % 8 == 0 else Mg, 8 if Mg % 8 == 0 else 1
    x = y2d.view(G * n, hw, 1, C).permute(0, 3, 1, 2)
    assert x.is_contiguous(memory_format=torch.channels_last)
    w = torch.rand(C, device="cuda") + 0.5
    bias = torch.randn(C, device="cuda")
    outs = []
    for ts in (None, st):
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        nbt = torch.zeros((), dtype=torch.long, device="cuda")
        yb, stat, bits = _ops().ghost_bn_fwd(x, w, bias, G, 1e-5, 0.1, rm, rv, relu, nbt, None, ts)
        outs.append((yb.float(), stat, rm, rv, nbt))
    (y0, s0, m0, v0, n0), (y1, s1, m1, v1, n1) = outs
    torch.testing.assert_close(s1, s0, rtol=2e-4, atol=2e-4)
    torch.testing.assert_close(m1, m0, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(v1, v0, rtol=1e-4, atol=1e-5)
    assert int(n0.item()) == int(n1.item()) == 1
    diff = (y1 - y0).abs()
    assert diff.max().item() <= 0.02 * y0.abs().max().item()
    assert (diff > 0).float().mean().item() < 0.02  # rare one-ulp rounding flips


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1, 2])
def test_bottleneck_fwd_bwd_with_bn_epilogue_statistics_gpu(stride):
    """A merged 2-client ResNet bottleneck step (1x1 / 3x3 / 1x1 + strided
    downsample) with its norms' statistics from the conv GEMMs' epilogues vs
    their own passes: output, input gradient and weight gradients agree to
    bf16 rounding, and the fusion engaged.  (A whole random-init ResNet-50 is
    the wrong probe: its forward amplifies one-ulp differences of the first
    norm, 4e-5, to ~1e-2 by layer 2 -- measured in round 4, profiles/r4_experiments.md.)"""
    from commefficient_amd.models.common import conv1x1, ghost_batchnorm, GhostBatchNorm2d
    from commefficient_amd.models.resnets import Bottleneck
    from commefficient_amd.ops import nn as onn

    torch.manual_seed(0)
    cin = 256 if stride == 1 else 128
    ds = None if stride == 1 else torch.nn.Sequential(conv1x1(cin, 256, stride), GhostBatchNorm2d(256))
    blk = Bottleneck(cin, 64, 16, stride, ds).cuda().train()
    x0 = torch.randn(64, cin, 16, 16, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    state = {k: v.clone() for k, v in blk.state_dict().items()}
    orig_take, orig_on = onn.take_bnstats, onn._EPI["on"]
    results = []
    for on in (False, True):
        blk.load_state_dict(state)
        blk.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        used = []

        def spy(t, G):
            r = orig_take(t, G)
            used.append(r is not None)
            return r

        onn._EPI["on"] = on
        onn.take_bnstats = spy
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16), ghost_batchnorm(blk, 2):
                y = blk(x)
            (y.float() * torch.linspace(-1, 1, y.shape[1], device="cuda").view(1, -1, 1, 1)).sum().backward()
        finally:
            onn.take_bnstats = orig_take
            onn._EPI["on"] = orig_on
        grads = torch.cat([p.grad.float().flatten() for p in blk.parameters()])
        results.append((y.float(), x.grad.float(), grads, sum(used)))
    (y0, dx0, g0, u0), (y1, dx1, g1, u1) = results
    assert u0 == 0 and u1 == (2 if stride == 1 else 4), (u0, u1)  # 1x1s (+ strided 3x3, downsample)

    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()

    assert rel(y1, y0) < 5e-3
    assert rel(dx1, dx0) < 1e-2
    assert rel(g1, g0) < 1e-2
