"""Native MFMA GEMMs (csrc/gemm.hip: mm_nt / mm_nn) vs an fp32 PyTorch
reference of the same op (bf16 operands upcast, fp32 math, one final
rounding), at the GPT-2 block and ResNet-101 1x1-conv shapes and with row
tails; plus the CPU reference path the CPU suite runs."""
import pytest
import torch
import torch.nn.functional as F

from commefficient_amd import _ext

SHAPES = [  # M, N, K
    (9600, 2304, 768),   # GPT-2 qkv
    (9600, 768, 768),    # attention projection
    (9600, 3072, 768),   # MLP up
    (9600, 768, 3072),   # MLP down
    (25088, 256, 1024),  # ResNet-101 bottleneck 1x1 (8 x 56 x 56 px)
    (9500, 768, 3072),   # 256-row tiles with a row tail (9500 % 256 = 28)
    (9500, 2304, 768),   # 256 x 256 tiles with a row tail
    (777, 128, 256),     # row tail
    (130, 64, 64),       # 64-wide tiles, tiny
]


def _ops():
    return _ext.ops()


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _mk(M, N, K, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    a = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    b = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=dev, generator=g)
    return a, b, bias


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(640, 50257, 768), (300, 100, 128), (129, 1000, 64), (64, 64 + 7, 192)])
def test_gemm_nt_n_edge_into_padded_rows(M, N, K):
    """NT GEMM with N no tile multiple (the tied LM head, V = 50,257): B rows
    past N read the zero page in-kernel, the output is a [M, N] view of rows
    padded to a multiple of 8 columns; columns past the padded chunk are never
    written."""
    a, b, _ = _mk(M, N, K, "cuda", seed=3)
    ld = -(-N // 8) * 8 + 16
    buf = torch.full((M, ld), 7.0, device="cuda").to(torch.bfloat16)
    out = buf[:, :N]
    _ops().mm_nt(a, b, None, out)
    assert _rel(out, a.float() @ b.float().t()) < 1e-2
    assert torch.all(buf[:, -(-N // 8) * 8:] == 7.0)  # beyond the straddling chunk: untouched


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("layout", ["nt", "nn"])
def test_gemm_matches_fp32(M, N, K, layout):
    a, b, bias = _mk(M, N, K, "cuda")
    ref = a.float() @ b.float().t()
    if layout == "nt":
        y = _ops().mm_nt(a, b)
    else:
        y = _ops().mm_nn(a, b.t().contiguous())
    assert y.dtype == torch.bfloat16 and y.shape == (M, N)
    assert _rel(y, ref) < 1e-2
    yb = _ops().mm_nt(a, b, bias) if layout == "nt" else _ops().mm_nn(a, b.t().contiguous(), bias)
    assert _rel(yb, ref + bias) < 1e-2
    b16 = bias.to(torch.bfloat16)  # bf16 bias (the GPT-2 Conv1D biases), added in the epilogue
    yh = _ops().mm_nt(a, b, b16) if layout == "nt" else _ops().mm_nn(a, b.t().contiguous(), b16)
    assert _rel(yh, ref + b16.float()) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(9600, 3072, 768), (777, 128, 256)])
def test_gemm_gelu_epilogue(M, N, K):
    a, b, bias = _mk(M, N, K, "cuda", seed=1)
    pre = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    y = _ops().mm_nn(a, b.t().contiguous(), bias, None, 0.0, 1, pre)
    ref = a.float() @ b.float().t() + bias
    assert _rel(pre, ref) < 1e-2
    # the activation is computed from the stored (bf16) pre-activation
    torch.testing.assert_close(y.float(), F.gelu(pre.float(), approximate="tanh"), rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_gemm_accumulates_into_out(out_dtype):
    M, N, K = 2000, 256, 512
    a, b, _ = _mk(M, N, K, "cuda", seed=2)
    c0 = torch.randn(M, N, device="cuda").to(out_dtype)
    out = c0.clone()
    _ops().mm_nt(a, b, None, out, 1.0)
    ref = a.float() @ b.float().t() + c0.float()
    assert _rel(out, ref) < 1e-2


def test_gemm_cpu_reference_semantics():
    a, b, bias = _mk(70, 128, 64, "cpu")
    y = _ops().mm_nt(a, b, bias)
    torch.testing.assert_close(y, (a.float() @ b.float().t() + bias).to(torch.bfloat16))
    pre = torch.empty(70, 128, dtype=torch.bfloat16)
    g = _ops().mm_nn(a, b.t().contiguous(), bias, None, 0.0, 1, pre)
    torch.testing.assert_close(pre, (a.float() @ b.float().t() + bias).to(torch.bfloat16))
    torch.testing.assert_close(g, F.gelu(pre.float(), approximate="tanh").to(torch.bfloat16))


@pytest.mark.gpu
@pytest.mark.parametrize("G,T,M,N", [(3, 640, 256, 512), (8, 1568, 512, 256), (1, 6272, 1024, 256),
                                     (2, 130, 256, 256), (4, 3136, 64, 256), (2, 700, 64, 64),
                                     (1, 900, 320, 128), (2, 5000, 64, 152), (3, 2000, 128, 72)])
def test_gemm_tn_grouped_vs_fp32(G, T, M, N):
    """csrc/gemm_tn.hip with G groups of T rows in one launch: sink[g] +=
    a_g^T b_g (the per-client 1x1-conv weight gradients), group rows strided
    like the per-group gradient rows of ops/grouped.py."""
    g = torch.Generator().manual_seed(G * T)
    a = torch.randn(G * T, M, generator=g).to(torch.bfloat16).cuda()
    b = torch.randn(G * T, N, generator=g).to(torch.bfloat16).cuda()
    big = torch.randn(G, M * N + 64, generator=g).cuda()  # padded group rows
    sink = big[:, :M * N].view(G, M, N)
    s0, pad = sink.clone(), big[:, M * N:].clone()
    _ops().gemm_tn_acc_grouped(sink, a, b, G)
    assert torch.equal(big[:, M * N:], pad)  # nothing written past a group's rows
    ref = s0 + torch.bmm(a.float().view(G, T, M).transpose(1, 2), b.float().view(G, T, N))
    torch.testing.assert_close(sink, ref, rtol=1e-4, atol=1e-3 * (T ** 0.5) / 10)
    # deterministic
    sink2 = s0.clone()
    _ops().gemm_tn_acc_grouped(sink2, a, b, G)
    assert torch.equal(sink, sink2)


@pytest.mark.gpu
@pytest.mark.parametrize("G", [1, 4])
def test_1x1_wgrad_native_route(G):
    """ops/nn.py _wgrad_gemm: 256-multiple 1x1 weight gradients run on the
    native TN GEMM (into a flat gradient view, or per-group rows) and match
    the fp32 product."""
    from commefficient_amd.ops import nn as onn
    P, K, C = 4 * 1568, 512, 256
    g = torch.Generator().manual_seed(7)
    g2d = torch.randn(P, K, generator=g).to(torch.bfloat16).cuda()
    x2d = torch.randn(P, C, generator=g).to(torch.bfloat16).cuda()
    assert onn._wgrad_tn_ok(g2d, x2d, None, G)
    ref = torch.bmm(g2d.float().view(G, P // G, K).transpose(1, 2), x2d.float().view(G, P // G, C))
    into = torch.randn(G, K, C, device="cuda")
    want = into + ref
    onn._wgrad_gemm(g2d, x2d, into if G > 1 else into.view(K, C), G)
    torch.testing.assert_close(into, want, rtol=1e-4, atol=1e-2)
    out = onn._wgrad_gemm(g2d, x2d, None, G)
    torch.testing.assert_close(out.view(G, K, C), ref, rtol=1e-4, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("G,T,M,N", [(8, 784, 128, 1152), (1, 3000, 64, 576), (2, 196, 512, 4608),
                                     (8, 12544, 64, 152)])
def test_gemm_tn_parts_sum_to_product(G, T, M, N):
    """gemm_tn_parts: the unsummed split products of each group (the column-
    image weight gradients' parts, ops/nn.py _wgrad_parts) add up to a_g^T b_g."""
    g = torch.Generator().manual_seed(T + M)
    a = torch.randn(G * T, M, generator=g).to(torch.bfloat16).cuda()
    b = torch.randn(G * T, N, generator=g).to(torch.bfloat16).cuda()
    parts, S = _ops().gemm_tn_parts(a, b, G)
    assert parts.shape == (G * S, M, N)
    got = parts.view(G, S, M, N).sum(1)
    ref = torch.bmm(a.float().view(G, T, M).transpose(1, 2), b.float().view(G, T, N))
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-3 * (T ** 0.5) / 10)


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,N,splits", [(77, 1017, 128, 0), (300, 4160, 256, 0), (640, 50257, 768, 0),
                                          (130, 2111, 192, 3)])
def test_mm_nn_splitk_matches_fp32(M, K, N, splits):
    """Split-K NN GEMM with the K tail folded into the reduction (the tied LM
    head's dh = g W, K = 50,257) vs an fp32 reference; a's rows padded (the CE
    gradient's layout: only the first K columns are read)."""
    from commefficient_amd._ext import ops as _ops
    g = torch.Generator(device="cuda").manual_seed(13)
    ld = -(-K // 8) * 8 + 8
    abuf = torch.randn(M, ld, device="cuda", generator=g).to(torch.bfloat16)
    abuf[:, K:] = float("nan")  # never read
    a = abuf[:, :K]
    b = (torch.randn(K, N, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    out = _ops().mm_nn_splitk(a, b, splits)
    ref = a.float() @ b.float()
    assert out.dtype == torch.bfloat16 and out.shape == (M, N)
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err < 5e-3, err
    assert torch.equal(out, _ops().mm_nn_splitk(a, b, splits))  # deterministic
