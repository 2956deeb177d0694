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
