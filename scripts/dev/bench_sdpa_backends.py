"""GPT-2 PersonaChat attention shapes (64 sequences x 12 heads, L ~ 110, d 64,
causal, dropout 0.1): fwd+bwd time of each SDPA backend."""
import time
import torch
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel

N, nh, L, hd = 64, 12, 112, 64
qkv = torch.randn(N * L, 3 * nh * hd, device="cuda", dtype=torch.bfloat16)
q, k, v = (t.view(N, L, nh, hd).transpose(1, 2) for t in qkv.split(nh * hd, dim=1))
q, k, v = (t.detach().requires_grad_() for t in (q, k, v))
g = torch.randn(N, nh, L, hd, device="cuda", dtype=torch.bfloat16)


def run(backend, p):
    with sdpa_kernel([backend]):
        o = F.scaled_dot_product_attention(q, k, v, dropout_p=p, is_causal=True)
        o.backward(g)


for be in (SDPBackend.FLASH_ATTENTION, SDPBackend.EFFICIENT_ATTENTION, SDPBackend.MATH):
    for p in (0.0, 0.1):
        try:
            for _ in range(3):
                run(be, p)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(20):
                run(be, p)
            torch.cuda.synchronize()
            print(be, p, f"{(time.perf_counter() - t) / 20 * 1e6:.1f} us fwd+bwd", flush=True)
        except Exception as e:
            print(be, p, "FAIL", repr(e)[:150], flush=True)
