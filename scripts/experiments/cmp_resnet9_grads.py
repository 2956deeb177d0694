"""Per-parameter gradient agreement of ResNet-9: native bf16 / MIOpen bf16 vs fp32."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from commefficient_amd.models import ResNet9
from commefficient_amd.ops import nn as cnn

torch.manual_seed(0)
m = ResNet9().cuda()
x = torch.randn(16, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
res = {}
for name in ("fp32", "miopen", "native"):
    m.zero_grad(set_to_none=True)
    if name == "fp32":
        cnn.set_conv_backend("miopen")
        y = m(x)
    else:
        cnn.set_conv_backend(name)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x.to(torch.bfloat16))
    y.float().square().sum().backward()
    res[name] = [p.grad.detach().float().clone() for p in m.parameters()]
names = [n for n, _ in m.named_parameters()]
for i, n in enumerate(names):
    r = res["fp32"][i]
    e = lambda a: ((a - r).norm() / r.norm()).item()
    print(f"{n:30s} miopen {e(res['miopen'][i]):.4f} native {e(res['native'][i]):.4f}")
