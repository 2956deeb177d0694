import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from commefficient_amd import _ext
_ext.load()
from commefficient_amd.models.common import ghost_batchnorm
from commefficient_amd.models.resnets import resnet50
from commefficient_amd.ops import nn as onn
torch.manual_seed(0)
model = resnet50(num_classes=10, input_hw=64).cuda().train()
x = torch.randn(64, 3, 64, 64, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
tgt = torch.randint(0, 10, (64,), device="cuda")
state = {k: v.clone() for k, v in model.state_dict().items()}
res = []
for on in (False, False, True):
    model.load_state_dict(state)
    model.zero_grad(set_to_none=True)
    onn._EPI["on"] = on
    with torch.autocast("cuda", dtype=torch.bfloat16), ghost_batchnorm(model, 2):
        out = model(x)
        loss = torch.nn.functional.cross_entropy(out.float(), tgt)
    loss.backward()
    res.append((loss.item(), out.float().clone(), {n: (p.grad.float().clone() if p.grad is not None else None) for n, p in model.named_parameters()}))
    print("on", on, "loss", loss.item(), flush=True)
for j in (1, 2):
    print("run", j, "vs 0: out rel", ((res[j][1] - res[0][1]).norm() / res[0][1].norm()).item())
    worst = []
    for n in res[0][2]:
        a, b = res[0][2][n], res[j][2][n]
        if a is None or b is None:
            print("  none-mismatch", n, a is None, b is None); continue
        r = ((b - a).norm() / a.norm().clamp_min(1e-12)).item()
        worst.append((r, n))
    worst.sort(reverse=True)
    for r, n in worst[:8]:
        print("  %.3e %s" % (r, n))
