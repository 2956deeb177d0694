"""Per-parameter error of grouped (per-client) weight gradients on the GPU
vs per-group fp32 autograd (debug helper for tests/test_grouped.py)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import torch, torch.nn.functional as F
from commefficient_amd.models.common import ghost_batchnorm
from commefficient_amd.models.resnets import Bottleneck, ResNet
from commefficient_amd.ops.grouped import GroupedGrads, grouped_grads
from commefficient_amd.parallel.flat import FlatParams
from test_grouped import _per_group_reference

G = int(sys.argv[1]) if len(sys.argv) > 1 else 2
HW = int(sys.argv[2]) if len(sys.argv) > 2 else 32
torch.manual_seed(0)
model = ResNet(Bottleneck, [1, 1, 1, 1], num_classes=7, input_hw=HW).cuda().to(memory_format=torch.channels_last)
x = torch.randn(4 * G, 3, HW, HW, device="cuda").to(memory_format=torch.channels_last)
y = torch.randint(0, 7, (4 * G,), device="cuda")
ref_model = ResNet(Bottleneck, [1, 1, 1, 1], num_classes=7, input_hw=HW).cuda().float()
with torch.no_grad():
    model.fc.weight.mul_(float(os.environ.get("FC_SCALE", "1")))
ref_model.load_state_dict(model.state_dict())
with torch.no_grad():
    for p in ref_model.parameters():
        p.copy_(p.to(torch.bfloat16).float())
ref = _per_group_reference(ref_model.to(memory_format=torch.channels_last), x, y, G)
names = [n for n, p in model.named_parameters()]
bufs = {}
for mode in ("grouped", "bf16-per-group"):
    m2 = model
    flat = FlatParams(m2, "cuda") if mode == "grouped" else flat
    index = {id(p): (o, p.shape) for p, o in zip(flat.params, flat.offsets)}
    if mode == "grouped":
        buf = torch.zeros(G, flat.d, device="cuda")
        flat.zero_grad()
        with grouped_grads(GroupedGrads(G, buf, index)), ghost_batchnorm(m2, G), torch.autocast("cuda", dtype=torch.bfloat16):
            per_ex = F.cross_entropy(m2(x).float(), y, reduction="none")
            (per_ex.sum() / 4).backward()
        print("leak", flat.g.abs().max().item())
    else:
        rows = []
        n = 4
        for g in range(G):
            flat.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m2(x[g*n:(g+1)*n]).float(), y[g*n:(g+1)*n])
            loss.backward()
            rows.append(flat.g.clone())
        buf = torch.stack(rows)
    bufs[mode] = buf.clone()
    print("==", mode, "rel err vs fp32 ref per group:",
          [round(((buf[g] - ref[g]).norm() / ref[g].norm()).item(), 4) for g in range(G)])
    continue
    for (nm, p), o in zip(m2.named_parameters(), flat.offsets):
        k = p.numel()
        for g in range(G):
            a, b = buf[g, o:o+k], ref[g, o:o+k]
            e = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
            if e > 0.03:
                print(f"{nm:40s} g{g} shape {tuple(p.shape)} err {e:.3f} |ref| {b.norm().item():.3e} |got| {a.norm().item():.3e}")
a, b = bufs["grouped"], bufs["bf16-per-group"]
print("grouped vs bf16 per-group:", [round(((a[g] - b[g]).norm() / b[g].norm()).item(), 4) for g in range(G)])
for (nm, p), o in zip(model.named_parameters(), flat.offsets):
    k = p.numel()
    for g in range(G):
        e = ((a[g, o:o+k] - b[g, o:o+k]).norm() / b[g, o:o+k].norm().clamp_min(1e-12)).item()
        if e > 0.05:
            print(f"{nm:40s} g{g} {tuple(p.shape)} grouped-vs-pergroup err {e:.3f}")
