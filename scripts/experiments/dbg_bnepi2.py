import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from commefficient_amd import _ext
_ext.load()
from commefficient_amd.models.common import ghost_batchnorm, GhostBatchNorm2d
from commefficient_amd.models.resnets import resnet50
from commefficient_amd.ops import nn as onn
torch.manual_seed(0)
model = resnet50(num_classes=10, input_hw=64).cuda().train()
x = torch.randn(64, 3, 64, 64, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
state = {k: v.clone() for k, v in model.state_dict().items()}
rec = {}
def hook(name):
    def f(m, inp, out):
        rec.setdefault(name, []).append((inp[0].float().clone(), out.float().clone(), getattr(inp[0], "_commeff_bnstats", "na")))
    return f
for n, m in model.named_modules():
    if isinstance(m, GhostBatchNorm2d):
        m.register_forward_hook(hook(n))
orig = onn.take_bnstats
log = []
def spy(t, G):
    st = getattr(t, "_commeff_bnstats", None)
    r = orig(t, G)
    log.append((tuple(t.shape), None if st is None else (st[1], st[2], t._version), r is not None))
    return r
onn.take_bnstats = spy
for on in (False, True):
    model.load_state_dict(state)
    onn._EPI["on"] = on
    log.clear()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16), ghost_batchnorm(model, 2):
        model(x)
    if on:
        for l in log[:12]: print("take", l)
names = list(rec.keys())
for n in names:
    (i0, o0, _), (i1, o1, _) = rec[n][0], rec[n][1]
    di = ((i1 - i0).norm() / i0.norm()).item(); do = ((o1 - o0).norm() / o0.norm()).item()
    print("%-22s in %.2e out %.2e" % (n, di, do), tuple(i0.shape))
    if do > 1e-2:
        break
