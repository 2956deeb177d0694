"""Round-0 per-client gradient rows: grouped path vs one client at a time
(tests/test_grouped.py engine geometry), before clip / weight decay / top-k.
Prints the relative error per client and the worst parameters."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from commefficient_amd.parallel.fed_model import FedModel  # noqa: E402
import test_grouped as tg  # noqa: E402

dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
rows = {}
orig = FedModel._client_tail


def rec(self, g, work):
    rows.setdefault(self._tag, []).append(g.detach().clone())
    return orig(self, g, work)


FedModel._client_tail = rec
for tag in ("on", "off"):
    fed, opt = tg._engine(tag, "cuda", dtype)
    fed.args.miopen_find = 0
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
    fed._tag = tag
    tg._rounds(fed, opt, "cuda", R=1)
    torch.cuda.synchronize()
    names = [(n, p.numel()) for n, p in fed.model.named_parameters()]
    offs = fed.flat.offsets
a, b = torch.stack(rows["on"]), torch.stack(rows["off"])
print("rows", a.shape, b.shape)
for c in range(a.shape[0]):
    print("client %d rel err %.4e |g| %.3e" % (c, ((a[c] - b[c]).norm() / b[c].norm()).item(),
                                                b[c].norm().item()))
for (n, k), o in zip(names, offs):
    for c in range(a.shape[0]):
        x, y = a[c, o:o + k], b[c, o:o + k]
        e = ((x - y).norm() / y.norm().clamp_min(1e-20)).item()
        if e > 2e-2:
            print("%-36s c%d numel %8d err %.3e |ref| %.3e" % (n, c, k, e, y.norm().item()))
# same ranking of top-k?
k = 300
for c in range(a.shape[0]):
    ia = set(a[c].abs().topk(k).indices.tolist())
    ib = set(b[c].abs().topk(k).indices.tolist())
    print("client %d top-%d overlap %d" % (c, k, len(ia & ib)))
