"""GPT-2 MLP backward junctions in isolation: bias + GELU backward (with the
bias-gradient column partials) on [T, 3072] and the bias-only pass on [T, 768]."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from commefficient_amd import _ext  # noqa: E402


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / n


ops = _ext.ops()
T = int(os.environ.get("T", "9400"))
for N, gelu in ((3072, True), (768, False)):
    gf = torch.randn(T, N, device="cuda").bfloat16()
    u = torch.randn(T, N, device="cuda").bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    us = timeit(lambda: ops.bias_act_bwd_part(gf, u if gelu else None, b, gelu))
    mb = T * N * 2 * (3 if gelu else 1) / 1e6
    print(json.dumps({"N": N, "gelu": gelu, "us": round(us, 1), "TB/s": round(mb / us, 2),
                      "blocks": os.environ.get("AB_BA_BLOCKS", "512")}))
