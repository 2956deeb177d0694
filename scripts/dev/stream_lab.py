"""Dev timing of the streamed conv forward on ResNet-9 shapes (500 images);
env COMMEFF_STREAM_* picks the variant.  One JSON line per run."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from commefficient_amd import ops  # noqa: E402

LAYERS = [("layer1", 64, 32, 128), ("res1", 128, 16, 128), ("layer2", 128, 16, 256), ("layer3", 256, 8, 512),
          ("l1dgrad", 128, 32, 64)]


def timeit(fn, n=30):
    for _ in range(5):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record(); fn(); b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return ts[len(ts) // 2]


out = {"tag": os.environ.get("TAG", ""), "ablate": os.environ.get("COMMEFF_STREAM_ABLATE", "0"),
       "grid": os.environ.get("COMMEFF_STREAM_GRID", "")}
torch.manual_seed(0)
for name, C, H, K in LAYERS:
    N = 500
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, 3, 3, device="cuda") * 0.05
    wf, wt = ops.conv_weight_prep(w)
    us = timeit(lambda: ops.conv3x3_fwd(x, wf, True))
    out[name] = round(us, 1)
    out[name + "_tf"] = round(2.0 * N * H * H * K * C * 9 / (us * 1e-6) / 1e12, 1)
print(json.dumps(out), flush=True)
