"""Dev timing of the native ResNet-9 conv3x3 kernels at the bench batch (500 images):
forward (ReLU epilogue), input gradient and weight gradient per layer, HIP-event
medians.  One JSON line; `TAG` labels it."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from commefficient_amd import ops  # noqa: E402

LAYERS = [("layer1", 64, 32, 128), ("res1", 128, 16, 128), ("layer2", 128, 16, 256),
          ("layer3", 256, 8, 512), ("res3", 512, 4, 512)]


def timeit(fn, n=30):
    for _ in range(5):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return ts[len(ts) // 2]


def main():
    out = {"tag": os.environ.get("TAG", "")}
    torch.manual_seed(0)
    N = 500
    tot = 0.0
    for name, C, H, K in LAYERS:
        x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn(N, K, H, H, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = torch.randn(K, C, 3, 3, device="cuda") * 0.05
        wf, wt = ops.conv_weight_prep(w)
        f = timeit(lambda: ops.conv3x3_fwd(x, wf, True))
        d = timeit(lambda: ops.conv3x3_fwd(dy, wt, False))
        g = timeit(lambda: ops.conv3x3_wgrad(dy, x))
        fl = 2.0 * N * H * H * K * C * 9
        out[name] = {"fwd": round(f, 1), "dgrad": round(d, 1), "wgrad": round(g, 1),
                     "fwd_tf": round(fl / f / 1e6, 0), "dgrad_tf": round(fl / d / 1e6, 0),
                     "wgrad_tf": round(fl / g / 1e6, 0)}
        tot += f + d + g
    out["total_us"] = round(tot, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
