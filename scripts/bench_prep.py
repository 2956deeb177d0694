#!/usr/bin/env python
"""Input-convolution (conv_prep) micro-benchmark at the headline batch
(500 x 3 x 32 x 32): forward and weight-gradient medians (HIP events).  The
tiles-per-wave knob COMMEFF_PREP_TPW (and the weight gradient's COMMEFF_PREP_WG_STEPS) is read
once per process, so a sweep runs this script once per value:

    for t in 2 4 8; do COMMEFF_PREP_TPW=$t python scripts/bench_prep.py; done
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from commefficient_amd.ops import nn as cnn  # noqa: E402


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    B, H, W = 500, 32, 32
    ops = cnn._ops()
    buf = torch.zeros(B, H, W, 4, dtype=torch.bfloat16, device="cuda")
    buf[..., :3] = torch.randn(B, H, W, 3, device="cuda").bfloat16()
    x = buf.permute(0, 3, 1, 2)[:, :3]
    w = torch.randn(64, 3, 3, 3, device="cuda") * 0.2
    y, mask = ops.conv_prep_fwd(x, w)
    r = {"tpw": os.environ.get("COMMEFF_PREP_TPW", "default")}
    r["fwd_us"] = timeit(lambda: ops.conv_prep_fwd(x, w))
    out_bytes = y.numel() * 2 + mask.numel() * 4 + B * H * W * 8
    r["fwd_TBps"] = out_bytes / r["fwd_us"] / 1e6
    gy = torch.randn_like(y, dtype=torch.float32).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dw = torch.zeros(64, 3, 3, 3, device="cuda")
    r["wgrad_us"] = timeit(lambda: ops.conv_prep_wgrad_into(gy, mask, x, dw))
    r["fill_y_us"] = timeit(lambda: y.fill_(0))  # write roofline at this size
    r["fill_TBps"] = y.numel() * 2 / r["fill_y_us"] / 1e6
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
