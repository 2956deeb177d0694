"""Dev timing of the sharded FetchSGD server's query + top-k on one rank's
group-major shard (ResNet-9 geometry: d = 6,568,640, 5 x 500,000, k = 50,000)
at world sizes 1 (whole table), 2, 4, 8: HIP-event medians, one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from commefficient_amd.ops import sketch_region  # noqa: E402
from commefficient_amd.ops.sketch_region import RegionHash  # noqa: E402


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
    d, c, r, k = 6568640, 500000, 5, 50000
    h = RegionHash(d, c, r, seed=5)
    out = {}
    for world in (1, 2, 4, 8):
        E, V, G = (torch.randn(r, c, device="cuda") * 1e-3 for _ in range(3))
        if world == 1:
            fn = lambda: sketch_region.topk(h, E, k, None, mom=(V, G, 0.9, 0.01, "virtual"))  # noqa: E731
        else:
            Gp = h.shard_groups(world)
            sh = lambda t: h.group_major(t, world)[:Gp].contiguous()  # noqa: E731
            Es, Vs, Gs = sh(E), sh(V), sh(G)
            fn = lambda: sketch_region.topk(h, Es, k, None, mom=(Vs, Gs, 0.9, 0.01, "virtual"), g0=0)  # noqa: E731
        out[f"world{world}_us"] = round(timeit(fn), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
