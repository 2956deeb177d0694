#!/usr/bin/env python
"""Host-vs-GPU lag per kernel from a torch.profiler chrome trace
(``bench.py --torch-profile DIR``): for every kernel, the time between the
host's launch call and the kernel's GPU start.  A lag near zero means the GPU
was waiting for the host (host-bound stretch); a large lag means the host ran
ahead.  Prints the last round (between the last two starts of --marker) with
the host-side Python op that issued each launch.

    python scripts/launch_lag.py gpurun_out/tp/bench_trace.json --marker enc_p1
"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="enc_p1")
    ap.add_argument("--quiet", action="store_true", help="summary lines only")
    args = ap.parse_args()
    ev = json.load(open(args.trace))["traceEvents"]
    launches, kernels = {}, []
    for e in ev:
        if e.get("ph") != "X":
            continue
        cat = e.get("cat", "")
        corr = e.get("args", {}).get("correlation")
        if cat == "cuda_runtime" and corr is not None:
            launches[corr] = e
        elif cat in ("kernel", "gpu_memcpy", "gpu_memset") and corr is not None:
            kernels.append(e)
    kernels.sort(key=lambda e: e["ts"])
    starts = [i for i, k in enumerate(kernels) if args.marker in k["name"]]
    if len(starts) < 2:
        print("marker not found twice")
        return
    a, b = starts[-2], starts[-1]
    t0 = kernels[a]["ts"]
    if not args.quiet:
        print("# gpu_t(us)  host_t(us)  lag(us)  dur(us)  kernel  <- runtime call")
    lags = []
    for k in kernels[a:b]:
        l = launches.get(k["args"]["correlation"])
        if l is None:
            continue
        lag = k["ts"] - (l["ts"] + l.get("dur", 0))
        lags.append(lag)
        if not args.quiet:
            print("%9.1f %10.1f %8.1f %8.1f  %-60s <- %s" % (k["ts"] - t0, l["ts"] - t0, lag, k.get("dur", 0),
                                                          k["name"][:60], l["name"]))
    print("# kernels %d  min lag %.1f  mean lag %.1f" % (len(lags), min(lags), sum(lags) / len(lags)))
    # GPU idle stretches of the round (union over streams) with the lag of the
    # kernel that ended each: lag ~ 0 there = the host had not launched it yet
    ks = sorted(kernels[a:b], key=lambda k: k["ts"])
    end, idle, host_idle = ks[0]["ts"], 0.0, 0.0
    for k in ks:
        if k["ts"] > end:
            gap = k["ts"] - end
            idle += gap
            l = launches.get(k["args"]["correlation"])
            if l is not None and k["ts"] - (l["ts"] + l.get("dur", 0)) < 50:
                host_idle += gap
        end = max(end, k["ts"] + k.get("dur", 0))
    print("# round %.1f us, GPU idle %.1f us, of which waiting on a late launch %.1f us"
          % (end - ks[0]["ts"], idle, host_idle))


if __name__ == "__main__":
    main()
