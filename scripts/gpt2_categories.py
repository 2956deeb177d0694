#!/usr/bin/env python
"""GPU time of one GPT-2 round (between the last two sketch-encode P1
kernels of a rocprofv3 kernel trace) by stream and kernel category."""
import collections
import csv
import sys


def cat(n):
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        return "hipBLASLt GEMM"
    for key, c in (("gemm_tn", "gemm_tn wgrad"), ("attn", "attention")):
        if key in n:
            return c
    if any(k in n for k in ("enc_p", "qry_q", "fx_", "enc_fx")):
        return "sketch codec"
    if any(k in n for k in ("hist_kernel", "count_kernel", "write_kernel")):
        return "topk"
    if any(k in n for k in ("resid_ln", "bias_gelu", "bias_act", "colsum")):
        return "LN/bias/GELU"
    if n.startswith("at::native") or "rocprim" in n or "softmax" in n:
        return "at::native/rocprim"
    return "other"


def main(path, detail=""):
    rows = []
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        n = n.replace("commeff::", "").split("(")[0]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], n))
    rows.sort()
    marks = [s for s, _, _, n in rows if "enc_p1" in n]
    lo, hi = marks[-2], marks[-1]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    ker = collections.defaultdict(lambda: [0.0, 0])
    for s, e, st, n in rows:
        if lo <= s < hi:
            per[st][cat(n)] += (e - s) / 1e3
            if detail and cat(n) == detail:
                ker[n][0] += (e - s) / 1e3
                ker[n][1] += 1
    print(f"# round window {(hi - lo) / 1e3:.1f} us")
    for st, d in sorted(per.items()):
        print(f"stream {st}: {sum(d.values()):.1f} us")
        for k, v in sorted(d.items(), key=lambda x: -x[1]):
            print(f"   {v:8.1f}  {k}")
    for n, (us, c) in sorted(ker.items(), key=lambda x: -x[1][0]):
        print(f"      {us:8.1f} {c:4d}  {n}")


if __name__ == "__main__":
    main(*sys.argv[1:])
