"""Which host ops launch the device-to-device copies of a torch.profiler chrome
trace: for every GPU event whose name matches a pattern (default: the runtime's
copy kernels / DtoD memcpys), the CPU ops enclosing its launch (by correlation
id -> runtime launch event -> enclosing CPU op intervals on that thread).
Usage: python scripts/dev/trace_copies.py trace.json [pattern]"""
import collections
import json
import sys


def main():
    tr = json.load(open(sys.argv[1]))
    pat = sys.argv[2] if len(sys.argv) > 2 else "copyBuffer|Memcpy DtoD|bfloat16_copy|direct_copy"
    pats = pat.split("|")
    ev = tr["traceEvents"] if isinstance(tr, dict) else tr
    gpu, launches, cpu_ops = [], {}, collections.defaultdict(list)
    for e in ev:
        if e.get("ph") != "X":
            continue
        cat = e.get("cat", "")
        args = e.get("args", {})
        if cat in ("kernel", "gpu_memcpy", "gpu_memset"):
            gpu.append(e)
        elif cat == "cuda_runtime":
            if "correlation" in args:
                launches[args["correlation"]] = e
        elif cat == "cpu_op":
            cpu_ops[(e.get("pid"), e.get("tid"))].append(e)
    for k in cpu_ops:
        cpu_ops[k].sort(key=lambda e: e["ts"])
    cnt = collections.Counter()
    for g in gpu:
        if not any(p in g.get("name", "") for p in pats):
            continue
        l = launches.get(g.get("args", {}).get("correlation"))
        if l is None:
            cnt[("<no launch>", g["name"][:40])] += 1
            continue
        t = l["ts"]
        chain = [o["name"] for o in cpu_ops[(l.get("pid"), l.get("tid"))] if o["ts"] <= t <= o["ts"] + o.get("dur", 0)]
        cnt[(" > ".join(chain[-4:]), g["name"][:40])] += 1
    for (chain, name), n in cnt.most_common(40):
        print(f"{n:5d}  {name:40s}  {chain}")


if __name__ == "__main__":
    main()
