import torch, time
a = torch.randn(7000, 768, device="cuda", dtype=torch.bfloat16)
b = torch.randn(7000, 3072, device="cuda", dtype=torch.bfloat16)
c = torch.zeros(768, 3072, device="cuda")
ref = a.float().t() @ b.float()
try:
    r = torch.mm(a.t(), b, out_dtype=torch.float32)
    print("mm out_dtype ok", r.dtype, float((r - ref).abs().max()))
except Exception as e:
    print("mm out_dtype FAIL", repr(e)[:300])
try:
    r = torch.addmm(c, a.t(), b, out_dtype=torch.float32)
    print("addmm out_dtype ok", r.dtype, float((r - ref).abs().max()))
except Exception as e:
    print("addmm out_dtype FAIL", repr(e)[:300])
try:
    c.zero_()
    torch.addmm(c, a.t(), b, out_dtype=torch.float32, out=c)
    torch.addmm(c, a.t(), b, out_dtype=torch.float32, out=c)
    print("addmm out= ok", float((c - 2 * ref).abs().max()), float(ref.abs().max()))
except Exception as e:
    print("addmm out= FAIL", repr(e)[:300])
for name, fn in [("bf16 mm", lambda: torch.mm(a.t(), b)),
                 ("f32 out mm", lambda: torch.mm(a.t(), b, out_dtype=torch.float32)),
                 ("addmm acc", lambda: torch.addmm(c, a.t(), b, out_dtype=torch.float32, out=c))]:
    try:
        for _ in range(3): fn()
        torch.cuda.synchronize(); t = time.perf_counter()
        for _ in range(20): fn()
        torch.cuda.synchronize(); print(name, (time.perf_counter() - t) / 20 * 1e6, "us")
    except Exception as e:
        print(name, "FAIL", repr(e)[:200])
