"""How far ahead of the GPU can the host enqueue?  Launches N long sleep
kernels back-to-back and records the host time of every launch: a launch that
takes ~one kernel's duration means the runtime blocked on an in-flight cap."""
import time
import torch

torch.cuda.init()
x = torch.zeros(1, device="cuda")
torch.cuda._sleep(1000)
torch.cuda.synchronize()
# calibrate: ~50 us per sleep kernel
t0 = time.perf_counter()
for _ in range(20):
    torch.cuda._sleep(100000)
torch.cuda.synchronize()
per = (time.perf_counter() - t0) / 20
cyc = int(100000 * 50e-6 / per)
torch.cuda.synchronize()
times = []
for i in range(400):
    h0 = time.perf_counter()
    torch.cuda._sleep(cyc)
    times.append((time.perf_counter() - h0) * 1e6)
torch.cuda.synchronize()
slow = [i for i, t in enumerate(times) if t > 25]
print("kernel ~50us; first blocking launch index:", slow[:5], "n_slow", len(slow))
print("launch us (first 10):", [round(t, 1) for t in times[:10]])
print("launch us (200-210):", [round(t, 1) for t in times[200:210]])
# same with x.add_ (small elementwise) interleaved: lead in kernels
