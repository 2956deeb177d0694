"""Debug helper: which state diverges between two identical GPU FetchSGD runs (used to
find that only the binned, LDS-atomic sketch path is not bitwise reproducible)."""
import sys, torch
sys.path.insert(0, '.')
from commefficient_amd import models
from commefficient_amd.data import make_synthetic
from commefficient_amd.data.device_loader import DeviceFedLoader
from commefficient_amd.parallel import dist
from commefficient_amd.parallel.fed_model import FedModel
from commefficient_amd.train.losses import cv_loss
from commefficient_amd.utils.args import parse_args

def run():
    dist.init("cuda")
    args = parse_args(argv=["--dataset_name", "CIFAR10", "--synthetic", "--synthetic_size", "800",
                            "--mode", "sketch", "--error_type", "virtual", "--local_momentum", "0",
                            "--virtual_momentum", "0.9", "--k", "5000", "--num_rows", "5",
                            "--num_cols", "50000", "--num_clients", "80", "--num_workers", "16",
                            "--local_batch_size", "-1", "--weight_decay", "5e-4",
                            "--device", "cuda"], probe_port=False)
    torch.manual_seed(0)
    ds = make_synthetic("CIFAR10", train=True, num_clients=80, size=800, seed=1)
    loader = DeviceFedLoader(ds, 16, -1, "cuda", seed=2, augment=True, out_bf16=True)
    model = models.build_model(args, 10)
    fed = FedModel(model, cv_loss, args, num_clients=80)
    b = next(iter(loader))
    fed(b)
    torch.cuda.synchronize()
    names = [n for n, _ in model.named_parameters()]
    return fed.flat.g.clone(), [(n, p.numel()) for n, p in model.named_parameters()], fed._payload.clone()

g1, meta, p1 = run()
g2, _, p2 = run()
o = 0
for n, k in meta:
    d = (g1[o:o+k] - g2[o:o+k]).abs()
    print(f"{n:40s} {k:8d} ndiff={(d>0).sum().item():8d} max={d.max().item():.3e}")
    o += k
d = (p1 - p2).abs()
print("payload ndiff", (d > 0).sum().item(), "max", d.max().item(), "numel", p1.numel())
