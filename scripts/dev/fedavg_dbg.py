import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from commefficient_amd import models
from commefficient_amd.parallel import dist
from commefficient_amd.parallel.fed_model import FedModel
from commefficient_amd.parallel.server import FedOptimizer
from commefficient_amd.utils.args import parse_args
from commefficient_amd.train import cv as drv
from commefficient_amd.train.losses import cv_loss
merge = sys.argv[1]
lr = float(sys.argv[2])
dev = sys.argv[3] if len(sys.argv) > 3 else "cpu"
ctx = dist.init(dev)
W = 10
argv = ["--dataset_name", "CIFAR100", "--synthetic", "--synthetic_size", "2000", "--model", "ResNet18",
        "--mode", "fedavg", "--error_type", "none", "--local_momentum", "0",
        "--virtual_momentum", "0.9", "--num_clients", "200", "--num_workers", str(W),
        "--local_batch_size", "-1", "--fedavg_batch_size", "-1", "--num_fedavg_epochs", "1",
        "--batchnorm", "--device", dev, "--merge_clients", merge, "--dtype", sys.argv[4] if len(sys.argv) > 4 else "fp32"]
args = parse_args(argv=argv, probe_port=False)
torch.manual_seed(0)
loader, _ = drv.get_data_loaders(args, ctx.device)
model = models.build_model(args, 100)
opt = torch.optim.SGD(model.parameters(), lr=lr)
fed = FedModel(model, cv_loss, args, cv_loss, num_clients=args.num_clients)
fopt = FedOptimizer(opt, args, fed)
it = iter(loader)
for i in range(int(sys.argv[5]) if len(sys.argv) > 5 else 8):
    rb = next(it)
    fopt.step()
    out = fed(rb)
    print(i, float(out[0].mean()), fed.w.norm().item())
