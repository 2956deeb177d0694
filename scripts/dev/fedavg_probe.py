import sys, torch, numpy as np
sys.path.insert(0, '.')
from commefficient_amd import models
from commefficient_amd.parallel import dist
from commefficient_amd.parallel.fed_model import FedModel
from commefficient_amd.parallel.server import FedOptimizer
from commefficient_amd.utils.args import parse_args
from commefficient_amd.train import cv as drv
from commefficient_amd.train.losses import cv_loss
mode = sys.argv[1]; lr = float(sys.argv[2]); W = int(sys.argv[3]); dev = sys.argv[4]; dt = sys.argv[5]
torch.set_num_threads(8)
ctx = dist.init(dev)
argv = ["--dataset_name", "CIFAR100", "--synthetic", "--model", "ResNet18", "--mode", mode,
        "--error_type", "none", "--local_momentum", "0", "--virtual_momentum", "0.9",
        "--num_clients", "2000", "--num_workers", str(W), "--local_batch_size", "-1",
        "--fedavg_batch_size", "-1", "--num_fedavg_epochs", "1", "--batchnorm", "--device", dev,
        "--dtype", dt, "--seed", "21"]
args = parse_args(argv=argv, probe_port=False)
torch.manual_seed(0)
loader, _ = drv.get_data_loaders(args, ctx.device)
model = models.build_model(args, 100)
opt = torch.optim.SGD(model.parameters(), lr=lr)
fed = FedModel(model, cv_loss, args, cv_loss, num_clients=args.num_clients)
fopt = FedOptimizer(opt, args, fed)
it = iter(loader)
for r in range(12):
    out = fed(next(it)); fopt.step()
    print(r, round(float(out[0].mean()), 4), float(fed.w.abs().max()), flush=True)
