"""Worker for test_distributed.py::test_two_ranks_one_gpu: one rank of a
2-rank run (torchrun env) of full-size ResNet-9 FetchSGD rounds on cuda:0,
both ranks on the same GPU over gloo (COMMEFF_DIST_BACKEND=gloo)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(out_dir, mode, rounds):
    from commefficient_amd import models
    from commefficient_amd.data import make_synthetic
    from commefficient_amd.data.device_loader import DeviceFedLoader
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.server import FedOptimizer
    from commefficient_amd.train.losses import cv_loss
    from commefficient_amd.utils.args import parse_args
    ctx = dist.init("cuda")
    extra = {"sketch": ["--error_type", "virtual", "--local_momentum", "0", "--virtual_momentum",
                        "0.9", "--k", "5000", "--num_rows", "5", "--num_cols", "50000"],
             "true_topk": ["--error_type", "virtual", "--local_momentum", "0",
                           "--virtual_momentum", "0.9", "--k", "5000"]}[mode]
    args = parse_args(argv=["--mode", mode, "--device", "cuda", "--dtype", "bf16",
                            "--num_clients", "40", "--num_workers", "8", "--local_batch_size",
                            "-1", "--dataset_name", "CIFAR10", "--synthetic"] + extra,
                      probe_port=False)
    torch.manual_seed(0)
    model = models.build_model(args, 10)
    ds = make_synthetic("CIFAR10", train=True, num_clients=40, size=400, seed=3)
    loader = DeviceFedLoader(ds, 8, -1, ctx.device, seed=5, augment=True, out_bf16=True)
    fed = FedModel(model, cv_loss, args, num_clients=40)
    opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.05), args, fed)
    it = iter(loader)
    losses = []
    for _ in range(rounds):
        loss, acc, dl, ul = fed(next(it))
        opt.step()
        losses.append(loss.clone())
    torch.cuda.synchronize()
    torch.save({"w": fed.w.cpu(), "loss": torch.stack(losses).cpu()},
               os.path.join(out_dir, f"r{ctx.rank}_w{ctx.world_size}.pt"))
    dist.shutdown()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]))
