#!/usr/bin/env python
"""Convergence runs: ResNet-9 on learnable synthetic CIFAR-10 through the
real training driver (train/cv.py), one run per compression mode, with the
reference's schedule (triangular LR 0 -> lr_scale at pivot_epoch -> 0 at
num_epochs; /root/reference/CommEfficient/cv_train.py:394-404) and the
reference's FetchSGD CIFAR-10 geometry (10,000 clients x 5 images, 100 per
round, k = 50,000, 5 x 500,000 sketch, virtual momentum 0.9 + virtual error;
server math fed_aggregator.py:568-613).

Writes one JSON line per (mode, epoch) to --out and prints a summary:

  python scripts/convergence.py --out profiles/r3_convergence.jsonl
  python scripts/convergence.py --modes sketch,uncompressed --epochs 6

Data: --difficulty hard (default) = 0.25 x the class's 4x4 block pattern +
0.2 x a random other class's pattern + Gaussian noise of std 60
(data/image_datasets.py SyntheticImageFedDataset); a matched filter that
knows the patterns scores ~94.6 %, so the curves test the optimisation path
end to end without saturating -- they are not CIFAR-10 accuracies.
Measured curves: profiles/r3_convergence.jsonl (tests/test_convergence.py).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# per mode: the reference flags (utils.py:102-230) for that mode's CIFAR-10 run
MODES = {
    "sketch": ["--mode", "sketch", "--error_type", "virtual", "--local_momentum", "0",
               "--virtual_momentum", "0.9", "--k", "50000", "--num_rows", "5",
               "--num_cols", "500000", "--num_blocks", "20"],
    # the same sketch in the reference's CSVec hash layout (numBlocks = 20
    # multiply-shift hashes; --encode planned) instead of the region family
    "sketch_planned": ["--mode", "sketch", "--error_type", "virtual", "--local_momentum", "0",
                       "--virtual_momentum", "0.9", "--k", "50000", "--num_rows", "5",
                       "--num_cols", "500000", "--num_blocks", "20", "--encode", "planned"],
    "true_topk": ["--mode", "true_topk", "--error_type", "virtual", "--local_momentum", "0",
                  "--virtual_momentum", "0.9", "--k", "50000"],
    "uncompressed": ["--mode", "uncompressed", "--error_type", "none", "--local_momentum", "0",
                     "--virtual_momentum", "0.9"],
    # local error / momentum live per client ([clients, d] fp32 each): 500 clients
    # of 100 images, 20 per round keeps that at 2 x 13 GB
    "local_topk": ["--mode", "local_topk", "--error_type", "local", "--local_momentum", "0.9",
                   "--virtual_momentum", "0", "--k", "50000", "--num_clients", "500",
                   "--num_workers", "20", "--local_batch_size", "25"],
    "fedavg": ["--mode", "fedavg", "--error_type", "none", "--local_momentum", "0",
               "--virtual_momentum", "0", "--num_fedavg_epochs", "1",
               "--fedavg_batch_size", "-1", "--num_clients", "500", "--num_workers", "20"],
}


class JsonlRows:
    def __init__(self, path, mode, extra):
        self.f = open(path, "a") if path else None
        self.mode, self.extra = mode, extra
        self.rows = []

    def append(self, row):
        r = dict(mode=self.mode, **self.extra, **{k: (float(v) if isinstance(v, (int, float))
                                                      else v) for k, v in row.items()})
        self.rows.append(r)
        if self.f is not None:
            self.f.write(json.dumps(r) + "\n")
            self.f.flush()


def run(mode, epochs, pivot, lr_scale, device, dtype, out, size, seed=21, extra=(),
        difficulty="hard"):
    from commefficient_amd.train import cv
    from commefficient_amd.utils.args import parse_args
    argv = ["--dataset_name", "CIFAR10", "--synthetic", "--synthetic_size", str(size),
            "--num_clients", "10000", "--num_workers", "100", "--local_batch_size", "-1",
            "--device", device, "--dtype", dtype, "--num_epochs", str(epochs),
            "--pivot_epoch", str(pivot), "--lr_scale", str(lr_scale), "--weight_decay", "5e-4",
            "--valid_batch_size", "100", "--seed", str(seed), "--port", "29731",
            "--synthetic_difficulty", difficulty]
    argv += MODES[mode] + list(extra)
    args = parse_args(argv=argv, probe_port=False)
    log = JsonlRows(out, mode, {"epochs": epochs, "lr_scale": lr_scale, "pivot": pivot,
                                "difficulty": difficulty,
                                "dtype": dtype, "clients": args.num_clients,
                                "per_round": args.num_workers})
    t0 = time.time()
    fed = cv.main(args, loggers=(log,))
    wall = time.time() - t0
    return log.rows, fed, wall


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--modes", default="sketch,true_topk,uncompressed,local_topk")
    p.add_argument("--epochs", type=float, default=24)
    p.add_argument("--pivot", type=float, default=5)
    p.add_argument("--lr_scale", type=str, default="0.4",
                   help="peak LR; one value, or mode=value pairs (e.g. sketch=0.4,uncompressed=0.1)")
    p.add_argument("--difficulty", default="hard", choices=["easy", "hard"])
    p.add_argument("--size", type=int, default=50000, help="synthetic training images")
    p.add_argument("--device", default="cuda")
    p.add_argument("--dtype", default="bf16")
    p.add_argument("--out", default="gpurun_out/convergence.jsonl")
    b = p.parse_args()
    if b.out:
        os.makedirs(os.path.dirname(b.out) or ".", exist_ok=True)
    summary = {}
    lrs = {}
    for part in b.lr_scale.split(","):
        if "=" in part:
            k, v = part.split("=")
            lrs[k] = float(v)
        else:
            lrs["*"] = float(part)
    for spec in b.modes.split(","):
        # "mode" (LR from --lr_scale) or "mode@lr" (matched / best-LR grids in one call)
        mode, _, lr_s = spec.partition("@")
        lr = float(lr_s) if lr_s else lrs.get(mode, lrs.get("*", 0.4))
        rows, fed, wall = run(mode, b.epochs, b.pivot, lr, b.device, b.dtype, b.out,
                              b.size, difficulty=b.difficulty)
        last = rows[-1] if rows else {}
        summary[spec] = {"test_acc": last.get("test_acc"), "test_loss": last.get("test_loss"),
                         "rounds": fed.round_idx, "wall_s": round(wall, 1), "lr_scale": lr}
        print("CONVERGENCE", spec, json.dumps(summary[spec]), flush=True)
    print("SUMMARY", json.dumps(summary))


if __name__ == "__main__":
    main()
