#!/usr/bin/env python
"""Throughput of the secondary BASELINE.json configurations (synthetic data,
random init, 1..N GPUs via torch.distributed.run):

  imagenet_local_topk  ResNet-101 ImageNet-shaped (3x224x224, 1000 classes),
                       local top-k + local error feedback
  gpt2_sketch          GPT-2-small double heads on PersonaChat-shaped tokens,
                       FetchSGD (k=50k, 5 x 500k)
  cifar100_fedavg      ResNet-18 CIFAR-100, 10,000 non-iid clients, 100/round
                       per GPU, FedAvg (1 local epoch)

Prints one JSON line per config (rank 0) with examples/s and ms/round.
Usage: python scripts/bench_configs.py --config NAME [--steps K --warmup W]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cfg_args(name, N, b):
    if name == "imagenet_local_topk":
        W = b.clients or 8 * N
        return W, ["--dataset_name", "ImageNet", "--synthetic", "--synthetic_size", str(W * 32 * 2),
                   "--model", "ResNet101", "--mode", "local_topk", "--error_type", "local",
                   "--local_momentum", "0.9", "--virtual_momentum", "0", "--k", "500000",
                   "--num_clients", str(W * 2), "--num_workers", str(W), "--local_batch_size", "32",
                   "--iid", "--batchnorm"]
    if name == "gpt2_sketch":
        W = b.clients or 4 * N
        return W, ["--dataset_name", "PERSONA", "--synthetic", "--model", "GPT2DoubleHeads",
                    "--mode", "sketch", "--error_type", "virtual", "--local_momentum", "0",
                    "--virtual_momentum", "0.9", "--k", "50000", "--num_rows", "5",
                    "--num_cols", "500000", "--num_clients", "17568", "--num_workers", str(W),
                    "--local_batch_size", "8", "--num_candidates", "2", "--max_history", "2",
                    # the next rounds' records built in 2 worker processes (the
                    # reference's DataLoader workers); the timed loop then pulls
                    # each round from the loader itself
                    "--train_dataloader_workers", "2"]
    if name == "cifar100_fedavg":
        W = b.clients or 100 * N
        return W, ["--dataset_name", "CIFAR100", "--synthetic", "--model", "ResNet18",
                   "--mode", "fedavg", "--error_type", "none", "--local_momentum", "0",
                   "--virtual_momentum", "0.9", "--num_clients", "10000", "--num_workers", str(W),
                   "--local_batch_size", "-1", "--fedavg_batch_size", "-1",
                   "--num_fedavg_epochs", "1", "--batchnorm"]
    if name == "cifar100_fedavg_local":
        # multi-step local SGD: 5 local epochs of full-batch steps per client
        W = b.clients or 100 * N
        return W, ["--dataset_name", "CIFAR100", "--synthetic", "--model", "ResNet18",
                   "--mode", "fedavg", "--error_type", "none", "--local_momentum", "0",
                   "--virtual_momentum", "0.9", "--num_clients", "10000", "--num_workers", str(W),
                   "--local_batch_size", "-1", "--fedavg_batch_size", "-1",
                   "--num_fedavg_epochs", "5", "--batchnorm"]
    if name == "imagenet_fixup50_uncompressed":
        # the reference's ImageNet example run (imagenet.sh:2-21): FixupResNet50,
        # uncompressed, 7 clients x 64 per round, virtual momentum. The script's
        # --mixup/--mixup_alpha flags are undefined in the reference's parser
        # (its mixup loss is unreachable, cv_train.py:74-80), so plain CE here.
        W = b.clients or 7 * N
        return W, ["--dataset_name", "ImageNet", "--synthetic", "--synthetic_size", str(W * 64 * 2),
                   "--model", "FixupResNet50", "--mode", "uncompressed", "--error_type", "virtual",
                   "--local_momentum", "0", "--virtual_momentum", "0.9", "--weight_decay", "1e-4",
                   "--num_clients", str(W), "--num_workers", str(W), "--local_batch_size", "64",
                   "--iid"]
    if name == "cifar10_resnet9_fedavg_local":
        # the headline model under FedAvg: 5 local full-batch steps per client
        W = b.clients or 100 * N
        return W, ["--dataset_name", "CIFAR10", "--synthetic", "--model", "ResNet9",
                   "--mode", "fedavg", "--error_type", "none", "--local_momentum", "0",
                   "--virtual_momentum", "0.9", "--num_clients", "10000", "--num_workers", str(W),
                   "--local_batch_size", "-1", "--fedavg_batch_size", "-1",
                   "--num_fedavg_epochs", "5"]
    raise ValueError(name)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", required=True,
                   choices=["imagenet_local_topk", "gpt2_sketch", "cifar100_fedavg",
                            "cifar100_fedavg_local", "cifar10_resnet9_fedavg_local",
                            "imagenet_fixup50_uncompressed"])
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--clients", type=int, default=0, help="clients per round (total)")
    p.add_argument("extra", nargs=argparse.REMAINDER,
                   help="extra fed_train flags after '--' (e.g. -- --encode direct)")
    b = p.parse_args()
    from commefficient_amd import models
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.server import FedOptimizer
    from commefficient_amd.utils.args import parse_args
    ctx = dist.init("cuda")
    N = ctx.world_size
    W, argv = cfg_args(b.config, N, b)
    extra = [x for x in b.extra if x != "--"]
    args = parse_args(argv=argv + ["--device", "cuda", "--seed", "21"] + extra, probe_port=False)
    torch.manual_seed(0)
    if b.config == "gpt2_sketch":
        from commefficient_amd.train import gpt2 as drv
        from commefficient_amd.models.gpt2 import GPT2DoubleHeads
        from commefficient_amd.train.losses import gpt2_loss_train, gpt2_loss_val
        model = GPT2DoubleHeads("gpt2")
        loader, _ = drv.get_data_loaders(args, ctx.device)
        loss, vloss = gpt2_loss_train, gpt2_loss_val
        unit = "utterances/s"
    else:
        from commefficient_amd.train import cv as drv
        from commefficient_amd.train.losses import cv_loss
        loader, _ = drv.get_data_loaders(args, ctx.device)
        ncls = {"ImageNet": 1000, "CIFAR100": 100, "CIFAR10": 10}[args.dataset_name]
        model = models.build_model(args, ncls)
        loss = vloss = cv_loss
        unit = "images/s"
    # FedAvg on non-iid single-class clients diverges at a constant 0.05 without the
    # reference warm-up schedule (5 local epochs: NaN loss by ~round 10); the
    # throughput is LR-independent
    opt = torch.optim.SGD(model.parameters(), lr=0.01 if b.config.startswith("cifar100_fedavg") else 0.05)
    fed = FedModel(model, loss, args, vloss, num_clients=args.num_clients)
    fopt = FedOptimizer(opt, args, fed)
    it = iter(loader)

    def next_batch():
        nonlocal it
        while True:
            try:
                rb = next(it)
            except StopIteration:
                it = iter(loader)
                continue
            if len(np.unique(rb.client_ids)) == W:
                return rb

    # with loader workers the rounds are pulled inside the timed loop (the
    # workers build the next rounds meanwhile); else built lazily from
    # pre-drawn batches (the records are assembled inside the timed rounds)
    streamed = getattr(args, "train_dataloader_workers", 0) > 0
    batches = [] if streamed else [next_batch() for _ in range(b.warmup + b.steps)]

    class _Batches:
        def __getitem__(self, i):
            return next_batch() if streamed else batches[i]
    batches_at = _Batches()
    n_ex = []
    for i in range(b.warmup):
        fed(batches_at[i])
        fopt.step()
    torch.cuda.synchronize()
    dist.barrier()
    if os.environ.get("COMMEFF_SYNC_DEBUG"):
        # report every host<->device synchronisation of the timed rounds with
        # the Python stack that caused it (they stall the host's enqueue-ahead)
        import traceback
        import warnings

        def _show(msg, cat, fn, ln, file=None, line=None):
            st = [f for f in traceback.extract_stack()[:-1] if "commefficient_amd" in f.filename
                  or "bench_configs" in f.filename or "transformers" in f.filename]
            print("SYNC:", str(msg)[:80], "|", " <- ".join(
                f"{os.path.basename(f.filename)}:{f.lineno}" for f in reversed(st[-6:])), flush=True)
        warnings.showwarning = _show
        warnings.simplefilter("always")
        torch.cuda.set_sync_debug_mode("warn")
    allocs0 = torch.cuda.memory_stats().get("num_device_alloc", 0)
    prof_out = os.environ.get("COMMEFF_PROFILE_ROUNDS")
    if prof_out:  # cProfile of the timed rounds only (host cost per call site)
        import cProfile
        cprof = cProfile.Profile()
        cprof.enable()
    t0 = time.perf_counter()
    host = 0.0  # host time spent enqueueing (the GPU idles when this is the bound)
    for i in range(b.warmup, b.warmup + b.steps):
        h0 = time.perf_counter()
        rb = batches_at[i]
        n_ex.append(len(rb))
        out = fed(rb)
        fopt.step()
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    if prof_out:
        cprof.disable()
        import pstats
        with open(prof_out, "w") as f:
            st = pstats.Stats(cprof, stream=f)
            st.sort_stats("tottime").print_stats(50)
            st.sort_stats("cumtime").print_stats(80)
    dist.barrier()
    el = dist.max_over_ranks(time.perf_counter() - t0)
    tp = os.environ.get("COMMEFF_TORCH_PROFILE")
    if tp:  # 3 more rounds under torch.profiler (host launch vs GPU start: scripts/launch_lag.py)
        from torch.profiler import ProfilerActivity, profile
        shapes = os.environ.get("COMMEFF_TORCH_PROFILE_SHAPES") == "1"
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=shapes) as prof:
            for i in range(b.warmup, b.warmup + min(3, b.steps)):
                fed(batches_at[i])
                fopt.step()
            torch.cuda.synchronize()
        if ctx.is_main:
            os.makedirs(tp, exist_ok=True)
            prof.export_chrome_trace(os.path.join(tp, "trace.json"))
    ss = os.environ.get("COMMEFF_STOCK_SITES")
    if ss:  # 2 more rounds: call sites of stock (aten) ops that launch kernels
        import collections
        import traceback
        from torch.utils._python_dispatch import TorchDispatchMode
        quiet = ("empty", "view", "as_strided", "_reshape_alias", "t.default", "transpose", "expand",
                 "slice", "select", "unsqueeze", "squeeze", "permute", "detach", "alias", "lift_fresh",
                 "unbind", "split", "narrow", "set_", "is_", "record_stream", "item",
                 "_local_scalar_dense", "resize_", "numpy_T")
        sites = collections.Counter()

        class _Sites(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                name = str(func)
                if not any(q in name for q in quiet):
                    st = [f for f in traceback.extract_stack()[:-1] if "commefficient_amd" in f.filename
                          or "bench_configs" in f.filename]
                    sites[(name, " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}"
                                             for f in reversed(st[-6:])))] += 1
                return func(*args, **(kwargs or {}))
        a0 = torch.cuda.memory_stats().get("num_device_alloc", 0)
        with _Sites():
            for i in range(b.warmup, b.warmup + min(2, b.steps)):
                fed(batches_at[i])
                fopt.step()
            torch.cuda.synchronize()
        if ctx.is_main:
            with open(ss, "w") as f:
                f.write(f"# device allocs in these 2 rounds: "
                        f"{torch.cuda.memory_stats().get('num_device_alloc', 0) - a0}\n")
                for (name, st), n in sites.most_common():
                    f.write(f"{n / 2:6.1f}/round {name} | {st}\n")
    ex = sum(n_ex)
    if ctx.is_main:
        print(json.dumps({"config": b.config, "n_gpus": N, "value": round(ex / el, 1),
                          "unit": unit, "ms_per_round": round(el / b.steps * 1e3, 2),
                          "clients_per_round": W, "examples_per_round": ex / b.steps,
                          "grad_size": fed.d, "loss_last": float(out[0].mean().item()),
                          "host_ms_per_round": round(host / b.steps * 1e3, 2),
                          # device allocations (hipMalloc) inside the timed rounds: each
                          # can synchronise the device
                          "device_allocs": torch.cuda.memory_stats().get("num_device_alloc", 0) - allocs0,
                          "dtype": args.dtype, "data": "synthetic",
                          "extra_flags": [x for x in b.extra if x != "--"]}), flush=True)
    if hasattr(loader, "close"):
        loader.close()
    dist.shutdown()


if __name__ == "__main__":
    main()
