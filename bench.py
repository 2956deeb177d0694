#!/usr/bin/env python
"""Headline benchmark (BASELINE.json): images/s + bytes/step of ResNet-9 on
CIFAR-10-shaped data with FetchSGD (Count Sketch, k=50,000, 5 x 500,000,
virtual momentum 0.9, virtual error, no local momentum) on 1/2/4/8 MI355X.

One "step" = one federated round: on-device batch assembly + augmentation,
forward/backward of this rank's clients (bf16), Count-Sketch encode, ONE RCCL
all-reduce of the 10 MB table (+ metrics), and the replicated server update
(momentum/error, median unsketch, top-k, heavy-hitter zeroing, weight apply,
download accounting).  Nothing is skipped in the timed region.

Weak scaling (default): every GPU runs --clients-per-gpu clients of
--client-size images per round (default 100 x 5 = 500 images/GPU/round;
10,000 non-iid clients of 5 images each as in the FetchSGD CIFAR-10 setup).
Strong scaling (--clients-per-round W): a fixed round of W clients in total,
split across the N ranks as the reference splits a round across its workers
(/root/reference/CommEfficient/fed_aggregator.py:230-237; balanced here, each
rank gets floor or ceil of W/N) -- the reference's own topology, e.g. W = 100
at N = 8 is 12-13 clients per rank.  Synthetic data of CIFAR shape, random-init
weights.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--clients-per-round W]
  N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

import commefficient_amd

METRIC = "images/sec + bytes/step, ResNet-9 CIFAR-10 FetchSGD at 1/2/4/8 MI355X"


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # 200 timed rounds after 50 warmup rounds (~0.5 s): 254.1-254.2k vs
    # 250.4-250.5k img/s with 30 after 5 on one box (clocks and caches settle)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--clients-per-gpu", type=int, default=100,
                   help="weak scaling: clients per rank per round (round = this x N)")
    p.add_argument("--clients-per-round", type=int, default=None,
                   help="strong scaling: total clients per round, split across the ranks "
                        "(fed_aggregator.py:230-237); overrides --clients-per-gpu")
    p.add_argument("--client-size", type=int, default=5)
    p.add_argument("--num-clients", type=int, default=10000)
    p.add_argument("--encode", default="region", choices=["region", "planned", "binned", "direct"],
                   help="sketch hash family / kernels (utils/args.py --encode)")
    p.add_argument("--conv", default="native", choices=["native", "miopen"],
                   help="3x3 conv units on the native MFMA kernels or on MIOpen")
    p.add_argument("--wgrad-stream", default="on", choices=["on", "off"],
                   help="weight gradients on a side stream (utils/args.py --wgrad_stream)")
    p.add_argument("--profile", action="store_true", help="per-phase HIP event timings")
    p.add_argument("--round-times", action="store_true",
                   help="HIP event per timed round; adds round_ms (GPU ms per round) to the JSON")
    p.add_argument("--torch-profile", default=None,
                   help="after the timed steps, trace 5 more with torch.profiler into this dir")
    p.add_argument("--miopen-find", type=int, default=int(os.environ.get("COMMEFF_MIOPEN_FIND", "0")),
                   help="torch.backends.cudnn.benchmark (ResNet-9 runs no MIOpen conv)")
    p.add_argument("--check-every", type=int, default=50,
                   help="cross-rank bitwise weight check every N rounds outside the timed "
                        "region (and once after it); exits non-zero on drift")
    b = p.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != b.gpus:
        sys.exit(f"--gpus {b.gpus} but WORLD_SIZE={world}: for --gpus > 1 launch with "
                 "torch.distributed.run --nproc-per-node N")
    from commefficient_amd.parallel import dist
    from commefficient_amd.utils.args import parse_args
    ctx = dist.init("cuda")
    N = ctx.world_size
    assert N == b.gpus, (N, b.gpus)
    # COMMEFF_DIST_BACKEND=gloo: the test suite's two-ranks-on-one-GPU rehearsal
    # of this script (tagged in the output); a real run is one rank per GPU on RCCL
    rehearsal = os.environ.get("COMMEFF_DIST_BACKEND") == "gloo"
    if N > 1 and not rehearsal:
        assert ctx.backend == "nccl", f"backend {ctx.backend!r}: the bench runs on RCCL"
        local = int(os.environ.get("LOCAL_WORLD_SIZE", str(N)))
        assert torch.cuda.device_count() >= local, "fewer visible GPUs than local ranks"
    strong = b.clients_per_round is not None
    W = b.clients_per_round if strong else b.clients_per_gpu * N
    if W < N:
        sys.exit(f"{W} clients per round cannot feed {N} ranks")
    n_train = b.num_clients * b.client_size
    argv = ["--dataset_name", "CIFAR10", "--synthetic", "--synthetic_size", str(n_train),
            "--mode", "sketch", "--error_type", "virtual", "--local_momentum", "0",
            "--virtual_momentum", "0.9", "--k", "50000", "--num_rows", "5", "--num_cols", "500000",
            "--num_blocks", "20", "--num_clients", str(b.num_clients), "--num_workers", str(W),
            "--local_batch_size", "-1", "--weight_decay", "5e-4", "--dtype", "bf16",
            "--device", "cuda", "--encode", b.encode, "--seed", "21",
            "--miopen_find", str(b.miopen_find), "--conv", b.conv, "--wgrad_stream", b.wgrad_stream]
    if b.profile:
        argv += ["--profile_dir", "gpurun_out/bench_profile"]
    args = parse_args(argv=argv, probe_port=False)

    from commefficient_amd import models
    from commefficient_amd.data import make_synthetic
    from commefficient_amd.data.device_loader import DeviceFedLoader
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.server import FedOptimizer
    from commefficient_amd.train.losses import cv_loss

    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    ds = make_synthetic("CIFAR10", train=True, num_clients=b.num_clients, size=n_train,
                        seed=args.seed)
    loader = DeviceFedLoader(ds, W, -1, ctx.device, seed=args.seed, augment=True, out_bf16=True)
    model = models.build_model(args, 10)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    fed = FedModel(model, cv_loss, args, num_clients=b.num_clients)
    fopt = FedOptimizer(opt, args, fed)
    if not b.profile:
        # per-round all-reduce time from HIP events (no syncs in the round)
        fed.timer.enable_only({"allreduce"})

    # pre-draw the rounds' client/row index arrays (host sampler), full rounds only
    rounds = []
    need = b.warmup + b.steps
    while len(rounds) < need:
        for r in loader.sampler:
            cids = ds.client_of(r)
            if len(np.unique(cids)) < W:
                continue
            rounds.append((cids, ds.data_index(r)))
            if len(rounds) >= need:
                break

    def step(i):
        cids, rows = rounds[i]
        out = fed(loader.make_batch(cids, rows))
        fopt.step()
        return out

    warm_host = []
    for i in range(b.warmup):
        h0 = time.perf_counter()
        out = step(i)
        warm_host.append(round((time.perf_counter() - h0) * 1000.0, 2))
        if b.check_every and N > 1 and (i + 1) % b.check_every == 0:
            dist.check_replicas(fed.w)
    # no host bookkeeping between the warmup and the timed rounds: the values
    # read afterwards are device snapshots taken here (no sync), so the GPU
    # idles only for the synchronize / barrier round trip (an idle GPU drops
    # its clock, and the first timed rounds then run slower)
    tw = time.perf_counter()  # end of the warmup enqueue
    # (plain copies: a reduction kernel used for the first time here would be
    # loaded from the code object now -- ~20 ms of GPU idle before the timed
    # rounds; the means / sums are taken after the timed region)
    first_loss_t = out[0].clone()
    dl_before_t = fed.accountant.client_download.clone()
    if fed.timer.enabled:
        fed.timer.discard()
    torch.cuda.synchronize()
    g0 = time.perf_counter()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gap_ms = (t0 - g0) * 1000.0
    host_s = 0.0  # host time spent enqueueing (no syncs inside a round)
    evs = []
    if b.round_times:
        evs.append(torch.cuda.Event(enable_timing=True))
        evs[-1].record()
    for i in range(b.warmup, b.warmup + b.steps):
        h0 = time.perf_counter()
        out = step(i)
        host_s += time.perf_counter() - h0
        if b.round_times:
            evs.append(torch.cuda.Event(enable_timing=True))
            evs[-1].record()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    elapsed = dist.max_over_ranks(t1 - t0)
    phases = fed.timer.summary() if fed.timer.enabled else {}
    checksum = None
    if b.check_every:
        # the replicated weights must be bitwise identical on every rank
        checksum = dist.check_replicas(fed.w)
    first_loss = float(first_loss_t.mean().item())
    last_loss = float(out[0].mean().item())
    dl = (float(fed.accountant.client_download.sum().item()) - float(dl_before_t.sum().item())) / b.steps
    if b.torch_profile:
        from torch.profiler import ProfilerActivity, profile
        stack = bool(os.environ.get("COMMEFF_PROF_STACK"))
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                     with_stack=stack) as prof:
            for i in range(b.warmup, b.warmup + min(b.steps, 5)):
                step(i)
            torch.cuda.synchronize()
        if ctx.is_main:
            os.makedirs(b.torch_profile, exist_ok=True)
            prof.export_chrome_trace(os.path.join(b.torch_profile, "bench_trace.json"))
            with open(os.path.join(b.torch_profile, "bench_ops.txt"), "w") as f:
                f.write(prof.key_averages().table(sort_by="cpu_time_total", row_limit=60))
                f.write("\n")
                f.write(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=60))
                if stack:
                    f.write("\n")
                    f.write(prof.key_averages(group_by_stack_n=8).table(
                        sort_by="self_cuda_time_total", row_limit=80))
    imgs_per_step = W * b.client_size
    ms = elapsed / b.steps * 1000.0
    value = imgs_per_step * b.steps / elapsed
    up_ref = fed.accountant.upload_per_client * W
    payload = fed.last_round.get("payload_bytes", 0)
    # ring-algorithm bytes each rank sends per round (all-reduce, or with the
    # sharded server reduce-scatter + metric all-reduce + k-list all-gather)
    wire = fed.last_round.get("wire_bytes", fed.accountant.wire_bytes_per_rank(payload // 4))
    if ctx.is_main:
        print(json.dumps({
            "metric": METRIC, "value": round(value, 1), "unit": "images/s", "n_gpus": N,
            "steps": b.steps, "warmup": b.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "strong" if strong else "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (CIFAR-10 shape, random-init ResNet-9)",
            "config": {"model": "ResNet9", "global_batch": imgs_per_step, "seq_len": None,
                       "image_hw": 32, "parallelism": f"dp{N}", "mode": "sketch",
                       "k": 50000, "num_rows": 5, "num_cols": 500000,
                       # numBlocks only shapes the csvec-layout hashes (--encode
                       # planned|binned|direct); the region family has no blocks
                       **({"num_blocks": 20} if b.encode != "region" else {}),
                       "clients_per_round": W, "clients_per_rank_max": -(-W // N),
                       "client_size": b.client_size,
                       "num_clients": b.num_clients, "encode": b.encode,
                       "server": ("sharded" if fed.shard_server else "replicated"),
                       "round_tape": bool(fed.last_round.get("taped"))},
            "bytes_per_step": {"upload_ref_accounting": up_ref,
                               "download_ref_accounting": dl,
                               "allreduce_payload_per_rank": payload,
                               "wire_per_rank_ring": wire},
            "loss_first": round(first_loss, 4), "loss_last": round(last_loss, 4),
            "phase_ms": {k: round(v, 3) for k, v in phases.items()},
            "backend": ctx.backend, "weights_checksum": checksum,
            **({"rehearsal": "gloo, ranks sharing one GPU"} if rehearsal and N > 1 else {}),
            "host_enqueue_ms_per_step": round(host_s / b.steps * 1000.0, 3),
            "barrier_before_timed_ms": round(gap_ms, 3),
            # host time from the last warmup enqueue to the first timed one
            # (includes the GPU draining the queued warmup rounds)
            "warmup_to_timed_ms": round((t0 - tw) * 1000.0, 3),
            "warmup_host_ms": warm_host,
            **({"round_ms": [round(evs[i].elapsed_time(evs[i + 1]), 3) for i in range(len(evs) - 1)]}
               if evs else {}),
        }), flush=True)
    dist.barrier()
    dist.shutdown()


if __name__ == "__main__":
    main()
