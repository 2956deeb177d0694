"""One rank of a multi-process run launched by torch.distributed.run
(tests/test_rccl.py): a few federated rounds in one mode, then a bitwise
cross-rank check of the replicated weights (dist.check_replicas raises on
drift -> non-zero exit) and the rank's results saved for comparison with the
single-process run.  On GPUs the backend is RCCL (one distinct GPU per rank);
``cpu`` runs the same code over gloo (the rehearsal in this container).

usage: rccl_worker.py OUT_DIR MODE ROUNDS {cuda,cpu}
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# per mode: reference flags + the multi-rank feature it exercises
MODES = {
    # sketch all-reduce + sharded unsketch (per-rank query shard, k-list all-gather)
    "sketch": ["--mode", "sketch", "--error_type", "virtual", "--local_momentum", "0",
               "--virtual_momentum", "0.9", "--k", "5000", "--num_rows", "5",
               "--num_cols", "50000", "--shard_unsketch", "on"],
    "true_topk": ["--mode", "true_topk", "--error_type", "virtual", "--local_momentum", "0",
                  "--virtual_momentum", "0.9", "--k", "5000"],
    # per-client local top-k lists all-gathered instead of a dense all-reduce
    "local_topk_sparse": ["--mode", "local_topk", "--error_type", "local",
                          "--local_momentum", "0.9", "--virtual_momentum", "0", "--k", "2000",
                          "--sparse_allgather", "on"],
    # dense gradient buckets all-reduced during the backward
    "uncompressed_overlap": ["--mode", "uncompressed", "--error_type", "none",
                             "--local_momentum", "0", "--virtual_momentum", "0.9",
                             "--overlap_allreduce", "on", "--allreduce_bucket_mb", "4"],
}


def main(out_dir, mode, rounds, device):
    from commefficient_amd import models
    from commefficient_amd.data import make_synthetic
    from commefficient_amd.data.device_loader import DeviceFedLoader
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.server import FedOptimizer
    from commefficient_amd.train.losses import cv_loss
    from commefficient_amd.utils.args import parse_args
    if device == "cpu":
        torch.set_num_threads(2)
    ctx = dist.init(device)
    if device == "cuda" and ctx.world_size > 1:
        # one distinct GPU per rank over RCCL: never a gloo or shared-GPU fallback
        assert ctx.backend == "nccl", ctx.backend
        assert torch.cuda.device_count() >= ctx.world_size
        assert ctx.device.index == ctx.local_rank
    W = 16
    extra = list(MODES[mode])
    if device == "cpu" and "--allreduce_bucket_mb" in extra:
        extra[extra.index("--allreduce_bucket_mb") + 1] = "0.01"  # the small CPU model
    args = parse_args(argv=["--device", device, "--dtype", "bf16" if device == "cuda" else "fp32",
                            "--num_clients", "80", "--num_workers", str(W), "--local_batch_size",
                            "-1", "--dataset_name", "CIFAR10", "--synthetic"] + extra,
                      probe_port=False)
    torch.manual_seed(0)
    if device == "cuda":
        model = models.build_model(args, 10)
    else:
        model = models.ResNet9(channels={"prep": 4, "layer1": 8, "layer2": 8, "layer3": 16})
    ds = make_synthetic("CIFAR10", train=True, num_clients=80, size=800, seed=3)
    loader = DeviceFedLoader(ds, W, -1, ctx.device, seed=5, augment=True,
                             out_bf16=device == "cuda")
    fed = FedModel(model, cv_loss, args, num_clients=80)
    opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.05), args, fed)
    it = iter(loader)
    losses = []
    for _ in range(rounds):
        loss, acc, dl, ul = fed(next(it))
        opt.step()
        losses.append(loss.clone())
    if device == "cuda":
        torch.cuda.synchronize()
    checksum = dist.check_replicas(fed.w)  # raises if any rank drifted
    info = dict(fed.last_round)
    if ctx.world_size > 1:
        if mode == "local_topk_sparse":
            assert info.get("sparse_allgather"), info
        if mode == "uncompressed_overlap":
            assert info.get("overlapped_buckets", 0) >= 2, info
            # the native wgrad kernels announce their in-place writes
            # (ops.nn._grad_written): buckets go out during the backward
            assert info.get("buckets_during_backward", 0) >= 1, info
    torch.save({"w": fed.w.cpu(), "loss": torch.stack(losses).cpu(), "checksum": checksum,
                "dl": fed.accountant.client_download.cpu()},
               os.path.join(out_dir, f"{mode}_r{ctx.rank}_w{ctx.world_size}.pt"))
    dist.barrier()
    dist.shutdown()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4] if len(sys.argv) > 4 else "cuda")
