"""Multi-process SPMD on CPU/gloo (world_size 2): the BASELINE.json "plumbing"
configuration.  Two ranks must end with bit-identical replicated weights that
equal a single-process run of the same rounds."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(rank, world, port, mode, out_dir, rounds, device="cpu"):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    if device == "cuda":  # ranks sharing one GPU: gloo (RCCL refuses duplicate devices)
        os.environ["COMMEFF_DIST_BACKEND"] = "gloo"
    torch.set_num_threads(2)
    from commefficient_amd import models
    from commefficient_amd.data import make_synthetic
    from commefficient_amd.data.device_loader import DeviceFedLoader
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.server import FedOptimizer
    from commefficient_amd.train.losses import cv_loss
    from commefficient_amd.utils.args import parse_args
    dist.init(device)
    extra = {"uncompressed": ["--local_momentum", "0", "--virtual_momentum", "0.9",
                              "--allreduce_bucket_mb", "0.01"],
             "sketch": ["--error_type", "virtual", "--local_momentum", "0", "--virtual_momentum",
                        "0.9", "--k", "300", "--num_rows", "3", "--num_cols", "2000"],
             "local_topk": ["--error_type", "local", "--local_momentum", "0.9", "--k", "300"],
             # (index, value) lists all-gathered instead of the dense all-reduce
             "local_topk_sparse": ["--error_type", "local", "--local_momentum", "0.9", "--k",
                                   "300", "--sparse_allgather", "on"],
             "fedavg": ["--local_momentum", "0", "--virtual_momentum", "0.5",
                        "--fedavg_batch_size", "2"],
             # the sharded server (reduce-scatter by region group) vs the
             # query-sharded one on a table of 9 groups
             "sketch_sharded": ["--error_type", "virtual", "--local_momentum", "0",
                                "--virtual_momentum", "0.9", "--k", "300", "--num_rows", "3",
                                "--num_cols", "20000", "--shard_unsketch", "on"],
             "sketch_query": ["--error_type", "virtual", "--local_momentum", "0",
                              "--virtual_momentum", "0.9", "--k", "300", "--num_rows", "3",
                              "--num_cols", "20000", "--shard_unsketch", "query"],
             # simulated client failures (same draw on every rank)
             "sketch_dropout": ["--error_type", "virtual", "--local_momentum", "0",
                                "--virtual_momentum", "0.9", "--k", "300", "--num_rows", "3",
                                "--num_cols", "2000", "--client_dropout", "0.5"],
             # one survivor: rank 1 computes nothing some rounds
             "uncompressed_dropout": ["--local_momentum", "0", "--virtual_momentum", "0.9",
                                      "--client_dropout", "0.95"]}[mode]
    lbs = "-1"
    base = mode.replace("_sparse", "").replace("_dropout", "").replace("_sharded", "").replace("_query", "")
    if device == "cuda":  # client rows in pinned host memory, compute on the GPU
        extra = extra + ["--client_state_device", "cpu"]
    args = parse_args(argv=["--mode", base, "--device", device, "--dtype", "fp32",
                            "--num_clients", "40", "--num_workers", "6", "--local_batch_size", lbs,
                            "--dataset_name", "CIFAR10", "--synthetic"] + extra, probe_port=False)
    torch.manual_seed(0)
    model = models.ResNet9(channels={"prep": 4, "layer1": 8, "layer2": 8, "layer3": 16})
    ds = make_synthetic("CIFAR10", train=True, num_clients=40, size=160, seed=3)
    loader = DeviceFedLoader(ds, 6, -1, device, seed=5, augment=True, out_bf16=False)
    model = model.to(device)
    fed = FedModel(model, cv_loss, args, num_clients=40)
    opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.05), args, fed)
    it = iter(loader)
    losses = []
    local = []
    for _ in range(rounds):
        try:
            b = next(it)
        except StopIteration:  # next epoch
            it = iter(loader)
            b = next(it)
        loss, acc, dl, ul = fed(b)
        opt.step()
        losses.append(loss.clone())
        local.append(fed.last_round["local_clients"])
    if mode.endswith("_sparse"):
        assert fed.last_round.get("sparse_allgather"), fed.last_round
    if mode == "sketch_sharded" and world > 1:
        assert fed.last_round.get("sharded_server"), fed.last_round
        assert fed.server.V.shape[0] == -(-9 // world)  # this rank's groups only
    if mode == "uncompressed" and world > 1:  # gradient buckets reduced during the backward
        assert fed.last_round.get("overlapped_buckets", 0) >= 2, fed.last_round
        assert fed.last_round.get("buckets_during_backward", 0) >= 1, fed.last_round
    if device == "cuda":
        assert fed.client_state.host_tier, "expected pinned host-tier client rows"
    sd = fed.server.state_dict()  # (sharded: gathered into the row-major format)
    torch.save({"w": fed.w.cpu(), "loss": torch.cat([l.reshape(-1) for l in losses]).cpu(),
                "dl": fed.accountant.client_download.cpu(), "V": sd["V"], "E": sd["E"],
                "local": torch.tensor(local), "migrated": fed.client_state.migrated},
               os.path.join(out_dir, f"r{rank}_w{world}.pt"))
    dist.shutdown()


@pytest.mark.parametrize("mode", ["uncompressed", "sketch", "local_topk", "local_topk_sparse",
                                  "fedavg", "sketch_dropout", "uncompressed_dropout"])
def test_gloo_two_ranks_match_single_process(mode):
    rounds = 3
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_run, args=(2, _free_port(), mode, d, rounds), nprocs=2,
                           start_method="spawn", join=True)
        mp.start_processes(_run, args=(1, _free_port(), mode, d, rounds), nprocs=1,
                           start_method="spawn", join=True)
        r0 = torch.load(os.path.join(d, "r0_w2.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "r1_w2.pt"), weights_only=True)
        s = torch.load(os.path.join(d, "r0_w1.pt"), weights_only=True)
    assert torch.equal(r0["w"], r1["w"]), "replicas diverged"
    torch.testing.assert_close(r0["w"], s["w"], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(r0["loss"], s["loss"], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(r0["dl"], s["dl"])


@pytest.mark.parametrize("world", [2])
def test_sharded_server_bitwise_equals_query_sharded(world):
    """The sharded FetchSGD server (tables reduce-scattered by region group,
    V / E / query / top-k per rank, packed k-lists merged in coordinate
    order) against the all-reduce + query-sharded server on the same 2 gloo
    ranks: the same sums, so bitwise the same weights, losses, accounting
    and server state (gathered back into the row-major format)."""
    rounds = 4
    with tempfile.TemporaryDirectory() as d:
        res = {}
        for mode in ("sketch_sharded", "sketch_query"):
            mp.start_processes(_run, args=(world, _free_port(), mode, d, rounds), nprocs=world,
                               start_method="spawn", join=True)
            res[mode] = [torch.load(os.path.join(d, f"r{r}_w{world}.pt"), weights_only=True)
                         for r in range(world)]
    a, b = res["sketch_sharded"], res["sketch_query"]
    for r in range(world):
        for key in ("w", "loss", "dl", "V", "E"):
            assert torch.equal(a[r][key], b[r][key]), (r, key)


def test_sharded_server_three_ranks_match_single_process():
    """3 ranks (9 groups, 3 per rank): replicas bitwise identical, and the
    same run as one process up to the collective's summation order (a ring
    all-reduce / reduce-scatter of 3 ranks adds in a position-dependent
    order, and the group-major payload puts a cell at another position than
    the row-major one -- so unlike 2 ranks, not bitwise the query path)."""
    rounds = 3
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_run, args=(3, _free_port(), "sketch_sharded", d, rounds), nprocs=3,
                           start_method="spawn", join=True)
        mp.start_processes(_run, args=(1, _free_port(), "sketch_sharded", d, rounds), nprocs=1,
                           start_method="spawn", join=True)
        rs = [torch.load(os.path.join(d, f"r{r}_w3.pt"), weights_only=True) for r in range(3)]
        s = torch.load(os.path.join(d, "r0_w1.pt"), weights_only=True)
    for r in (1, 2):
        assert torch.equal(rs[0]["w"], rs[r]["w"]) and torch.equal(rs[0]["V"], rs[r]["V"])
    torch.testing.assert_close(rs[0]["w"], s["w"], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rs[0]["loss"], s["loss"], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rs[0]["V"], s["V"], rtol=1e-3, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sketch", "true_topk"])
def test_two_ranks_one_gpu(mode):
    """The multi-rank GPU path (device tensors, native kernels, replicated
    server update) with two ranks sharing cuda:0 over gloo (RCCL refuses
    duplicate devices): replicas bit-identical, round-0 losses equal to the
    single-rank run, weights equal up to rare top-k near-tie flips."""
    import subprocess
    import sys
    worker = os.path.join(os.path.dirname(__file__), "dist_gpu_worker.py")
    rounds = 3
    env = dict(os.environ, COMMEFF_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    with tempfile.TemporaryDirectory() as d:
        for n in (2, 1):
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={n}", "--master-addr=127.0.0.1",
                   f"--master-port={_free_port()}", worker, d, mode, str(rounds)]
            subprocess.run(cmd, env=env, check=True, timeout=240)
        r0 = torch.load(os.path.join(d, "r0_w2.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "r1_w2.pt"), weights_only=True)
        s = torch.load(os.path.join(d, "r0_w1.pt"), weights_only=True)
    assert torch.equal(r0["w"], r1["w"]), "replicas diverged"
    assert torch.isfinite(r0["loss"]).all()
    dw = (r0["w"] - s["w"]).abs()
    print(f"round-0 loss max diff {(r0['loss'][0] - s['loss'][0]).abs().max().item():.3e}; "
          f"later rounds {(r0['loss'] - s['loss']).abs().max().item():.3e}; "
          f"|dw| max {dw.max().item():.3e}, frac > 1e-4 {(dw > 1e-4).float().mean().item():.3e}, "
          f"frac > 0 {(dw > 0).float().mean().item():.3e}")
    # round 0 runs at identical weights, and every example's forward is
    # computed the same way whatever the per-rank batch split (per-pixel
    # MFMA accumulation order, per-example head): identical per-client losses
    torch.testing.assert_close(r0["loss"][0], s["loss"][0], rtol=1e-6, atol=1e-7)
    # the weight gradient sums over a rank's examples first (fp32 reassociation,
    # ~1e-7 relative), so a top-k near-tie can flip: of the k = 5,000
    # coordinates updated per round, only a few may differ afterwards
    # (measured: 0-7.6e-5 of the coordinates beyond 1e-4, max |dw| 1.6e-4;
    # later-round losses 4-7e-6 apart)
    assert (dw > 1e-4).float().mean() < 5e-4, dw
    assert dw.max() < 1e-3, dw.max()
    torch.testing.assert_close(r0["loss"], s["loss"], rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_bench_two_ranks_one_gpu(scaling):
    """bench.py's multi-rank path (the driver's N>1 scaling run) end to end:
    two ranks over gloo sharing cuda:0, one JSON line from rank 0 with the
    whole-job throughput over both ranks' clients.  Strong scaling: a fixed
    41-client round split 21 / 20 across the ranks (fed_aggregator.py:230-237)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, COMMEFF_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    mode = ["--clients-per-gpu", "20"] if scaling == "weak" else ["--clients-per-round", "41"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "2",
           "--num-clients", "2000"] + mode
    res = subprocess.run(cmd, env=env, timeout=300, capture_output=True, text=True, cwd=root)
    assert res.returncode == 0, res.stderr[-4000:]
    out = res.stdout
    lines = [json.loads(x) for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out
    r = lines[0]
    W = 40 if scaling == "weak" else 41
    assert r["n_gpus"] == 2 and r["steps"] == 3 and r["warmup"] == 2
    assert r["scaling"] == scaling
    assert r["config"]["global_batch"] == W * 5 and r["config"]["parallelism"] == "dp2"
    assert r["config"]["clients_per_rank_max"] == (20 if scaling == "weak" else 21)
    assert r["value"] > 0 and abs(r["value"] - W * 5 * 1000 / r["ms_per_step"]) < 0.01 * r["value"]
    assert r["bytes_per_step"]["allreduce_payload_per_rank"] > 0


def _overlap_shadow_worker(rank, port, out_dir):
    os.environ.update({"RANK": "0", "WORLD_SIZE": "1", "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    import torch.distributed as tdist
    import torch.nn as nn
    from commefficient_amd.parallel.flat import FlatParams
    from commefficient_amd.parallel.overlap import OverlapReducer
    tdist.init_process_group("gloo", rank=0, world_size=1)
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(8, 16), nn.ReLU(), nn.Linear(16, 16), nn.ReLU(),
                          nn.Linear(16, 3))
    flat = FlatParams(model, "cpu")
    shadow = flat.make_bf16_shadow()
    x = torch.randn(5, 8)
    res = []
    for use_overlap in (False, True):
        flat.zero_grad()
        flat.refresh_shadow()
        red = OverlapReducer(flat, flat.shadow_params, 200, shadow=True) if use_overlap else None
        if red:
            red.arm()
        shadow(x.to(torch.bfloat16)).float().pow(2).sum().backward()
        if red:
            early = red.finish()
            red.remove()
            assert early >= 1 and len(red.buckets) >= 2
        else:
            flat.collect_shadow_grads()
        res.append(flat.g.clone())
    torch.save(res, os.path.join(out_dir, "ovl.pt"))
    tdist.destroy_process_group()


def test_overlap_reducer_moves_replica_grads():
    """The overlapped reducer's hooks on the bf16 replica gather exactly what
    collect_shadow_grads gathers (world 1: the all-reduce is the identity)."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_overlap_shadow_worker, args=(_free_port(), d), nprocs=1,
                           start_method="spawn", join=True)
        a, b = torch.load(os.path.join(d, "ovl.pt"), weights_only=True)
    assert a.abs().sum() > 0
    torch.testing.assert_close(a, b)


def test_client_state_ownership_balanced_three_ranks():
    """Per-client state (local error + momentum) on 3 gloo ranks: every round
    gives each rank W/3 +- 1 clients (balanced ownership, state.py assign; the
    reference chunks clients evenly, fed_aggregator.py:230-237), the moved
    clients' rows travel with them, and the run equals the single process."""
    rounds = 14  # 84 participations of 40 clients: returning clients must move
    mode = "local_topk"
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_run, args=(3, _free_port(), mode, d, rounds), nprocs=3,
                           start_method="spawn", join=True)
        mp.start_processes(_run, args=(1, _free_port(), mode, d, rounds), nprocs=1,
                           start_method="spawn", join=True)
        rs = [torch.load(os.path.join(d, f"r{r}_w3.pt"), weights_only=True) for r in range(3)]
        s = torch.load(os.path.join(d, "r0_w1.pt"), weights_only=True)
    counts = torch.stack([r["local"] for r in rs])  # [rank, round]
    assert (counts.max(0).values - counts.min(0).values <= 1).all(), counts
    assert rs[0]["migrated"] > 0, "the sampled rounds never needed a move (test too weak)"
    for r in rs[1:]:
        assert torch.equal(rs[0]["w"], r["w"]), "replicas diverged"
    torch.testing.assert_close(rs[0]["w"], s["w"], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rs[0]["loss"], s["loss"], rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_client_state_host_tier_migration_three_ranks_gpu():
    """The same 3-rank ownership run with CUDA compute and the client rows in
    pinned host memory (--client_state_device cpu) over gloo: a moved row is sent
    only after its last write-back (a non_blocking D2H copy on the compute stream)
    has landed (state.py _migrate), so the run equals the single GPU process."""
    import torch.cuda
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    rounds, mode = 14, "local_topk"
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_run, args=(3, _free_port(), mode, d, rounds, "cuda"), nprocs=3,
                           start_method="spawn", join=True)
        mp.start_processes(_run, args=(1, _free_port(), mode, d, rounds, "cuda"), nprocs=1,
                           start_method="spawn", join=True)
        rs = [torch.load(os.path.join(d, f"r{r}_w3.pt"), weights_only=True) for r in range(3)]
        s = torch.load(os.path.join(d, "r0_w1.pt"), weights_only=True)
    assert rs[0]["migrated"] > 0, "the sampled rounds never needed a move (test too weak)"
    for r in rs[1:]:
        assert torch.equal(rs[0]["w"], r["w"]), "replicas diverged"
    torch.testing.assert_close(rs[0]["w"], s["w"], rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(rs[0]["loss"], s["loss"], rtol=1e-3, atol=1e-4)


def _ckpt_worker(rank, world, port, out_dir, what):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(2)
    from commefficient_amd import models
    from commefficient_amd.data import make_synthetic
    from commefficient_amd.data.device_loader import DeviceFedLoader
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.server import FedOptimizer
    from commefficient_amd.train.cv import save_checkpoint
    from commefficient_amd.train.losses import cv_loss
    from commefficient_amd.utils.args import parse_args
    dist.init("cpu")
    argv = ["--mode", "sketch", "--device", "cpu", "--dtype", "fp32", "--num_clients", "40",
            "--num_workers", "6", "--local_batch_size", "-1", "--dataset_name", "CIFAR10",
            "--synthetic", "--error_type", "virtual", "--local_momentum", "0",
            "--virtual_momentum", "0.9", "--k", "300", "--num_rows", "3", "--num_cols", "20000",
            "--shard_unsketch", "on", "--checkpoint_path", os.path.join(out_dir, "ck_"),
            "--skip_nonfinite", "1"]
    args = parse_args(argv=argv, probe_port=False)
    torch.manual_seed(0)
    model = models.ResNet9(channels={"prep": 4, "layer1": 8, "layer2": 8, "layer3": 16})
    ds = make_synthetic("CIFAR10", train=True, num_clients=40, size=160, seed=3)
    loader = DeviceFedLoader(ds, 6, -1, "cpu", seed=5, augment=True)
    fed = FedModel(model, cv_loss, args, num_clients=40)
    opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.05), args, fed)
    assert fed.shard_server
    it = iter(loader)
    for r in range(3):
        fed(next(it))
        if what == "nonfinite" and r == 1 and rank == 1:
            # a NaN that lands in ONE rank's reduce-scattered groups only
            fed._pending[0].view(-1)[-1] = float("nan")
        opt.step()
    if what == "nonfinite":
        assert fed.skipped_rounds == 1, fed.skipped_rounds  # on EVERY rank
    else:
        save_checkpoint(fed, args, {"epoch": 0, "iter": 3})  # every rank calls it
    torch.save({"w": fed.w.clone(), "V": fed.server.state_dict()["V"]},
               os.path.join(out_dir, f"{what}_r{rank}.pt"))
    dist.shutdown()


def test_checkpoint_sharded_server_two_ranks():
    """save_checkpoint with the sharded server on 2 ranks: the gathers of V / E
    run on every rank (no hang) and the file holds the full row-major state."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_ckpt_worker, args=(2, _free_port(), d, "ckpt"), nprocs=2,
                           start_method="spawn", join=True)
        ck = torch.load(os.path.join(d, "ck_ResNet9.fedstate.pt"), weights_only=True)
        r0 = torch.load(os.path.join(d, "ckpt_r0.pt"), weights_only=True)
    assert ck["server"]["V"].shape == (3, 20000)
    assert torch.equal(ck["server"]["V"], r0["V"])
    assert torch.equal(ck["w"], r0["w"])


def test_skip_nonfinite_decided_globally_two_ranks():
    """A NaN in one rank's shard of the sharded server's table makes EVERY
    rank skip the round (an all-reduced flag), so the collectives stay paired
    and the replicas stay identical."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_ckpt_worker, args=(2, _free_port(), d, "nonfinite"), nprocs=2,
                           start_method="spawn", join=True)
        r0 = torch.load(os.path.join(d, "nonfinite_r0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "nonfinite_r1.pt"), weights_only=True)
    assert torch.equal(r0["w"], r1["w"])
    assert torch.isfinite(r0["w"]).all()
