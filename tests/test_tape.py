"""Launch tapes (parallel/tape.py, csrc/launch.h, csrc/tape.cpp): a recorded
round replayed from C++ must give bitwise the eager round's results, and a
recording that contains a launch outside the tape must be refused."""
import numpy as np
import pytest
import torch


@pytest.mark.gpu
def test_tape_records_native_launches_and_refuses_foreign_kernels():
    from commefficient_amd import ops
    from commefficient_amd.parallel.tape import RoundTapes
    dev = torch.device("cuda", 0)
    t = torch.ones(1000, device=dev)
    u = torch.ones(10, device=dev)
    tapes = RoundTapes(dev)
    rep = tapes.record("native", lambda: ops.zero_(t))
    assert rep is not None
    torch.cuda.synchronize()
    assert t.sum().item() == 1000  # nothing executed while recording
    tapes.replay(rep)
    torch.cuda.synchronize()
    assert t.abs().sum().item() == 0
    t.fill_(2.0)
    tapes.replay(rep)
    torch.cuda.synchronize()
    assert t.abs().sum().item() == 0
    with pytest.warns(UserWarning, match="incomplete"):
        bad = tapes.record("foreign", lambda: (ops.zero_(t), u.add_(1.0)))
    assert bad is None and "foreign" in tapes.failed


@pytest.mark.gpu
def test_tape_side_lane_fork_join_replays():
    """A fork onto the side lane (ops/lanes.py) is recorded and replayed
    with event waits; the side work is ordered after the main work before it
    and the main work after the join waits for it."""
    from commefficient_amd import ops
    from commefficient_amd.ops import lanes
    from commefficient_amd.parallel.tape import RoundTapes
    from commefficient_amd._ext import ops as _ops
    dev = torch.device("cuda", 0)
    a = torch.ones(1 << 20, device=dev)
    b = torch.ones(1 << 20, device=dev)
    out = torch.zeros(4, device=dev)
    lanes.set_enabled(True)

    def body():
        ops.zero_(a)
        with lanes.fork(a):
            ops.zero_(b)
        lanes.join()
        ops.zero_(out)

    tapes = RoundTapes(dev)
    rep = tapes.record("lane", body)
    assert rep is not None and rep.side != 0
    assert sum(int(_ops().tape_forks(x)) for k, x in rep.segments if k == "tape") == 1
    torch.cuda.synchronize()
    assert a.sum().item() == a.numel() and b.sum().item() == b.numel()
    for _ in range(3):
        a.fill_(1.0)
        b.fill_(1.0)
        tapes.replay(rep)
        torch.cuda.synchronize()
        assert a.abs().sum().item() == 0 and b.abs().sum().item() == 0
    assert not lanes.pending()


def _bench_engine(mode: str, tape: str, W: int = 40, n: int = 5, more=()):
    from commefficient_amd import models
    from commefficient_amd.data import make_synthetic
    from commefficient_amd.data.device_loader import DeviceFedLoader
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.server import FedOptimizer
    from commefficient_amd.train.losses import cv_loss
    from commefficient_amd.utils.args import parse_args
    dist.init("cuda")
    extra = {"sketch": ["--error_type", "virtual", "--local_momentum", "0", "--virtual_momentum",
                        "0.9", "--k", "20000", "--num_rows", "5", "--num_cols", "200000"],
             "true_topk": ["--error_type", "virtual", "--local_momentum", "0",
                           "--virtual_momentum", "0.9", "--k", "20000"],
             "uncompressed": ["--local_momentum", "0", "--virtual_momentum", "0.9"]}[mode]
    args = parse_args(argv=["--dataset_name", "CIFAR10", "--synthetic", "--synthetic_size", "2000",
                            "--mode", mode, "--num_clients", "400", "--num_workers", str(W),
                            "--local_batch_size", "-1", "--weight_decay", "5e-4", "--dtype", "bf16",
                            "--device", "cuda", "--seed", "21", "--round_tape", tape] + extra + list(more),
                      probe_port=False)
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    ds = make_synthetic("CIFAR10", train=True, num_clients=400, size=2000, seed=args.seed)
    loader = DeviceFedLoader(ds, W, -1, "cuda", seed=args.seed, augment=True, out_bf16=True)
    model = models.build_model(args, 10)
    fed = FedModel(model, cv_loss, args, num_clients=400)
    opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1), args, fed)
    return fed, opt, loader, ds, W


def _run(fed, opt, loader, ds, W, rounds):
    losses, dls = [], []
    it = iter(loader.sampler)
    done = 0
    while done < rounds:
        r = next(it)
        cids = ds.client_of(r)
        if len(np.unique(cids)) < W:
            continue
        out = fed(loader.make_batch(cids, ds.data_index(r)))
        opt.param_groups[0]["lr"] = 0.1 * (1 + done % 3)  # a changing LR reaches the replay
        opt.step()
        losses.append(out[0].clone())
        dls.append(out[2].clone())
        done += 1
    torch.cuda.synchronize()
    return torch.stack(losses), torch.stack(dls)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sketch", "true_topk", "uncompressed"])
def test_taped_rounds_bitwise_equal_eager(mode):
    rounds = 7
    res = {}
    # eager / taped, and taped without the conv weight gradients' side lane
    for tape, more in (("off", ()), ("auto", ()), ("auto1", ("--wgrad_stream", "off"))):
        fed, opt, loader, ds, W = _bench_engine(mode, tape[:4], more=more)
        losses, dls = _run(fed, opt, loader, ds, W, rounds)
        res[tape] = (fed.w.clone(), losses, dls, fed.accountant.last_mod.clone(), fed.server.V.clone())
        if tape != "off":
            assert fed.last_round.get("taped"), (fed.last_round, fed._tapes.last_counts)
            assert fed._tapes.replays >= 2 * (rounds - 2), fed._tapes.replays
    for other in ("auto", "auto1"):
        for a, b in zip(res["off"], res[other]):
            assert torch.equal(a, b), (other, (a - b).abs().max())
