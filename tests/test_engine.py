"""End-to-end engine semantics on CPU against the numpy oracle of all five
modes (tests/engine_oracle.py), merged-vs-per-client exactness, byte
accounting and checkpoint round trips."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from commefficient_amd.parallel import dist
from commefficient_amd.parallel.fed_model import FedModel
from commefficient_amd.parallel.server import FedOptimizer
from commefficient_amd.utils.args import parse_args
from engine_oracle import LinearFedOracle


def lin_loss(model, inputs, targets, args):
    pred = model(*inputs).squeeze(-1)
    return (pred - targets) ** 2, [torch.zeros_like(targets)]


def make_engine(d, argv, num_clients, lr):
    dist.init("cpu")
    args = parse_args(argv=argv + ["--device", "cpu", "--num_clients", str(num_clients),
                                   "--dtype", "fp32"], probe_port=False)
    model = nn.Linear(d, 1, bias=False)
    nn.init.zeros_(model.weight)
    fed = FedModel(model, lin_loss, args, num_clients=num_clients)
    opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=lr), args, fed)
    return fed, opt, args


def data(N, d):
    X = torch.arange(N * d, dtype=torch.float32).view(N, d) / (N * d)
    y = torch.arange(N, dtype=torch.float32) / N
    return X, y


def split(N, W):
    cids = torch.zeros(N, dtype=torch.int64)
    for i in range(W):
        cids[i * N // W:(i + 1) * N // W] = i
    return cids


CASES = [
    # mode, extra argv, oracle kwargs
    ("uncompressed", ["--virtual_momentum", "0.9", "--local_momentum", "0"],
     dict(rho=0.9)),
    ("uncompressed", ["--virtual_momentum", "0", "--local_momentum", "0.5"],
     dict(rho_l=0.5)),
    ("true_topk", ["--error_type", "virtual", "--virtual_momentum", "0.9", "--local_momentum", "0",
                   "--k", "2"], dict(rho=0.9, k=2, error_type="virtual")),
    ("true_topk", ["--error_type", "virtual", "--virtual_momentum", "0", "--local_momentum", "0.9",
                   "--k", "1"], dict(rho_l=0.9, k=1, error_type="virtual")),
    ("local_topk", ["--error_type", "local", "--virtual_momentum", "0.5", "--local_momentum", "0.9",
                    "--k", "2"], dict(rho=0.5, rho_l=0.9, k=2, error_type="local")),
    ("local_topk", ["--error_type", "none", "--virtual_momentum", "0", "--local_momentum", "0",
                    "--k", "1"], dict(k=1)),
    ("fedavg", ["--virtual_momentum", "0.9", "--local_momentum", "0", "--local_batch_size", "-1",
                "--fedavg_batch_size", "2", "--num_fedavg_epochs", "2"],
     dict(rho=0.9, fedavg_epochs=2, fedavg_bs=2)),
    # one full-batch local step: takes the merged (linear) path
    ("fedavg", ["--virtual_momentum", "0.5", "--local_momentum", "0", "--local_batch_size", "-1"],
     dict(rho=0.5)),
    ("sketch", ["--error_type", "virtual", "--virtual_momentum", "0.9", "--local_momentum", "0",
                "--k", "2", "--num_rows", "1", "--num_cols", "100003", "--num_blocks", "1"],
     dict(rho=0.9, k=2, error_type="virtual")),
]


@pytest.mark.parametrize("W", [1, 2])
@pytest.mark.parametrize("wd", [0.0, 5e-3])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_modes_match_numpy_oracle(case, W, wd):
    mode, extra, okw = CASES[case]
    N, d, lr = 8, 4, 0.3
    argv = ["--mode", mode, "--num_workers", str(W), "--weight_decay", str(wd)] + extra
    if mode != "fedavg":
        argv += ["--local_batch_size", str(N // W)]
    fed, opt, args = make_engine(d, argv, W, lr)
    omode = "sketch_exact" if mode == "sketch" else mode
    orc = LinearFedOracle(d, omode, wd=wd, num_workers=W, **okw)
    X, y = data(N, d)
    cids = split(N, W)
    clients = [(i, X[cids == i].double().numpy(), y[cids == i].double().numpy()) for i in range(W)]
    for rnd in range(4):
        fed((cids, X, y))
        opt.param_groups[0]["lr"] = lr
        opt.step()
        w_exp = orc.round(clients, lr)
        np.testing.assert_allclose(fed.w.double().numpy(), w_exp, rtol=2e-4, atol=2e-6,
                                   err_msg=f"round {rnd}")


EXTRA_CASES = [
    ("uncompressed", ["--topk_down", "--k", "2", "--local_momentum", "0",
                      "--virtual_momentum", "0.5"], dict(topk_down=True, k=2, rho=0.5)),
    ("local_topk", ["--topk_down", "--k", "2", "--error_type", "local", "--local_momentum", "0"],
     dict(topk_down=True, k=2, error_type="local")),
    ("uncompressed", ["--max_grad_norm", "0.05", "--local_momentum", "0"],
     dict(max_grad_norm=0.05)),
    ("true_topk", ["--dp", "--l2_norm_clip", "0.02", "--noise_multiplier", "0",
                   "--error_type", "virtual", "--local_momentum", "0", "--k", "2"],
     dict(dp_clip=0.02, k=2, error_type="virtual")),
    ("uncompressed", ["--microbatch_size", "1", "--local_momentum", "0"], dict()),
]


@pytest.mark.parametrize("W", [1, 2])
@pytest.mark.parametrize("case", range(len(EXTRA_CASES)))
def test_client_side_options_match_oracle(case, W):
    mode, extra, okw = EXTRA_CASES[case]
    N, d, lr, wd = 8, 4, 0.3, 5e-3
    argv = ["--mode", mode, "--num_workers", str(W), "--weight_decay", str(wd),
            "--local_batch_size", str(N // W)] + extra
    fed, opt, args = make_engine(d, argv, W, lr)
    orc = LinearFedOracle(d, mode, wd=wd, num_workers=W, **okw)
    X, y = data(N, d)
    cids = split(N, W)
    clients = [(i, X[cids == i].double().numpy(), y[cids == i].double().numpy()) for i in range(W)]
    for rnd in range(4):
        fed((cids, X, y))
        opt.step()
        w_exp = orc.round(clients, lr)
        np.testing.assert_allclose(fed.w.double().numpy(), w_exp, rtol=2e-4, atol=2e-6,
                                   err_msg=f"round {rnd}")


def test_reference_linear_scenario_first_steps():
    """The unit_test.py:185 scenario (N=4, d=1, one worker, lr 0.005,
    X=arange, y=arange, squared error) re-derived for mean-gradient
    semantics: w1 = 0.005*7 = 0.035, w2 = w1 + 0.005*(2*(14 - 14*w1))/4."""
    fed, opt, _ = make_engine(1, ["--mode", "uncompressed", "--local_momentum", "0",
                                  "--virtual_momentum", "0", "--weight_decay", "0",
                                  "--num_workers", "1", "--local_batch_size", "4"], 1, 0.005)
    X = torch.arange(4, dtype=torch.float32).view(4, 1)
    y = torch.arange(4, dtype=torch.float32)
    cids = torch.zeros(4, dtype=torch.int64)
    fed((cids, X, y))
    opt.step()
    assert abs(fed.w.item() - 0.035) < 1e-7
    fed((cids, X, y))
    opt.step()
    w1 = 0.035
    assert abs(fed.w.item() - (w1 + 0.005 * 2 * (14 - 14 * w1) / 4)) < 1e-6


@pytest.mark.parametrize("mode", ["uncompressed", "true_topk", "sketch"])
def test_merged_equals_per_client(mode):
    """Merging a rank's clients into one forward/backward is exact."""
    from commefficient_amd import models
    from commefficient_amd.train.losses import cv_loss
    dist.init("cpu")
    outs = []
    for merge in ("on", "off"):
        torch.manual_seed(0)
        argv = ["--mode", mode, "--local_momentum", "0", "--virtual_momentum", "0.9",
                "--error_type", "virtual" if mode != "uncompressed" else "none", "--k", "500",
                "--num_rows", "3", "--num_cols", "4000", "--num_workers", "4",
                "--local_batch_size", "3", "--device", "cpu", "--dtype", "fp32",
                "--num_clients", "4", "--merge_clients", merge, "--weight_decay", "5e-4"]
        args = parse_args(argv=argv, probe_port=False)
        model = models.ResNet9(channels={"prep": 4, "layer1": 8, "layer2": 8, "layer3": 16})
        fed = FedModel(model, cv_loss, args, num_clients=4)
        opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1), args, fed)
        g = torch.Generator().manual_seed(1)
        X = torch.randn(12, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (12,), generator=g)
        cids = torch.tensor([0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3])
        res = fed((cids, X, y))
        opt.step()
        outs.append((fed.w.clone(), res[0].clone()))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-5, atol=1e-6)


def test_byte_accounting_matches_reference_formulas():
    fed, opt, args = make_engine(4, ["--mode", "true_topk", "--error_type", "virtual",
                                     "--local_momentum", "0", "--k", "1", "--num_workers", "2",
                                     "--local_batch_size", "2"], 4, 0.3)
    X, y = data(8, 4)
    # round 0: clients 0,1 (never seen anything changed) -> 0 download
    cids = torch.tensor([0, 0, 1, 1, 0, 0, 1, 1])
    _, _, dl, ul = fed((cids, X, y))
    opt.step()
    assert dl.tolist() == [0.0, 0.0]
    assert ul == 2 * 4 * 4  # 4 bytes * d per client in true_topk
    # round 1: clients 1,2. client 1 saw round 0's weights: 1 coord changed since;
    # client 2 starts from the initial weights: same 1 coord
    cids = torch.tensor([1, 1, 2, 2, 1, 1, 2, 2])
    _, _, dl, _ = fed((cids, X, y))
    opt.step()
    assert dl.tolist() == [4.0, 4.0]
    # round 2: client 0 last saw round 0 -> changes of rounds 0 and 1 (1 or 2 coords)
    cids = torch.tensor([0, 0, 3, 3, 0, 0, 3, 3])
    _, _, dl, _ = fed((cids, X, y))
    changed = int((fed.w != 0).sum())
    assert dl.tolist() == [4.0 * changed, 4.0 * changed]


def test_checkpoint_state_dict_format(tmp_path):
    from commefficient_amd import models
    m = models.ResNet9()
    keys = list(m.state_dict().keys())
    assert keys[0] == "n.prep.conv.weight" and keys[-1] == "n.linear.weight"
    fed, opt, args = make_engine(3, ["--mode", "uncompressed", "--local_momentum", "0",
                                     "--num_workers", "1", "--local_batch_size", "2"], 1, 0.1)
    X, y = data(2, 3)
    fed((torch.zeros(2, dtype=torch.int64), X, y))
    opt.step()
    p = tmp_path / "ckpt.pt"
    torch.save(fed.state_dict(), p)
    sd = torch.load(p, weights_only=True)
    torch.testing.assert_close(sd["weight"].view(-1), fed.w)
    fs = fed.fed_state_dict()
    torch.save(fs, tmp_path / "f.pt")
    fs2 = torch.load(tmp_path / "f.pt", weights_only=True)
    fed2, _, _ = make_engine(3, ["--mode", "uncompressed", "--local_momentum", "0",
                                 "--num_workers", "1", "--local_batch_size", "2"], 1, 0.1)
    fed2.load_fed_state_dict(fs2)
    torch.testing.assert_close(fed2.w, fed.w)
    assert fed2.round_idx == 1


def test_fedavg_hack_step_sets_lr_without_pending_round():
    """cv_train.py:198-203 'HACK STEP': with no round pending, FedOptimizer.step
    still writes g_lr (fed_aggregator.py:441-444).  When the schedule reaches
    lr=0, the next round's local SGD must run at lr 0 (no weight change apart
    from the server momentum V)."""
    fed, opt, args = make_engine(4, ["--mode", "fedavg", "--virtual_momentum", "0",
                                     "--local_momentum", "0", "--local_batch_size", "-1",
                                     "--num_workers", "2"], 2, 0.3)
    X, y = data(8, 4)
    cids = split(8, 2)
    opt.step()  # hack step before the first round: sets the LR only
    assert fed.fedavg_lr == pytest.approx(0.3)
    fed((cids, X, y))
    opt.step()
    w1 = fed.w.clone()
    assert (w1 != 0).any()
    opt.param_groups[0]["lr"] = 0.0
    opt.step()  # no round pending: hack step with lr 0
    assert fed.fedavg_lr == 0.0
    fed((cids, X, y))
    opt.step()
    torch.testing.assert_close(fed.w, w1)


def test_client_dropout_equals_round_of_survivors():
    """--client_dropout removes whole clients before the round: the update
    equals a dropout-free round over the surviving clients' examples."""
    N, d, W = 24, 6, 6
    X, y = data(N, d)
    cids = split(N, W)
    argv = ["--mode", "uncompressed", "--virtual_momentum", "0.9", "--local_momentum", "0",
            "--num_workers", str(W), "--local_batch_size", "-1", "--weight_decay", "0"]
    fa, oa, _ = make_engine(d, argv + ["--client_dropout", "0.5"], W, 0.1)
    out_a = fa((cids, X, y))
    oa.step()
    dropped = fa.last_round.get("dropped_clients", 0)
    assert 0 < dropped < W
    # the survivors of round 0, drawn as the engine does
    rng = np.random.default_rng([int(fa.args.seed), 0, 0x0D40])
    keep_c = np.arange(W)[rng.random(W) >= 0.5]
    assert len(keep_c) == W - dropped
    keep = np.isin(cids.numpy(), keep_c)
    fb, ob, _ = make_engine(d, argv, W, 0.1)
    out_b = fb((cids[keep], X[keep], y[keep]))
    ob.step()
    torch.testing.assert_close(fa.w, fb.w)
    assert len(out_a[0]) == len(keep_c) == len(out_b[0])
    # accounting: only the survivors downloaded / uploaded
    assert (fa.accountant.client_upload > 0).sum().item() == len(keep_c)


def test_nonfinite_round_skipped_and_injected():
    """Fault injection corrupts round 1's aggregate; with --skip_nonfinite the
    server drops that round (weights, V unchanged) and training goes on;
    without it the NaN reaches the weights (the reference's behaviour: the
    driver then stops on the NaN loss)."""
    N, d, W = 12, 5, 3
    X, y = data(N, d)
    cids = split(N, W)
    argv = ["--mode", "uncompressed", "--virtual_momentum", "0.9", "--local_momentum", "0",
            "--num_workers", str(W), "--local_batch_size", "-1", "--inject_nonfinite_round", "1"]
    fa, oa, _ = make_engine(d, argv + ["--skip_nonfinite", "1"], W, 0.1)
    fa((cids, X, y)); oa.step()
    w0, V0 = fa.w.clone(), fa.server.V.clone()
    fa((cids, X, y)); oa.step()
    assert fa.skipped_rounds == 1 and fa.last_round.get("skipped_nonfinite")
    assert torch.equal(fa.w, w0) and torch.equal(fa.server.V, V0)
    fa((cids, X, y)); oa.step()
    assert torch.isfinite(fa.w).all() and not torch.equal(fa.w, w0)
    fb, ob, _ = make_engine(d, argv, W, 0.1)
    for _ in range(2):
        fb((cids, X, y)); ob.step()
    assert fb.skipped_rounds == 0 and not torch.isfinite(fb.w).all()


def _ref_scenario(d, W, k, r, c, lr=0.005):
    """Two FetchSGD rounds of the unit_test.py:23-26 linear problem (X =
    arange(4d).view(4, d), y = arange(4), squared error, w0 = 0, momentum 0,
    virtual error) on ``W`` clients with an r x c sketch."""
    argv = ["--mode", "sketch", "--error_type", "virtual", "--virtual_momentum", "0",
            "--local_momentum", "0", "--weight_decay", "0", "--k", str(k), "--num_rows", str(r),
            "--num_cols", str(c), "--num_blocks", "1", "--num_workers", str(W),
            "--local_batch_size", str(4 // W)]
    fed, opt, _ = make_engine(d, argv, W, lr)
    X = torch.arange(4 * d, dtype=torch.float32).view(4, d)
    y = torch.arange(4, dtype=torch.float32)
    cids = split(4, W)
    ws = []
    for _ in range(2):
        fed((cids, X, y))
        opt.param_groups[0]["lr"] = lr
        opt.step()
        ws.append(fed.w.double().numpy().copy())
    return ws, X.double().numpy(), y.double().numpy()


def _G(w, X, y):
    """Round gradient = mean over the round's examples of d/dw (x.w - y)^2
    (each client's mean gradient weighted n_i / B)."""
    return 2.0 * X.T @ (X @ w - y) / len(y)


@pytest.mark.parametrize("W", [1, 2])
def test_reference_oracle_one_weight_tiny_sketch(W):
    """unit_test.py:185-186 (d=1, k=1, 1x1 sketch, 1 or 2 workers): one
    coordinate, so the sketch estimate s*s*g is exact and every round is a
    plain gradient step.  Re-derived: G(0) = -7 -> w1 = 0.035;
    G(w1) = 7 w1 - 7 -> w2 = w1 + 0.005 (7 - 7 w1) = 0.068775."""
    (w1, w2), X, y = _ref_scenario(1, W, 1, 1, 1)
    np.testing.assert_allclose(w1, [0.035], rtol=1e-6)
    np.testing.assert_allclose(w2, [0.068775], rtol=1e-6)


@pytest.mark.parametrize("W", [1, 2])
def test_reference_oracle_two_weights_large_sketch(W):
    """unit_test.py:187,191 (d=2, k=2, 9x1000 sketch, 1 or 2 workers): the
    median of 9 rows recovers both coordinates exactly and k = d, so two
    plain gradient steps: G(0) = (-14, -17) -> w1 = (0.07, 0.085)."""
    (w1, w2), X, y = _ref_scenario(2, W, 2, 9, 1000)
    e1 = -0.005 * _G(np.zeros(2), X, y)
    np.testing.assert_allclose(e1, [0.07, 0.085], rtol=1e-12)
    e2 = e1 - 0.005 * _G(e1, X, y)
    np.testing.assert_allclose(w1, e1, rtol=1e-6)
    np.testing.assert_allclose(w2, e2, rtol=1e-6)


def test_reference_oracle_two_weights_one_bucket():
    """unit_test.py:188-190 (d=2, k=2, 1x1 sketch): both coordinates share
    the single bucket, table = s0 g0 + s1 g1 and est_i = s_i * table, so the
    update is (g0+g1, g0+g1) when the signs agree and (g0-g1, g1-g0) when
    they differ (the reference's three admissible w1).  Both are selected
    (k = d) and heavy-hitter zeroing clears the bucket, so round 2 repeats
    the construction at w1 with the same signs."""
    (w1, w2), X, y = _ref_scenario(2, 1, 2, 1, 1)
    lr = 0.005

    def step(w, same):
        g = _G(w, X, y)
        t = g[0] + g[1] if same else g[0] - g[1]
        return w - lr * (np.array([t, t]) if same else np.array([t, -t]))

    opts = {same: step(np.zeros(2), same) for same in (True, False)}
    same = [s for s, e in opts.items() if np.allclose(w1, e, rtol=1e-6)]
    assert same, (w1, opts)
    np.testing.assert_allclose(w2, step(opts[same[0]], same[0]), rtol=1e-6)


def test_reference_oracle_two_workers_top1():
    """unit_test.py:192 (d=2, W=2, k=1, 9x1000 sketch): exact estimates but
    only the largest coordinate moves; the other stays in the virtual error
    and is added to the next round's gradient before the next top-1."""
    (w1, w2), X, y = _ref_scenario(2, 2, 1, 9, 1000)
    lr = 0.005
    g0 = _G(np.zeros(2), X, y)            # (-14, -17): coordinate 1 wins
    i = int(np.argmax(np.abs(g0)))
    e1 = np.zeros(2)
    e1[i] = -lr * g0[i]
    err = g0.copy()
    err[i] = 0.0                          # E[nz] = 0
    est = err + _G(e1, X, y)              # E += V (momentum 0: V = S)
    j = int(np.argmax(np.abs(est)))
    e2 = e1.copy()
    e2[j] -= lr * est[j]
    np.testing.assert_allclose(w1, e1, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(w2, e2, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
def test_host_tier_client_state_prefetch_matches_device_tier():
    """Per-client state in host memory (--client_state_device cpu) with the
    round's next clients prefetched on a side stream gives the device-resident
    run (local momentum + local error, local top-k).  The fp32 convolutions
    are not bitwise reproducible run to run (MIOpen algorithm choice), so the
    tiers are compared at a tolerance far below what one stale prefetched row
    (a client's state missing its previous round) moves the weights by."""
    import copy
    from commefficient_amd import models
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.server import FedOptimizer
    from commefficient_amd.train.losses import cv_loss
    from commefficient_amd.utils.args import parse_args
    dist.init("cuda")
    torch.manual_seed(0)
    base = models.ResNet9(channels={"prep": 16, "layer1": 32, "layer2": 32, "layer3": 64})
    res = {}
    for where in ("gpu", "cpu"):
        args = parse_args(argv=["--dataset_name", "CIFAR10", "--mode", "local_topk", "--error_type", "local",
                                "--local_momentum", "0.9", "--virtual_momentum", "0", "--k", "500",
                                "--num_workers", "6", "--num_clients", "12", "--local_batch_size", "-1",
                                "--device", "cuda", "--dtype", "fp32", "--client_state_device", where,
                                "--client_prefetch", "2"], probe_port=False)
        model = copy.deepcopy(base).cuda()
        fed = FedModel(model, cv_loss, args, num_clients=12)
        assert fed.client_state.host_tier == (where == "cpu")
        opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.05), args, fed)
        g = torch.Generator().manual_seed(3)
        for r in range(4):
            x = torch.randn(24, 3, 32, 32, generator=g).cuda()
            y = torch.randint(0, 10, (24,), generator=g).cuda()
            cids = torch.arange(6).repeat_interleave(4) + 6 * (r % 2)
            fed((cids, x, y))
            opt.step()
        torch.cuda.synchronize()
        res[where] = fed.w.clone()
    torch.testing.assert_close(res["cpu"], res["gpu"], rtol=1e-4, atol=2e-6)
