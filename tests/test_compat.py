"""The reference's helper API (commefficient_amd/compat.py) against the
engine's fused server update and plain-torch definitions."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from commefficient_amd import compat
from commefficient_amd.ops import CSVec
from commefficient_amd.parallel.server import ServerState
from commefficient_amd.utils.args import parse_args


def test_topk_dense_and_rows():
    g = torch.Generator().manual_seed(0)
    v = torch.randn(1000, generator=g)
    out = compat._topk(v, 10)
    keep = torch.topk(v.abs(), 10).indices
    ref = torch.zeros_like(v)
    ref[keep] = v[keep]
    assert torch.equal(out, ref)
    m = torch.randn(3, 50, generator=g)
    out2 = compat._topk(m, 4)
    assert ((out2 != 0).sum(1) == 4).all()


def test_grad_helpers_and_clip():
    model = nn.Linear(4, 3)
    args = parse_args(argv=["--device", "cpu", "--weight_decay", "0.5", "--num_workers", "2",
                            "--mode", "uncompressed"],
                      probe_port=False)
    model(torch.ones(2, 4)).sum().backward()
    g = compat.get_grad(model, args)
    ref = torch.cat([model.weight.grad.view(-1), model.bias.grad]) + 0.25 * torch.cat(
        [model.weight.data.view(-1), model.bias.data])
    torch.testing.assert_close(g, ref)
    compat.zero_grad(model)
    assert model.weight.grad.abs().sum() == 0
    x = torch.full((4,), 3.0)
    torch.testing.assert_close(compat.clip_grad(1.0, x).norm(), torch.tensor(1.0))
    assert compat.clip_grad(100.0, x) is x
    res = compat.split_results([(1.0, 2.0), (3.0, 4.0)], 2)
    assert np.array_equal(res[0], [1.0, 3.0]) and np.array_equal(res[1], [2.0, 4.0])
    assert isinstance(compat.shms(), list)


MODES = [("uncompressed", ["--virtual_momentum", "0.9", "--local_momentum", "0"]),
         ("true_topk", ["--virtual_momentum", "0.9", "--error_type", "virtual", "--k", "7",
                        "--local_momentum", "0"]),
         ("local_topk", ["--virtual_momentum", "0.5", "--error_type", "local", "--k", "7"]),
         ("fedavg", ["--virtual_momentum", "0.5", "--local_batch_size", "-1", "--local_momentum", "0"]),
         ("sketch", ["--virtual_momentum", "0.9", "--error_type", "virtual", "--k", "7",
                     "--local_momentum", "0", "--num_rows", "3", "--num_cols", "101",
                     "--num_blocks", "2"])]


@pytest.mark.parametrize("mode,extra", MODES)
def test_get_server_update_matches_engine(mode, extra):
    """Two steps of the reference-API update == the engine's fused update."""
    d = 300
    args = parse_args(argv=["--mode", mode, "--device", "cpu"] + extra, probe_port=False)
    args.grad_size = d
    lr = 1.0 if mode == "fedavg" else 0.3
    sk = CSVec(d, args.num_cols, args.num_rows, "cpu", args.num_blocks,
               seed=args.sketch_seed, kernel=args.encode) if mode == "sketch" else None
    eng = ServerState(args, d, "cpu", sk)
    shape = eng.V.shape
    V, E = torch.zeros(shape), torch.zeros(shape)
    w_eng = torch.randn(d, generator=torch.Generator().manual_seed(1))
    w_api = w_eng.clone()
    last_mod = torch.full((d,), -1, dtype=torch.int32)
    g = torch.Generator().manual_seed(2)
    for step in range(2):
        if mode == "sketch":
            s = sk.like()
            s.accumulateVec(torch.randn(d, generator=g))
            G = s.table.clone()
        else:
            G = torch.randn(d, generator=g)
        upd, V, E = compat.get_server_update(G.clone(), V, E, args, lr)
        w_api -= upd
        eng.update(G.clone(), lr, w_eng, last_mod, step)
    torch.testing.assert_close(w_api, w_eng, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(V, eng.V, rtol=1e-5, atol=1e-6)
