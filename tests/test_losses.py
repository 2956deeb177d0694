"""Loss-function parity: the GPT-2 train loss reproduces the reference's HF
lm_loss -- ONE token-weighted mean over all labelled tokens of a client's batch
(gpt2_train.py:88-99) -- both per client and in a merged multi-client batch."""
import pytest
import torch
import torch.nn.functional as F

from commefficient_amd.models.gpt2 import GPT2DoubleHeads
from commefficient_amd.parallel import dist
from commefficient_amd.parallel.fed_model import FedModel
from commefficient_amd.parallel.server import FedOptimizer
from commefficient_amd.train.losses import gpt2_loss_train, token_weighted
from commefficient_amd.utils.args import parse_args


def _batch(B=4, C=2, L=12, V=300, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, V, (B, C, L), generator=g)
    tt = torch.randint(0, V, (B, C, L), generator=g)
    mc_tok = torch.full((B, C), L - 1)
    labels = torch.full((B, C, L), -100)
    # very different numbers of labelled tokens per example
    for b in range(B):
        n = 2 + 3 * b
        labels[b, -1, L - n:] = ids[b, -1, L - n:]
    mc = torch.full((B,), C - 1)
    return ids, mc_tok, labels, tt, mc


def _tiny():
    torch.manual_seed(0)
    m = GPT2DoubleHeads("gpt2", n_layer=1, n_embd=32, n_head=2, n_positions=64)
    for mod in m.modules():  # deterministic forwards (train mode inside FedModel)
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    return m


class _A:
    lm_coef, mc_coef = 1.0, 0.5


def test_token_weighted_group_means():
    ts = torch.tensor([1., 2., 3., 4., 5.])
    nt = torch.tensor([1., 1., 2., 3., 4.])
    r = token_weighted(ts, nt, torch.tensor([7, 7, 9, 9, 9]))
    torch.testing.assert_close(r[:2].mean(), torch.tensor(3 / 2))
    torch.testing.assert_close(r[2:].mean(), torch.tensor(12 / 9))
    torch.testing.assert_close(token_weighted(ts, nt).mean(), torch.tensor(15 / 11))


def test_gpt2_loss_mean_is_hf_token_mean():
    model = _tiny().eval()  # no dropout: both forwards identical
    ids, mc_tok, labels, tt, mc = _batch()
    per_ex, _ = gpt2_loss_train(model, (ids, mc_tok, labels, tt), mc, _A())
    out = model.model(input_ids=ids, token_type_ids=tt, mc_token_ids=mc_tok)
    lm = F.cross_entropy(out.logits[..., :-1, :].reshape(-1, out.logits.size(-1)),
                         labels[..., 1:].reshape(-1), ignore_index=-100)  # HF lm_loss
    mcl = F.cross_entropy(out.mc_logits, mc)
    torch.testing.assert_close(per_ex.mean(), lm + 0.5 * mcl, rtol=1e-5, atol=1e-6)


def test_gpt2_merged_equals_per_client():
    dist.init("cpu")
    ids, mc_tok, labels, tt, mc = _batch()
    res = []
    for merge in ("on", "off"):
        model = _tiny()
        args = parse_args(argv=["--mode", "uncompressed", "--local_momentum", "0",
                                "--virtual_momentum", "0", "--num_workers", "2",
                                "--local_batch_size", "2", "--device", "cpu", "--dtype", "fp32",
                                "--num_clients", "2", "--merge_clients", merge,
                                "--weight_decay", "0", "--lm_coef", "1", "--mc_coef", "0.5"],
                          probe_port=False)
        fed = FedModel(model, gpt2_loss_train, args, num_clients=2)
        opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1), args, fed)
        cids = torch.tensor([0, 0, 1, 1])
        fed((cids, ids, mc_tok, labels, tt, mc))
        opt.step()
        res.append(fed.w.clone())
    torch.testing.assert_close(res[0], res[1], rtol=1e-4, atol=1e-6)


def test_gpt2_label_position_lm_head_matches_full_logits():
    """LM head evaluated only at the labelled positions (data/fed_persona.py
    label_positions) gives the full-logit loss and gradients."""
    from commefficient_amd.data.fed_persona import label_positions
    ids, mc_tok, labels, tt, mc = _batch()
    labels[1, 0, 3:5] = ids[1, 0, 3:5]  # labels in a non-final candidate too
    lp = label_positions(labels)
    assert lp.shape[0] == 4 and (lp >= 0).sum() == (labels[..., 1:] != -100).sum()
    grads = []
    for inputs in ((ids, mc_tok, labels, tt), (ids, mc_tok, labels, tt, lp)):
        model = _tiny().eval()
        per_ex, _ = gpt2_loss_train(model, inputs, mc, _A())
        per_ex.sum().backward()
        grads.append((per_ex.detach(), torch.cat([p.grad.reshape(-1) for p in model.parameters()])))
    torch.testing.assert_close(grads[0][0], grads[1][0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(grads[0][1], grads[1][1], rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_gpt2_weight_cast_once_matches_autocast_gpu():
    """bf16 model replica refreshed by one cast per forward (--weight_cast
    once, parallel/flat.py) vs per-op autocast: same update to bf16 accuracy,
    and the flat fp32 gradient receives every parameter's gradient."""
    dist.init("cuda")
    ids, mc_tok, labels, tt, mc = (t.cuda() for t in _batch())
    res = []
    for wc in ("once", "autocast"):
        model = _tiny()
        args = parse_args(argv=["--mode", "uncompressed", "--local_momentum", "0",
                                "--virtual_momentum", "0", "--num_workers", "2",
                                "--local_batch_size", "2", "--device", "cuda", "--dtype", "bf16",
                                "--num_clients", "2", "--weight_decay", "0",
                                "--weight_cast", wc], probe_port=False)
        fed = FedModel(model, gpt2_loss_train, args, num_clients=2)
        assert (fed._shadow is not None) == (wc == "once")
        opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1), args, fed)
        w0 = fed.w.clone()
        loss = fed((torch.tensor([0, 0, 1, 1]), ids, mc_tok, labels, tt, mc))[0]
        opt.step()
        res.append((fed.w - w0, loss))
    (d1, l1), (d2, l2) = res
    torch.testing.assert_close(l1, l2, rtol=3e-2, atol=3e-2)
    assert (d1 != 0).float().mean() > 0.9  # every parameter got its gradient
    assert ((d1 - d2).norm() / d2.norm()) < 5e-2
