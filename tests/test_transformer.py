"""GPT-2 block-junction kernels (csrc/transformer.hip, ops/transformer.py).

CPU: the native-path forward/backward (on the PyTorch references of the
kernels) equals HF's GPT2Model in fp32 to bf16 accuracy, dropout masks have
the requested rate and the backward uses the forward's mask.
GPU: every kernel against its fp32 PyTorch reference (same dropout hash), and
the whole native GPT-2 hidden-state forward/backward against HF on the GPU.
"""
import pytest
import torch
import torch.nn.functional as F

from commefficient_amd.models.gpt2 import build_double_heads
from commefficient_amd.ops import transformer as tx


def _tiny_gpt2(n_embd=256, n_layer=2, n_head=4, seed=0):
    torch.manual_seed(seed)
    m = build_double_heads("gpt2", n_special=0, n_layer=n_layer, n_embd=n_embd, n_head=n_head,
                           n_positions=64)
    return m


def _inputs(Nb=3, C=2, L=20, V=500, seed=1, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, V, (Nb, C, L), generator=g)
    tt = torch.randint(0, V, (Nb, C, L), generator=g)
    return ids.to(device), tt.to(device)


def _grads(model):
    return {n: p.grad.detach().float().clone() for n, p in model.named_parameters()
            if p.grad is not None}


def _hf_vs_native(device):
    import copy
    ref = _tiny_gpt2().to(device).eval()
    # bf16-representable weights so both sides start from identical parameters
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    nat = copy.deepcopy(ref).to(torch.bfloat16)
    ids, tt = _inputs(device=device)
    gw = torch.randn(*ids.shape, 256, generator=torch.Generator().manual_seed(3)).to(device)
    h_ref = ref.transformer(input_ids=ids, token_type_ids=tt, use_cache=False)[0]
    (h_ref * gw).sum().backward()
    assert tx.native_ok(nat.transformer, ids)
    h_nat = tx.gpt2_hidden(nat.transformer, ids, tt)
    (h_nat.float() * gw).sum().backward()
    torch.testing.assert_close(h_nat.float(), h_ref, rtol=3e-2, atol=6e-2)
    gr, gn = _grads(ref), _grads(nat)
    assert set(gr) == set(gn)
    for n in gr:
        if "multiple_choice" in n or "lm_head" in n:
            continue
        rel = (gn[n] - gr[n]).norm() / gr[n].norm().clamp_min(1e-6)
        assert rel < 6e-2, (n, float(rel))


def test_native_path_matches_hf_cpu():
    _hf_vs_native("cpu")


def test_dropout_mask_rate_and_determinism():
    k = tx.drop_keep(1 << 16, seed=12345, p=0.1)
    assert abs(1 - k.float().mean().item() - 0.1) < 0.01
    assert torch.equal(k, tx.drop_keep(1 << 16, seed=12345, p=0.1))
    assert not torch.equal(k, tx.drop_keep(1 << 16, seed=12346, p=0.1))


def test_resid_ln_dropout_backward_uses_forward_mask():
    """With dropout the junction's gradient equals autograd through an explicit
    composition that uses the same keep mask."""
    torch.manual_seed(0)
    M, H, p = 16, 256, 0.25
    x = torch.randn(M, H).to(torch.bfloat16).requires_grad_()
    o = torch.randn(M, 64).to(torch.bfloat16).requires_grad_()
    W = (torch.randn(64, H) * 0.1).to(torch.bfloat16).requires_grad_()
    b = (torch.randn(H) * 0.1).to(torch.bfloat16).requires_grad_()
    gam = (1 + 0.1 * torch.randn(H)).to(torch.bfloat16).requires_grad_()
    bet = (0.1 * torch.randn(H)).to(torch.bfloat16).requires_grad_()
    h, y = tx._ResidLN.apply(x, o, W, b, gam, bet, p, 777, 1e-5)
    gy, gh = torch.randn(M, H), torch.randn(M, H)
    (y.float() * gy).sum().add_((h.float() * gh).sum()).backward()
    keep = tx.drop_keep(M * H, 777, p).view(M, H).float()
    leaves = [t.detach().float().requires_grad_() for t in (x, o, W, b, gam, bet)]
    xf, of, Wf, bf, gf, bef = leaves
    hf = xf + keep * (of @ Wf + bf) / (1 - p)
    yf = torch.nn.functional.layer_norm(hf, (H,), gf, bef, 1e-5)
    (yf * gy).sum().add_((hf * gh).sum()).backward()
    torch.testing.assert_close(h.float(), hf, rtol=2e-2, atol=5e-2)
    for a, r in zip((x, o, W, b, gam, bet), leaves):
        rel = (a.grad.float() - r.grad).norm() / r.grad.norm()
        assert rel < 3e-2, float(rel)


# ---------------------------------------------------------------- GPU
def _rows(M, H, dev, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(M, H, generator=g) * scale).to(torch.bfloat16).to(dev)


@pytest.mark.gpu
@pytest.mark.parametrize("H", [256, 768, 1024])
@pytest.mark.parametrize("p_drop", [0.0, 0.1])
@pytest.mark.parametrize("branch", [True, False])
def test_resid_ln_kernels_vs_reference_gpu(H, p_drop, branch):
    from commefficient_amd._ext import ops
    dev = "cuda"
    M = 1000
    x, p = _rows(M, H, dev, seed=1), _rows(M, H, dev, 0.5, seed=2)
    bias = _rows(1, H, dev, 0.1, seed=3).view(H)
    gam = (1 + _rows(1, H, dev, 0.1, seed=4).float()).to(torch.bfloat16).view(H)
    bet = _rows(1, H, dev, 0.1, seed=5).view(H)
    pb = p if branch else None
    bb = bias if branch else None
    out = ops().resid_ln_fwd(x, pb, bb, gam, bet, p_drop, 99, 1e-5, True)
    ref = tx._ref_resid_ln_fwd(x, pb, bb, gam, bet, p_drop, 99, 1e-5, True)
    torch.testing.assert_close(out[0].float(), ref[0].float(), rtol=1e-2, atol=1e-2)
    assert torch.equal(out[0] == 0, ref[0] == 0)  # identical dropout masks
    torch.testing.assert_close(out[1].float(), ref[1].float(), rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(out[2], ref[2], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out[3], ref[3], rtol=1e-3, atol=1e-3)
    gy, gh = _rows(M, H, dev, seed=6), _rows(M, H, dev, seed=7)
    h = out[0]
    bo = ops().resid_ln_bwd(gy, gh, h, out[2], out[3], gam, p_drop, 99, True, branch)
    br = tx._ref_resid_ln_bwd(gy, gh, h, out[2], out[3], gam, p_drop, 99, True, branch)
    for a, r in zip(bo, br):
        if r.numel() == 0:
            continue
        rel = (a.float() - r.float()).norm() / r.float().norm().clamp_min(1e-6)
        assert rel < 1e-2, float(rel)
    assert torch.equal(bo[1] == 0, br[1] == 0) or p_drop == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("N", [768, 2304, 3072])
def test_bias_gelu_kernels_vs_reference_gpu(N):
    from commefficient_amd._ext import ops
    dev = "cuda"
    M = 777
    u = _rows(M, N, dev, 2.0, seed=1)
    b = _rows(1, N, dev, 0.5, seed=2).view(N)
    f = ops().bias_gelu_fwd(u, b)
    torch.testing.assert_close(f.float(), tx._ref_bias_gelu_fwd(u, b).float(), rtol=1e-2,
                               atol=1e-2)
    gf = _rows(M, N, dev, seed=3)
    for gelu in (True, False):
        du, db = ops().bias_act_bwd(gf, u, b, gelu)
        rdu, rdb = tx._ref_bias_act_bwd(gf, u, b, gelu)
        if gelu:
            torch.testing.assert_close(du.float(), rdu.float(), rtol=2e-2, atol=2e-2)
        rel = (db.float() - rdb.float()).norm() / rdb.float().norm()
        assert rel < 1e-2, float(rel)


@pytest.mark.gpu
def test_native_path_matches_hf_gpu():
    _hf_vs_native("cuda")


@pytest.mark.gpu
def test_native_gpt2_loss_grad_deterministic_gpu():
    """Same seeds -> bitwise identical gradients (fixed-order reductions) for
    every parameter whose gradient does not pass through the attention
    backward (the last block's MLP / ln_2 and ln_f)."""
    import copy
    base = _tiny_gpt2().cuda().to(torch.bfloat16).train()
    ids, tt = _inputs(device="cuda")
    out = []
    for _ in range(2):
        m = copy.deepcopy(base)
        m.transformer._commeff_seeds = tx._Seeds(5)
        torch.manual_seed(0)  # attention dropout
        h = tx.gpt2_hidden(m.transformer, ids, tt)
        h.float().square().mean().backward()
        keep = ("h.1.mlp", "h.1.ln_2", "ln_f", "h.1.attn.c_proj")
        out.append(torch.cat([p.grad.reshape(-1).float() for n, p in m.named_parameters()
                              if p.grad is not None and any(k in n for k in keep)]))
    assert torch.equal(out[0], out[1])


def _sink_vs_cat(device):
    """grad_sinks (fp32 accumulation into the flat gradient) == the bf16
    replica's .grad gathered by collect_shadow_grads, over two backward passes
    (microbatch accumulation)."""
    from commefficient_amd.parallel.flat import FlatParams
    ids, tt = _inputs(device=device)
    res = []
    for use_sinks in (True, False):
        m = _tiny_gpt2().to(device).eval()
        flat = FlatParams(m, device)
        sh = flat.make_bf16_shadow()
        flat.refresh_shadow()
        flat.zero_grad()
        for rep in range(2):
            with tx.grad_sinks(flat.grad_sink_map() if use_sinks else None):
                h = tx.gpt2_hidden(sh.transformer, ids[:, :, rep:], tt[:, :, rep:])
            h.float().square().mean().backward()
            tx.join_wgrad_stream()
            flat.collect_shadow_grads()
        res.append(flat.g.clone())
    a, b = res
    assert (a != 0).float().mean() > 0.05  # wte rows of unused tokens stay 0
    rel = (a - b).norm() / b.norm()
    assert rel < 2e-2, float(rel)


def test_grad_sinks_match_collected_grads_cpu():
    _sink_vs_cat("cpu")


@pytest.mark.gpu
def test_grad_sinks_match_collected_grads_gpu():
    _sink_vs_cat("cuda")


@pytest.mark.gpu
def test_side_stream_column_sums_bitwise_gpu(monkeypatch):
    """The junctions' column sums queued on the weight-gradient side stream
    (colsum_into after resid_ln_bwd_part / bias_act_bwd_part) give the flat
    gradient bitwise equal to the in-line sums (same kernel, same order)."""
    from commefficient_amd.parallel.flat import FlatParams
    ids, tt = _inputs(device="cuda")
    res = []
    for side in (True, False):
        monkeypatch.setattr(tx, "_COLSUM_SIDE", side)
        torch.manual_seed(0)
        m = _tiny_gpt2().to("cuda").eval()
        flat = FlatParams(m, "cuda")
        sh = flat.make_bf16_shadow()
        flat.refresh_shadow()
        flat.zero_grad()
        for rep in range(2):
            with tx.grad_sinks(flat.grad_sink_map()):
                h = tx.gpt2_hidden(sh.transformer, ids[:, :, rep:], tt[:, :, rep:])
            h.float().square().mean().backward()
            tx.join_wgrad_stream()
        torch.cuda.synchronize()
        res.append(flat.g.clone())
    assert torch.equal(res[0], res[1])


@pytest.mark.gpu
def test_fedmodel_native_transformer_matches_hf_gpu():
    """One FetchSGD-free (uncompressed) round of a GPT-2 double-heads model
    through FedModel: native junctions + fp32 gradient sinks vs HF modules."""
    from commefficient_amd.models.gpt2 import GPT2DoubleHeads
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.server import FedOptimizer
    from commefficient_amd.train.losses import gpt2_loss_train
    from commefficient_amd.utils.args import parse_args
    dist.init("cuda")
    ids, tt = _inputs(Nb=4, device="cuda")
    mc_tok = torch.full((4, 2), 19, device="cuda")
    labels = torch.full((4, 2, 20), -100, device="cuda")
    labels[:, -1, 12:] = ids[:, -1, 12:]
    mc = torch.ones(4, dtype=torch.long, device="cuda")
    res = []
    for impl in ("native", "hf"):
        torch.manual_seed(0)
        model = GPT2DoubleHeads("gpt2", n_layer=2, n_embd=256, n_head=4, n_positions=64)
        for mod in model.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
        args = parse_args(argv=["--mode", "uncompressed", "--local_momentum", "0",
                                "--virtual_momentum", "0", "--num_workers", "2",
                                "--local_batch_size", "2", "--device", "cuda", "--dtype", "bf16",
                                "--num_clients", "2", "--weight_decay", "0",
                                "--weight_cast", "once", "--transformer", impl], probe_port=False)
        fed = FedModel(model, gpt2_loss_train, args, num_clients=2)
        opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1), args, fed)
        w0 = fed.w.clone()
        loss = fed((torch.tensor([0, 0, 1, 1]), ids, mc_tok, labels, tt, mc))[0]
        opt.step()
        res.append((fed.w - w0, loss))
    (d1, l1), (d2, l2) = res
    torch.testing.assert_close(l1, l2, rtol=2e-2, atol=2e-2)
    assert (d1 != 0).float().mean() > 0.9
    assert ((d1 - d2).norm() / d2.norm()) < 5e-2


def _unpad_vs_padded(device):
    """Token-wise ops on the real tokens only (host lengths) == the padded
    forward at every real position, and the same parameter gradients."""
    import copy
    base = _tiny_gpt2().to(device).to(torch.bfloat16).eval()
    ids, tt = _inputs(device=device)
    lens = torch.tensor([[20, 13], [7, 16], [20, 1]])  # host lengths, right padding
    mask = (torch.arange(20)[None, None, :] < lens[..., None]).to(device)
    gw = torch.randn(*ids.shape, 256, generator=torch.Generator().manual_seed(3)).to(device)
    gw = gw * mask[..., None]  # the losses read real positions only
    outs = []
    for use in (False, True):
        m = copy.deepcopy(base)
        h = tx.gpt2_hidden(m.transformer, ids, tt, lens if use else None)
        (h.float() * gw).sum().backward()
        outs.append((h.float() * mask[..., None], _grads(m)))
    (h0, g0), (h1, g1) = outs
    torch.testing.assert_close(h1, h0, rtol=2e-2, atol=3e-2)
    for n in g0:
        rel = (g1[n] - g0[n]).norm() / g0[n].norm().clamp_min(1e-6)
        assert rel < 3e-2, (n, float(rel))


def test_unpadded_tokens_match_padded_cpu():
    _unpad_vs_padded("cpu")


@pytest.mark.gpu
def test_unpadded_tokens_match_padded_gpu():
    _unpad_vs_padded("cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("unpad", [False, True])
def test_rows_heads_layout_kernels_gpu(unpad):
    from commefficient_amd._ext import ops
    N, L, nh, hd = 5, 24, 12, 64
    H = nh * hd
    lens = torch.tensor([24, 3, 17, 1, 10]) if unpad else torch.full((5,), 24)
    tok, inv, _, _ = tx.real_token_index(lens, L, "cpu")
    Mr = tok.numel()
    g = torch.Generator().manual_seed(0)
    qkv = torch.randn(Mr, 3 * H, generator=g).to(torch.bfloat16)
    ti, ii = (tok.cuda(), inv.cuda()) if unpad else (None, None)
    out = ops().pad_rows(qkv.cuda(), ii, N * L)
    assert torch.equal(out.cpu(), tx._ref_pad_rows(qkv, inv if unpad else None, N * L))
    # strided sources (a transposed [N, L, nh, hd] tensor) back to rows
    srcs = [torch.randn(N, L, nh, hd, generator=g).to(torch.bfloat16).transpose(1, 2)
            for _ in range(3)]
    got = ops().heads_to_rows([s.cuda() for s in srcs], ti, Mr)
    exp = tx._ref_heads_to_rows(srcs, tok if unpad else None, Mr)
    assert torch.equal(got.cpu(), exp)


def _attn_case(device, lens=(37, 128, 1, 90), nh=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    lens_t = torch.tensor(lens, dtype=torch.int32)
    start = torch.cat([torch.zeros(1, dtype=torch.int32), lens_t.cumsum(0)[:-1].int()])
    M = int(lens_t.sum())
    qkv = (torch.randn(M, 3 * nh * 64, generator=g) * 0.5).to(torch.bfloat16).to(device)
    return qkv, start.to(device), lens_t.to(device), nh


def test_fused_attention_reference_matches_sdpa_cpu():
    """The kernel's fp32 reference (no dropout) == per-sequence causal SDPA."""
    import torch.nn.functional as F
    qkv, start, lens, nh = _attn_case("cpu")
    o, _ = tx._ref_attn(qkv, start, lens, nh, 0.0, 0)
    for n in range(start.numel()):
        s0, L = int(start[n]), int(lens[n])
        x = qkv[s0:s0 + L].float().view(L, 3, nh, 64).permute(1, 2, 0, 3)
        ref = F.scaled_dot_product_attention(x[0], x[1], x[2], is_causal=True)
        torch.testing.assert_close(o[s0:s0 + L].float(), ref.transpose(0, 1).reshape(L, -1),
                                   rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("lens", [(37, 128, 1, 90),             # all-in-LDS kernels
                                  (200, 64, 1, 129),            # flash kernels, ld 256
                                  (512, 300, 17),               # ld 512
                                  (1024, 5)])                   # GPT-2's n_positions
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_fused_attention_kernels_vs_reference_gpu(p, lens):
    """csrc/attention.hip forward (O, LSE) and backward (dQ, dK, dV) vs the
    fp32 PyTorch reference of the same math and dropout hash, for the short
    (<= 128 tokens) and the long (flash-style, up to 1024) kernel families."""
    from commefficient_amd._ext import ops
    qkv, start, lens_t, nh = _attn_case("cuda", lens=lens)
    L = max(lens)
    ld = tx.attn_lse_ld(L)
    o, lse = ops().attn_fwd(qkv, start, lens_t, nh, p, 1234, L)
    assert lse.numel() == len(lens) * nh * ld
    ro, rlse = tx._ref_attn(qkv.cpu(), start.cpu(), lens_t.cpu(), nh, p, 1234, L)
    torch.testing.assert_close(o.float().cpu(), ro.float(), rtol=2e-2, atol=2e-2)
    valid = torch.zeros(len(lens) * nh, ld, dtype=torch.bool)
    for n, Ln in enumerate(lens):
        valid[n * nh:(n + 1) * nh, :Ln] = True
    torch.testing.assert_close(lse.cpu().view(-1, ld)[valid], rlse.view(-1, ld)[valid],
                               rtol=1e-3, atol=1e-3)
    gout = (torch.randn(o.shape, generator=torch.Generator().manual_seed(5)) * 0.5).to(
        torch.bfloat16)
    dq = ops().attn_bwd(qkv, o, gout.cuda(), lse, start, lens_t, nh, p, 1234, L)
    x = qkv.cpu().float().requires_grad_()
    rref, _ = tx._ref_attn(x, start.cpu(), lens_t.cpu(), nh, p, 1234, L)
    rref.float().backward(gout.float())
    for part in range(3):
        a = dq.float().cpu()[:, part * nh * 64:(part + 1) * nh * 64]
        r = x.grad[:, part * nh * 64:(part + 1) * nh * 64]
        rel = (a - r).norm() / r.norm()
        assert rel < 3e-2, (part, float(rel))


def test_attention_reference_long_matches_sdpa_cpu():
    """The reference at a flash-kernel length (LSE stride 256) == causal SDPA."""
    import torch.nn.functional as F
    qkv, start, lens, nh = _attn_case("cpu", lens=(200, 3), nh=2)
    o, lse = tx._ref_attn(qkv, start, lens, nh, 0.0, 0, 200)
    assert lse.numel() == 2 * 2 * 256
    x = qkv[:200].float().view(200, 3, nh, 64).permute(1, 2, 0, 3)
    ref = F.scaled_dot_product_attention(x[0], x[1], x[2], is_causal=True)
    torch.testing.assert_close(o[:200].float(), ref.transpose(0, 1).reshape(200, -1),
                               rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_native_path_fused_attention_matches_sdpa_path_gpu():
    """gpt2_hidden with the fused attention == with the SDPA path (no dropout)."""
    import copy
    base = _tiny_gpt2().cuda().to(torch.bfloat16).eval()
    ids, tt = _inputs(device="cuda")
    lens = torch.tensor([[20, 13], [7, 16], [20, 1]])
    mask = (torch.arange(20)[None, None, :] < lens[..., None]).cuda()
    gw = torch.randn(*ids.shape, 256, generator=torch.Generator().manual_seed(3)).cuda()
    gw = gw * mask[..., None]
    outs = []
    for fused in (True, False):
        tx.set_fused_attention(fused)
        m = copy.deepcopy(base)
        h = tx.gpt2_hidden(m.transformer, ids, tt, lens)
        (h.float() * gw).sum().backward()
        outs.append((h.float() * mask[..., None], _grads(m)))
    tx.set_fused_attention(True)
    (h0, g0), (h1, g1) = outs
    torch.testing.assert_close(h0, h1, rtol=2e-2, atol=3e-2)
    for n in g0:
        rel = (g1[n] - g0[n]).norm() / g0[n].norm().clamp_min(1e-6)
        assert rel < 3e-2, (n, float(rel))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sketch", "uncompressed"])
def test_bf16_replica_follows_sparse_server_steps_gpu(mode):
    """--weight_cast once: after a sparse (FetchSGD) server step the bf16
    replica is patched at the k changed coordinates instead of re-cast
    (parallel/flat.py weight mirror); it must equal bf16(w) bitwise before
    every forward, in sparse and dense modes alike."""
    from commefficient_amd.models.gpt2 import GPT2DoubleHeads
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.server import FedOptimizer
    from commefficient_amd.train.losses import gpt2_loss_train
    from commefficient_amd.utils.args import parse_args
    dist.init("cuda")
    ids, tt = _inputs(Nb=4, device="cuda")
    mc_tok = torch.full((4, 2), 19, device="cuda")
    labels = torch.full((4, 2, 20), -100, device="cuda")
    labels[:, -1, 12:] = ids[:, -1, 12:]
    mc = torch.ones(4, dtype=torch.long, device="cuda")
    torch.manual_seed(0)
    model = GPT2DoubleHeads("gpt2", n_layer=2, n_embd=256, n_head=4, n_positions=64)
    extra = (["--error_type", "virtual", "--k", "5000", "--num_rows", "5", "--num_cols", "20000"]
             if mode == "sketch" else [])
    args = parse_args(argv=["--mode", mode, "--local_momentum", "0", "--virtual_momentum", "0.9",
                            "--num_workers", "2", "--local_batch_size", "2", "--device", "cuda",
                            "--dtype", "bf16", "--num_clients", "2", "--weight_cast", "once"] + extra, probe_port=False)
    fed = FedModel(model, gpt2_loss_train, args, num_clients=2)
    opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1), args, fed)
    flat = fed.flat
    for r in range(3):
        w0 = fed.w.clone()
        fed((torch.tensor([0, 0, 1, 1]), ids, mc_tok, labels, tt, mc))
        assert torch.equal(flat.wb, fed.w.to(torch.bfloat16))  # what this round's forward used
        opt.step()
        assert not torch.equal(fed.w, w0)
        if mode == "sketch":
            assert flat._wb_valid == fed.w.data_ptr()  # patched, not re-cast next round
            assert torch.equal(flat.wb, fed.w.to(torch.bfloat16))
        else:
            assert flat._wb_valid is None


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1000, 256, 512), (9600, 768, 2304), (333, 768, 768),
                                   (4100, 3072, 768)])
def test_gemm_tn_wgrad_vs_fp32_reference_gpu(shape):
    """csrc/gemm_tn.hip: sink += a^T b (split-K slabs or direct) vs the fp32
    product of the same bf16 operands, token counts not multiples of 64."""
    from commefficient_amd._ext import ops
    T, M, N = shape
    g = torch.Generator().manual_seed(T)
    a = torch.randn(T, M, generator=g).to(torch.bfloat16).cuda()
    b = torch.randn(T, N, generator=g).to(torch.bfloat16).cuda()
    sink0 = torch.randn(M, N, generator=g).cuda()
    sink = sink0.clone()
    ops().gemm_tn_acc(sink, a, b)
    ref = sink0 + a.float().t() @ b.float()
    torch.testing.assert_close(sink, ref, rtol=1e-4, atol=1e-3 * (T ** 0.5) / 10)
    # deterministic: a second call adds the identical product
    sink2 = sink0.clone()
    ops().gemm_tn_acc(sink2, a, b)
    assert torch.equal(sink, sink2)
    # through the transformer helper on a column view of a wider buffer (a^T view)
    big = torch.zeros(M, N + 256, device="cuda")
    view = big[:, :N]
    tx._acc_mm(view, a.t(), b)
    torch.testing.assert_close(view, ref - sink0, rtol=1e-4, atol=1e-3 * (T ** 0.5) / 10)


@pytest.mark.gpu
@pytest.mark.parametrize("sinked", [False, True])
def test_lm_head_native_vs_fp32_gpu(sinked, monkeypatch):
    """The tied LM head (vocabulary 50,257, no tile multiple) on the native
    GEMMs (ops/transformer.py _LMHead): logits, dh and dW (returned, or
    accumulated into an fp32 gradient sink on the side stream) vs the fp32
    products of the same bf16 operands, for an external (unpadded) output
    gradient."""
    V, H, T = 50257, 768, 600
    monkeypatch.setattr(tx, "_LM_NATIVE", True)
    g = torch.Generator().manual_seed(5)
    head = torch.nn.Linear(H, V, bias=False).to(torch.bfloat16).cuda()
    with torch.no_grad():
        head.weight.copy_((torch.randn(V, H, generator=g) * 0.05).to(torch.bfloat16))
    m = type("M", (), {})()
    m.lm_head = head
    h = torch.randn(T, H, generator=g).to(torch.bfloat16).cuda().requires_grad_(True)
    gy = torch.randn(T, V, generator=g).to(torch.bfloat16).cuda()
    W = head.weight
    sink0 = torch.randn(V, H, generator=g).cuda()
    sink = sink0.clone()
    with tx.grad_sinks({id(W): sink} if sinked else None):
        logits = tx.lm_head(m, h)
        assert logits.shape == (T, V) and logits.grad_fn is not None
        fns = [logits.grad_fn] + [f for f, _ in logits.grad_fn.next_functions if f is not None]
        assert any(type(f).__name__.startswith("_LMHead") for f in fns)
        logits.backward(gy)
    tx.join_wgrad_stream()
    torch.cuda.synchronize()
    ref = h.detach().float() @ W.detach().float().t()
    rel = lambda a, b: ((a.float() - b).abs().max() / b.abs().max()).item()  # noqa: E731
    assert rel(logits.detach(), ref) < 1e-2
    assert rel(h.grad, gy.float() @ W.detach().float()) < 1e-2
    dw_ref = gy.float().t() @ h.detach().float()
    if sinked:
        assert W.grad is None
        torch.testing.assert_close(sink - sink0, dw_ref, rtol=1e-3, atol=2e-2)
    else:
        assert rel(W.grad, dw_ref) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("dw_tn", [False, True])
def test_lm_head_native_ce_chain_padded_gradient(dw_tn, monkeypatch):
    """LM head -> native cross-entropy on the padded logits -> backward: the
    gradient stays in the padded layout end to end (no copies), dW goes into
    the sink (hipBLASLt, or the TN GEMM's M = V edge tile), and the result
    matches the fp32 chain on the same bf16 operands."""
    from commefficient_amd.ops.nn import cross_entropy_correct
    monkeypatch.setattr(tx, "_LM_DW_TN", dw_tn)
    V, H, T = 50257, 768, 512
    g = torch.Generator().manual_seed(7)
    head = torch.nn.Linear(H, V, bias=False).to(torch.bfloat16).cuda()
    with torch.no_grad():
        head.weight.copy_((torch.randn(V, H, generator=g) * 0.05).to(torch.bfloat16))
    m = type("M", (), {})()
    m.lm_head = head
    W = head.weight
    h = torch.randn(T, H, generator=g).to(torch.bfloat16).cuda().requires_grad_(True)
    tgt = torch.randint(0, V, (T,), generator=g).cuda()
    tgt[::5] = -100
    w = torch.rand(T, generator=g).cuda()
    sink = torch.zeros(V, H, device="cuda")
    with tx.grad_sinks({id(W): sink}):
        logits = tx.lm_head(m, h)
        assert logits.stride(0) == -(-V // 8) * 8  # the padded buffer itself
        loss, _ = cross_entropy_correct(logits, tgt)
        (loss * w).sum().backward()
    tx.join_wgrad_stream()
    torch.cuda.synchronize()
    hr = h.detach().float().requires_grad_(True)
    Wr = W.detach().float().requires_grad_(True)
    ref = F.cross_entropy(hr @ Wr.t(), tgt, ignore_index=-100, reduction="none")
    (ref * w).sum().backward()
    rel = lambda a, b: ((a.float() - b).abs().max() / b.abs().max()).item()  # noqa: E731
    assert rel(loss, ref) < 1e-2
    assert rel(h.grad, hr.grad) < 2e-2
    assert rel(sink, Wr.grad) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("with_tt,with_tok,sink", [(True, True, True), (True, False, False), (False, True, False)])
def test_native_embedding_vs_fp32(with_tt, with_tok, sink):
    """csrc/embed.hip: e = wte[ids] + wpe[t % L] (+ wte[tt]) on the real token
    rows, and the sort-free fixed-point backward into the fp32 table
    gradients (or the returned gradients), vs an fp32 index_add reference;
    bitwise deterministic across runs."""
    from commefficient_amd.ops import transformer as tx
    torch.manual_seed(0)
    V, P, H, N, L = 50257, 1024, 768, 6, 40
    wte = (torch.randn(V, H, device="cuda") * 0.02).bfloat16().requires_grad_(True)
    wpe = (torch.randn(P, H, device="cuda") * 0.02).bfloat16().requires_grad_(True)
    ids = torch.randint(0, V, (N * L,), device="cuda")
    ids[::7] = 13  # repeated tokens
    tt = torch.randint(50254, 50257, (N * L,), device="cuda") if with_tt else None
    lengths = torch.tensor([40, 33, 7, 40, 1, 25])
    tok = tx.real_token_index(lengths, L, "cuda")[0] if with_tok else None
    rows = tok.long() if tok is not None else torch.arange(N * L, device="cuda")
    de = (torch.randn(rows.numel(), H, device="cuda")).bfloat16()

    def run():
        sinks = None
        if sink:
            gw, gp = torch.zeros(V, H, device="cuda"), torch.zeros(P, H, device="cuda")
            sinks = {id(wte): gw, id(wpe): gp}
        wte.grad = wpe.grad = None
        with tx.grad_sinks(sinks):
            e = tx._Embed.apply(wte, wpe, ids, tt, tok, L)
        e.backward(de)
        if sink:
            return e, gw, gp
        return e, wte.grad.float(), wpe.grad.float()

    e, gw, gp = run()
    ref = wte.detach().float()[ids[rows]] + wpe.detach().float()[rows % L]
    if tt is not None:
        ref = ref + wte.detach().float()[tt[rows]]
    torch.testing.assert_close(e.float(), ref.bfloat16().float(), rtol=1e-2, atol=1e-3)
    rgw = torch.zeros(V, H, device="cuda").index_add_(0, ids[rows], de.float())
    if tt is not None:
        rgw.index_add_(0, tt[rows], de.float())
    rgp = torch.zeros(P, H, device="cuda").index_add_(0, rows % L, de.float())
    tol = 1e-5 if sink else 2e-2  # (returned gradients are bf16)
    torch.testing.assert_close(gw, rgw, rtol=tol, atol=tol)
    torch.testing.assert_close(gp, rgp, rtol=tol, atol=tol)
    e2, gw2, gp2 = run()  # deterministic, and the workspace was left zeroed
    assert torch.equal(gw, gw2) and torch.equal(gp, gp2)


@pytest.mark.gpu
def test_native_embedding_nonfinite_and_out_of_range():
    """The fixed-point embedding backward (csrc/embed.hip) does not turn NaN /
    Inf or huge gradients into finite garbage: values outside the exact range
    go to the fp32 spill accumulator, so the table gradient matches
    index_add's, NaN and Inf included; the next call is clean again."""
    from commefficient_amd.ops import transformer as tx
    torch.manual_seed(1)
    V, P, H, N, L = 1000, 64, 256, 4, 32
    wte = (torch.randn(V, H, device="cuda") * 0.02).bfloat16().requires_grad_(True)
    wpe = (torch.randn(P, H, device="cuda") * 0.02).bfloat16().requires_grad_(True)
    ids = torch.randint(0, V, (N * L,), device="cuda")
    ids[5] = ids[9] = 77  # a poisoned key shared with finite rows
    tt = torch.randint(997, 1000, (N * L,), device="cuda")
    de = torch.randn(N * L, H, device="cuda").bfloat16()
    de[5, 3] = float("nan")
    de[9, 4] = float("inf")
    de[9, 5] = 3.0e30  # finite, far past the fixed-point range
    de[17, 6] = -65536.0

    def run(d):
        gw, gp = torch.zeros(V, H, device="cuda"), torch.zeros(P, H, device="cuda")
        with tx.grad_sinks({id(wte): gw, id(wpe): gp}):
            e = tx._Embed.apply(wte, wpe, ids, tt, None, L)
        e.backward(d)
        return gw, gp

    gw, gp = run(de)
    rows = torch.arange(N * L, device="cuda")
    rgw = torch.zeros(V, H, device="cuda").index_add_(0, ids, de.float()).index_add_(0, tt, de.float())
    rgp = torch.zeros(P, H, device="cuda").index_add_(0, rows % L, de.float())
    assert torch.isnan(gw[77, 3]) and torch.isinf(gw[77, 4]) and gw[77, 4] > 0
    torch.testing.assert_close(gw, rgw, rtol=1e-5, atol=1e-5, equal_nan=True)
    torch.testing.assert_close(gp, rgp, rtol=1e-5, atol=1e-5, equal_nan=True)
    # workspace (fixed-point accumulator, spill, flags) left zeroed
    de2 = torch.randn(N * L, H, device="cuda").bfloat16()
    gw2, _ = run(de2)
    rgw2 = torch.zeros(V, H, device="cuda").index_add_(0, ids, de2.float()).index_add_(0, tt, de2.float())
    assert torch.isfinite(gw2).all()
    torch.testing.assert_close(gw2, rgw2, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_gpt2_nan_embedding_gradient_round_skipped(monkeypatch):
    """A NaN in the embedding's input gradient reaches the round's aggregate
    as a NaN (no integer-cast laundering in the native backward), so
    --skip_nonfinite drops that round: the weights stay bitwise where they
    were, and the next round trains again (mini GPT-2 under FetchSGD)."""
    import importlib.util
    import os
    from commefficient_amd.ops import transformer as tx
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts",
                        "gpt2_learning.py")
    spec = importlib.util.spec_from_file_location("gpt2_learning", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    extra = ["--mode", "sketch", "--error_type", "virtual", "--local_momentum", "0",
             "--virtual_momentum", "0.9", "--num_rows", "5", "--num_cols", "500000", "--k", "50000",
             "--lr_scale", "0.1", "--skip_nonfinite", "1", "--round_tape", "off"]
    args, fed, opt, train_loader, _ = mod.build(extra, "mini")
    poison = {"on": False, "hits": 0}
    orig = tx._Embed.backward

    def backward(ctx, de):
        if poison["on"]:
            de = de.clone()
            de[0, 0] = float("nan")
            poison["hits"] += 1
        return orig(ctx, de)

    monkeypatch.setattr(tx._Embed, "backward", staticmethod(backward))
    ws = []
    it = iter(train_loader)
    for r in range(3):
        batch = next(it)
        poison["on"] = r == 1
        fed(batch)
        opt.step()
        torch.cuda.synchronize()
        ws.append(fed.w.detach().clone())
    assert poison["hits"] >= 1, "the native embedding backward did not run"
    assert fed.skipped_rounds == 1, fed.skipped_rounds
    assert torch.isfinite(ws[2]).all()
    assert torch.equal(ws[0], ws[1]), "the poisoned round changed the weights"
    assert not torch.equal(ws[1], ws[2]), "training did not resume"
