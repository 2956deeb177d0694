"""Numerics of the native codec ops (CPU C++ backend and HIP gfx950 backend)
against the pure-torch oracles in tests/oracle.py."""
import pytest
import torch
import torch.nn.functional as F

from commefficient_amd import ops
from commefficient_amd.ops import CSVec, make_hashes
from oracle import OracleSketch, topk_oracle

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _sketch_pair(d, c, r, nb, device, seed=42):
    sk = CSVec(d, c, r, device=device, numBlocks=nb, seed=seed)
    h, bo, bs = make_hashes(r, c, nb, seed)
    orc = OracleSketch(h, bo, bs, d, c, r, nb)
    return sk, orc


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("d,c,r,nb", [(1000, 37, 5, 1), (5000, 101, 3, 4), (777, 50, 1, 1),
                                      (20000, 900, 5, 20), (3000, 64, 4, 1)])
def test_encode_matches_oracle(device, d, c, r, nb):
    torch.manual_seed(0)
    sk, orc = _sketch_pair(d, c, r, nb, device)
    v = torch.randn(d)
    sk.accumulateVec(v.to(device))
    orc.accumulate_vec(v)
    torch.testing.assert_close(sk.table.cpu().double(), orc.table, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("device", DEVICES)
def test_encode_direct_and_scaled_weight_term(device):
    torch.manual_seed(1)
    d, c, r = 4000, 211, 5
    sk, orc = _sketch_pair(d, c, r, 1, device)
    g, w = torch.randn(d), torch.randn(d)
    sk.accumulateVec(g.to(device), scale=3.0, wvec=w.to(device), wscale=0.25, dense=False)
    orc.accumulate_vec(3.0 * g + 0.25 * w)
    torch.testing.assert_close(sk.table.cpu().double(), orc.table, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("device", DEVICES)
def test_sketch_linearity(device):
    torch.manual_seed(2)
    d, c, r = 3000, 97, 5
    a, b = torch.randn(d), torch.randn(d)
    s1 = CSVec(d, c, r, device=device)
    s2 = s1.like()
    s3 = s1.like()
    s1.accumulateVec(a.to(device))
    s2.accumulateVec(b.to(device))
    s3.accumulateVec((a + b).to(device))
    torch.testing.assert_close(s1.table + s2.table, s3.table, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("r,nb", [(5, 1), (3, 7), (4, 1), (1, 1), (16, 2)])
def test_query_matches_oracle(device, r, nb):
    torch.manual_seed(3)
    d, c = 5000, 257
    sk, orc = _sketch_pair(d, c, r, nb, device)
    v = torch.randn(d)
    sk.accumulateVec(v.to(device))
    orc.accumulate_vec(v)
    est = sk.query().cpu().double()
    torch.testing.assert_close(est, orc.query(), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("device", DEVICES)
def test_heavy_hitter_recovery(device):
    torch.manual_seed(4)
    d, c, r, k = 50000, 2000, 5, 20
    v = torch.randn(d) * 0.01
    hh = torch.randperm(d)[:k]
    v[hh] = torch.randn(k).sign() * (10 + torch.rand(k))
    sk = CSVec(d, c, r, device=device, numBlocks=4)
    sk.accumulateVec(v.to(device))
    idx, vals = sk.unsketch_sparse(k)
    assert set(idx.cpu().tolist()) == set(hh.tolist())
    torch.testing.assert_close(vals.cpu(), v[idx.cpu()], rtol=0, atol=0.2)


@pytest.mark.parametrize("device", DEVICES)
def test_l2estimate(device):
    torch.manual_seed(5)
    d, c, r = 5000, 300, 5
    sk, orc = _sketch_pair(d, c, r, 1, device)
    v = torch.randn(d)
    sk.accumulateVec(v.to(device))
    orc.accumulate_vec(v)
    torch.testing.assert_close(sk.l2estimate().cpu().double(), orc.l2estimate(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("device", DEVICES)
def test_zero_heavy_hitters_matches_nonzero_mask(device):
    """zero_heavy_hitters == reference `nz = S(delta).nonzero(); T[nz] = 0`."""
    torch.manual_seed(6)
    d, c, r, k = 4000, 150, 5, 30
    sk = CSVec(d, c, r, device=device)
    sk.accumulateVec(torch.randn(d).to(device))
    other = torch.randn(r, c).to(device)
    idx, vals = sk.unsketch_sparse(k)
    # reference semantics via re-sketching the sparse update
    delta = torch.zeros(d)
    delta[idx.cpu()] = vals.cpu()
    resk = sk.like()
    resk.accumulateVec(delta.to(device), dense=False)
    mask = resk.table.cpu() != 0
    exp_t = sk.table.cpu().clone()
    exp_t[mask] = 0
    exp_o = other.cpu().clone()
    exp_o[mask] = 0
    sk.zero_heavy_hitters(idx, vals, other)
    torch.testing.assert_close(sk.table.cpu(), exp_t)
    torch.testing.assert_close(other.cpu(), exp_o)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("n,k", [(1000, 10), (100000, 5000), (12345, 1), (4096, 4095),
                                 (50, 50), (300000, 50000)])
def test_topk_matches_oracle(device, n, k):
    torch.manual_seed(7)
    x = torch.randn(n)
    idx, vals = ops.topk_abs(x.to(device), k)
    if n <= 20000:
        ei, ev = topk_oracle(x, k)
        assert torch.equal(idx.cpu(), ei)
        assert torch.equal(vals.cpu(), ev)
    else:
        thr = x.abs().sort(descending=True).values[k - 1]
        assert idx.numel() == k
        assert torch.all(idx.cpu()[1:] > idx.cpu()[:-1])
        assert torch.all(x[idx.cpu()].abs() >= thr)
        assert torch.equal(vals.cpu(), x[idx.cpu()])


@pytest.mark.parametrize("device", DEVICES)
def test_topk_ties_lower_index_wins(device):
    x = torch.tensor([1.0, -3.0, 3.0, 2.0, -3.0, 0.5, 3.0, 1.0])
    idx, vals = ops.topk_abs(x.to(device), 2)
    assert idx.cpu().tolist() == [1, 2]
    idx, vals = ops.topk_abs(x.to(device), 4)
    assert idx.cpu().tolist() == [1, 2, 4, 6]
    # many identical values (sparse vectors are mostly zeros)
    z = torch.zeros(10000)
    z[[5, 500, 9000]] = torch.tensor([1.0, -2.0, 3.0])
    idx, vals = ops.topk_abs(z.to(device), 10)
    assert idx.cpu().tolist() == [0, 1, 2, 3, 4, 5, 6, 7, 500, 9000]


@pytest.mark.parametrize("device", DEVICES)
def test_topk_dense_matches_reference_topk(device):
    torch.manual_seed(8)
    x = torch.randn(5000)
    out = ops.topk_dense(x.to(device), 100).cpu()
    ref = torch.zeros_like(x)
    ti = torch.topk(x ** 2, 100, sorted=False).indices
    ref[ti] = x[ti]
    torch.testing.assert_close(out, ref)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("mode", ["none", "virtual", "local"])
def test_momentum_ef(device, mode):
    torch.manual_seed(9)
    n = 10003
    V, E, G = torch.randn(n), torch.randn(n), torch.randn(n)
    Vd, Ed, Gd = V.clone().to(device), E.clone().to(device), G.clone().to(device)
    ops.momentum_ef(Vd, Ed, Gd, 0.9, 0.5, mode)
    V2 = 0.9 * V + 0.5 * G
    E2 = E + V2 if mode == "virtual" else (V2 if mode == "local" else E)
    torch.testing.assert_close(Vd.cpu(), V2)
    torch.testing.assert_close(Ed.cpu(), E2)


@pytest.mark.parametrize("device", DEVICES)
def test_apply_and_count(device):
    torch.manual_seed(10)
    n = 5000
    w = torch.randn(n)
    wd = w.clone().to(device)
    lm = torch.full((n,), -1, dtype=torch.int32, device=device)
    idx = torch.tensor([3, 10, 4000], dtype=torch.int64)
    vals = torch.tensor([1.0, 0.0, -2.0])
    ops.sparse_apply(wd, idx.to(device), vals.to(device), 0.1, None, lm, 0)
    exp = w.clone()
    exp[idx] -= 0.1 * vals
    torch.testing.assert_close(wd.cpu(), exp)
    assert (lm.cpu() == 0).sum().item() == 2  # the 0-valued update changed nothing
    delta = torch.zeros(n)
    delta[:100] = 1.0
    lrv = torch.full((n,), 0.5)
    ops.dense_apply(wd, delta.to(device), 0.0, lrv.to(device), lm, 1)
    exp -= 0.5 * delta
    torch.testing.assert_close(wd.cpu(), exp)
    cnt = ops.count_ge(lm, torch.tensor([-1, 0, 1, 2], dtype=torch.int32))
    # last_mod: 100 coords == 1 (incl. idx 3), idx 4000 == 0, rest -1
    assert cnt.cpu().tolist() == [n, 101, 100, 0]


@pytest.mark.parametrize("device", DEVICES)
def test_l2norm_clip_noise(device):
    torch.manual_seed(11)
    x = torch.randn(20000)
    xd = x.clone().to(device)
    nrm = ops.l2norm(xd)
    torch.testing.assert_close(nrm.cpu(), x.norm(), rtol=1e-5, atol=1e-5)
    ops.clip_noise(xd, nrm, clip=1.0, noise_std=0.0)
    torch.testing.assert_close(xd.cpu(), x / x.norm(), rtol=1e-5, atol=1e-6)
    z = torch.zeros(200000, device=device)
    ops.clip_noise(z, None, 0.0, 2.0, seed=123, offset=0)
    assert abs(z.mean().item()) < 0.05 and abs(z.std().item() - 2.0) < 0.05


@pytest.mark.parametrize("device", DEVICES)
def test_client_state(device):
    torch.manual_seed(12)
    n = 3001
    g, u, e = torch.randn(n), torch.randn(n), torch.randn(n)
    gd, ud, ed = g.clone().to(device), u.clone().to(device), e.clone().to(device)
    ops.client_state(gd, ud, ed, 0.9)
    u2 = 0.9 * u + g
    torch.testing.assert_close(ud.cpu(), u2)
    torch.testing.assert_close(ed.cpu(), e + u2)
    ops.zero_at(torch.tensor([0, 5]).to(device), ud, ed)
    assert ud.cpu()[0] == 0 and ed.cpu()[5] == 0


@pytest.mark.parametrize("device", DEVICES)
def test_augment_shapes_and_identity(device):
    torch.manual_seed(13)
    data = torch.randint(0, 256, (10, 8, 8, 3), dtype=torch.uint8)
    idx = torch.tensor([3, 7, 0])
    mean = torch.tensor([0.1, 0.2, 0.3])
    inv = torch.tensor([2.0, 3.0, 4.0])
    out = ops.augment_u8_nhwc(data.to(device), idx.to(device), 0, False, mean, inv, 0,
                              out_bf16=False).cpu()
    assert out.shape == (3, 3, 8, 8)
    ref = (data[idx].permute(0, 3, 1, 2).float() / 255 - mean.view(1, 3, 1, 1)) * inv.view(1, 3, 1, 1)
    torch.testing.assert_close(out, ref, rtol=1e-2, atol=2e-2)
    out2 = ops.augment_u8_nhwc(data.to(device), idx.to(device), 4, True, mean, inv, 99).float().cpu()
    assert out2.shape == (3, 3, 8, 8) and torch.isfinite(out2).all()


@pytest.mark.gpu
@pytest.mark.parametrize("d,c,r,nb", [(6568640, 500000, 5, 20), (1234567, 100003, 3, 1)])
@pytest.mark.parametrize("kernel", ["planned", "binned"])
def test_large_sketch_gpu_matches_cpu_backend(d, c, r, nb, kernel):
    """Full-size (ResNet-9 d) encode + query + top-k on the GPU vs the
    native CPU backend (deterministic row-parallel encode)."""
    g = torch.Generator().manual_seed(0)
    v = torch.randn(d, generator=g) * torch.rand(d, generator=g) ** 4
    w = torch.randn(d, generator=g)
    cpu = CSVec(d, c, r, device="cpu", numBlocks=nb)
    gpu = CSVec(d, c, r, device="cuda", numBlocks=nb, kernel=kernel)
    cpu.accumulateVec(v, 2.0, w, 1e-3)
    gpu.accumulateVec(v.cuda(), 2.0, w.cuda(), 1e-3)
    torch.testing.assert_close(gpu.table.cpu(), cpu.table, rtol=1e-4, atol=1e-4)
    gpu.accumulateVec(v.cuda(), 2.0, w.cuda(), 1e-3)  # scratch re-armed: second encode adds
    torch.testing.assert_close(gpu.table.cpu(), 2 * cpu.table, rtol=1e-4, atol=2e-4)
    est_c = cpu.query()
    est_g = gpu.like(cpu.table.cuda()).query()
    torch.testing.assert_close(est_g.cpu(), est_c)
    if kernel == "planned":  # atomic-free: bitwise reproducible
        t1 = gpu.like()
        t1.accumulateVec(v.cuda(), 1.0)
        t2 = gpu.like()
        t2.accumulateVec(v.cuda(), 1.0)
        assert torch.equal(t1.table, t2.table)
    ic, vc = ops.topk_abs(est_c, 50000)
    ig, vg = ops.topk_abs(est_g, 50000)
    assert torch.equal(ig.cpu(), ic) and torch.equal(vg.cpu(), vc)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,k", [((6, 16, 8, 8), 2), ((3, 64, 32, 32), 2), ((5, 32, 4, 4), 4)])
def test_relu_maxpool_fused_matches_torch(shape, k):
    from commefficient_amd.ops.nn import relu_maxpool
    torch.manual_seed(0)
    x = torch.randn(shape, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    x2 = x.detach().clone().requires_grad_(True)
    y = relu_maxpool(x, k)
    y2 = torch.nn.functional.max_pool2d(torch.relu(x2.float()), k)
    torch.testing.assert_close(y.float(), y2, rtol=0, atol=0)
    g = torch.randn_like(y2)
    y.backward(g.to(torch.bfloat16))
    y2.backward(g)
    torch.testing.assert_close(x.grad.float(), x2.grad.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("device", DEVICES)
def test_count_ge_random_matches_torch(device):
    g = torch.Generator().manual_seed(5)
    n = 300_001
    lm = torch.randint(-1, 200, (n,), generator=g, dtype=torch.int32)
    lm[: n // 2] = 7  # one hot bin (wave-aggregated path)
    thr = torch.unique(torch.randint(-1, 210, (90,), generator=g, dtype=torch.int32))
    cnt = ops.count_ge(lm.to(device), thr.to(device)).cpu()
    exp = torch.stack([(lm >= t).sum() for t in thr])
    assert cnt.tolist() == exp.tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("T", [1, 37, 1024])
def test_account_round_matches_reference(T):
    g = torch.Generator().manual_seed(T)
    d, C = 1_000_003, 5000
    lm = torch.randint(-1, 3000, (d,), generator=g, dtype=torch.int32)
    lm[: d // 3] = 17
    thr = torch.unique(torch.randint(-1, 3000, (4 * T,), generator=g, dtype=torch.int64))[:T]
    T = thr.numel()
    W = 3 * T
    inv = torch.randint(0, T, (W,), generator=g)
    inv[:T] = torch.arange(T)
    clients = torch.randperm(C, generator=g)[:W]
    cdl = torch.rand(C, generator=g, dtype=torch.float64)
    cul = torch.rand(C, generator=g, dtype=torch.float64)
    meta = torch.cat([thr, inv, clients]).cuda()
    cdl_d, cul_d = cdl.cuda(), cul.cuda()
    dl = ops.account_round(lm.cuda(), meta, T, W, cdl_d, cul_d, 123.0).cpu()
    cnt = torch.stack([(lm >= t).sum() for t in thr]).to(torch.float64) * 4
    exp = cnt[inv]
    assert torch.equal(dl, exp)
    cdl[clients] += exp
    cul[clients] += 123.0
    assert torch.equal(cdl_d.cpu(), cdl) and torch.equal(cul_d.cpu(), cul)


@pytest.mark.parametrize("device", DEVICES)
def test_apply_maintains_change_histogram(device):
    """sparse/dense apply keep hist[r+1] == #{i : last_mod[i] == r} exactly."""
    g = torch.Generator().manual_seed(11)
    d, cap = 200_003, 64
    w = torch.randn(d, generator=g).to(device)
    lm = torch.full((d,), -1, dtype=torch.int32, device=device)
    hist = torch.zeros(cap, dtype=torch.int32, device=device)
    hist[0] = d
    for r in range(6):
        if r % 3 == 2:
            delta = torch.randn(d, generator=g)
            delta[torch.rand(d, generator=g) < 0.3] = 0  # unchanged coordinates keep their stamp
            ops.dense_apply(w, delta.to(device), 0.1, None, lm, r, None, hist)
        else:
            idx = torch.randperm(d, generator=g)[:5000].sort().values
            vals = torch.randn(5000, generator=g)
            vals[:100] = 0
            ops.sparse_apply(w, idx.to(device), vals.to(device), 0.1, None, lm, r, None, hist)
        exp = torch.bincount(lm.cpu().long() + 1, minlength=cap).to(torch.int32)
        assert torch.equal(hist.cpu(), exp), r


@pytest.mark.parametrize("device", DEVICES)
def test_account_hist_matches_count(device):
    g = torch.Generator().manual_seed(3)
    d, C, W, cap = 500_001, 3000, 700, 4096
    lm = torch.randint(-1, 2500, (d,), generator=g, dtype=torch.int32)
    lm[: d // 4] = 9
    hist = torch.bincount(lm.long() + 1, minlength=cap).to(torch.int32)
    seen = torch.randint(0, 2600, (W,), generator=g)
    clients = torch.randperm(C, generator=g)[:W]
    cdl = torch.rand(C, generator=g, dtype=torch.float64)
    cul = torch.rand(C, generator=g, dtype=torch.float64)
    cdl_d, cul_d = cdl.to(device), cul.to(device)
    meta = torch.cat([seen, clients]).to(device)
    dl = ops.account_hist(hist.to(device), meta, W, cdl_d, cul_d, 7.0).cpu()
    exp = torch.stack([(lm >= s).sum() for s in seen]).to(torch.float64) * 4
    assert torch.equal(dl, exp)
    cdl[clients] += exp
    cul[clients] += 7.0
    assert torch.equal(cdl_d.cpu(), cdl) and torch.equal(cul_d.cpu(), cul)


@pytest.mark.gpu
@pytest.mark.parametrize("counts_dtype", [torch.int64, torch.float32])
def test_client_means_matches_index_add(counts_dtype):
    """Native per-client mean metrics vs the zeros + index_add + divide
    composition it replaces (fed_model.py _metric_sums)."""
    g = torch.Generator().manual_seed(0)
    W = 37
    counts = torch.randint(1, 9, (W,), generator=g)
    local = torch.rand(W, generator=g) < 0.6          # clients computed on this rank
    slot = torch.cat([torch.full((int(counts[w]),), w) for w in range(W) if local[w]])
    n = slot.numel()
    rows = [torch.randn(n, generator=g), (torch.rand(n, generator=g) < 0.5).float()]
    ref = torch.zeros(2, W)
    for i, r in enumerate(rows):
        ref[i].index_add_(0, slot, r)
    ref /= counts.float()
    out = torch.full((2, W), float("nan"), device="cuda")
    ops.client_means(out, [r.cuda() for r in rows], slot.cuda(), counts.to(counts_dtype).cuda())
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("r,nb", [(5, 1), (3, 7), (4, 1), (16, 2)])
def test_query_rows_matches_oracle(r, nb):
    """Row-wise two-pass query (the GPU path without a plan) vs the oracle."""
    torch.manual_seed(5)
    d, c = 30011, 997
    sk = CSVec(d, c, r, device="cuda", numBlocks=nb, kernel="binned")
    h, bo, bs = make_hashes(r, c, nb, 42)
    orc = OracleSketch(h, bo, bs, d, c, r, nb)
    v = torch.randn(d)
    sk.accumulateVec(v.cuda())
    orc.accumulate_vec(v)
    est = sk.query().cpu().double()
    torch.testing.assert_close(est, orc.query(), rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_planned_encode_overwrite_equals_zero_then_add():
    """overwrite=True writes every bucket (no separate zeroing pass) and equals
    zero + accumulate bitwise."""
    torch.manual_seed(9)
    d, c, r = 200003, 50000, 5
    sk = CSVec(d, c, r, device="cuda", numBlocks=3)
    assert sk._use_plan()
    v = torch.randn(d, device="cuda")
    w = torch.randn(d, device="cuda")
    sk.table.normal_()  # garbage that overwrite must not keep
    sk.accumulateVec(v, 0.5, w, 0.1, overwrite=True)
    ref = sk.like()
    ref.accumulateVec(v, 0.5, w, 0.1)
    assert torch.equal(sk.table, ref.table)


@pytest.mark.gpu
def test_topk_hint_never_changes_the_result():
    """topk_abs with a per-site lower-bound hint (csrc/topk.hip: pass 0 counts
    only keys >= the previous threshold / 2, a fill-in pass adds the rest when
    that was too few) returns bitwise the unhinted result over a sequence of
    vectors whose scale jumps up and down (stale-bound fallback), with ties,
    zeros, NaN-free sparse vectors and k close to n."""
    if not torch.cuda.is_available():
        pytest.skip("GPU only")
    g = torch.Generator().manual_seed(11)
    hint = ops.topk_hint(("test_hint", 0), "cuda")
    hint.zero_()
    seq = []
    for scale in (1.0, 1.3, 0.01, 100.0, 100.0, 0.5):
        seq.append((torch.randn(300000, generator=g) * scale, 5000))
    z = torch.zeros(300000)
    z[::97] = torch.randn(z[::97].numel(), generator=g)
    seq += [(z, 5000), (z, 3000), (torch.ones(300000), 7), (torch.randn(4096, generator=g), 4000)]
    for x, k in seq:
        a = ops.topk_abs(x.cuda(), k)
        b = ops.topk_abs(x.cuda(), k, hint)
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert int(hint.item()) != 0


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("has_w,has_u,has_e", [(True, True, True), (True, False, True), (False, True, False),
                                               (True, False, False), (False, False, False)])
def test_client_tail_matches_composition(device, has_w, has_u, has_e):
    """ops.client_tail == weight decay (axpby) + the n_i scale + client_state
    (fed_worker.py:184-230 after utils.py:257-258)."""
    from commefficient_amd import ops
    torch.manual_seed(3)
    n = 4096 + 8
    g = torch.randn(n, device=device)
    w = torch.randn(n, device=device) if has_w else None
    u = torch.randn(n, device=device) if has_u else None
    e = torch.randn(n, device=device) if has_e else None
    wd, scale, rho = 5e-4, 7.0, 0.9
    ref_g = g.double() + (wd * w.double() if has_w else 0.0)
    ref_g = ref_g * scale
    ref_u = rho * u.double() + ref_g if has_u else None
    t = ref_u if has_u else ref_g
    ref_e = e.double() + t if has_e else None
    g2, u2, e2 = g.clone(), (u.clone() if has_u else None), (e.clone() if has_e else None)
    ops.client_tail(g2, w, wd, scale, u2, e2, rho)
    if has_u:
        torch.testing.assert_close(u2.double(), ref_u, rtol=1e-6, atol=1e-5)
    if has_e:
        torch.testing.assert_close(e2.double(), ref_e, rtol=1e-6, atol=1e-5)
    if not has_u and not has_e:
        torch.testing.assert_close(g2.double(), ref_g, rtol=1e-6, atol=1e-5)


@pytest.mark.gpu
def test_fused_ce_padded_rows_vector_kernel():
    """Logits as rows of a buffer padded to a multiple of 8 columns (the native
    LM head's output; csrc/loss.hip ce_fwd_rowv_kernel): NaN pads are never
    read, loss / top-1 / gradient match the fp32 reference, the gradient comes
    back in the same row layout with zero pad columns, and the backward scale
    keeps them zero."""
    from commefficient_amd.ops.nn import cross_entropy_correct
    torch.manual_seed(1)
    V, B = 50257, 9
    ld = -(-V // 8) * 8
    buf = torch.full((B, ld), float("nan"), device="cuda").to(torch.bfloat16)
    buf[:, :V] = (torch.randn(B, V, device="cuda") * 3).to(torch.bfloat16)
    buf[3, 77] = buf[3, 4000] = 40.0  # a tie for the max: the lower index wins
    tgt = torch.tensor([5, -100, 50256, 77, 0, 123, 4000, 50255, 8], device="cuda")
    x = buf[:, :V].requires_grad_(True)
    loss, correct = cross_entropy_correct(x, tgt)
    w = torch.randn(B, device="cuda")
    (loss * w).sum().backward()
    xr = buf[:, :V].float().clone().requires_grad_(True)
    ref = F.cross_entropy(xr, tgt, ignore_index=-100, reduction="none")
    (ref * w).sum().backward()
    torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-4)
    keep = tgt >= 0
    torch.testing.assert_close(correct[keep], (xr.argmax(1) == tgt).float()[keep])
    assert correct[3] == 1.0
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=2e-4)
    # the op itself: the unit gradient in the logits' row layout, zero pad columns
    _, _, gunit = torch.ops.commeff.ce_fwd(buf[:, :V], tgt)
    assert gunit.stride(0) == ld
    pads = torch.as_strided(gunit, (B, ld - V), (ld, 1), gunit.storage_offset() + V)
    assert torch.all(pads == 0)
    torch.ops.commeff.scale_rows(gunit, w)
    assert torch.all(pads == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_fused_ce_ignore_rows_and_backward(dtype):
    """The GPT-2 LM loss at the labelled positions (train/losses.py): rows
    labelled -100 get zero loss and gradient; backward scales the unit
    gradient row by row in place (csrc/loss.hip scale_rows)."""
    from commefficient_amd.ops.nn import cross_entropy_correct
    torch.manual_seed(0)
    V = 50257
    logits = (torch.randn(7, V, device="cuda") * 3).to(dtype)
    tgt = torch.tensor([5, -100, 50256, 0, -100, 123, 4000], device="cuda")
    x = logits.clone().requires_grad_(True)
    loss, _ = cross_entropy_correct(x, tgt)
    w = torch.randn(7, device="cuda")
    (loss * w).sum().backward()
    xr = logits.float().clone().requires_grad_(True)
    ref = F.cross_entropy(xr, tgt, ignore_index=-100, reduction="none")
    (ref * w).sum().backward()
    torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-4)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol, atol=tol * 1e-2)
    assert x.grad[1].abs().max() == 0 and x.grad[4].abs().max() == 0
