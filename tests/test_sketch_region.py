"""Region-permutation Count Sketch (ops/sketch_region.py, csrc/sketch_region.hip).

CPU: the family's structure (bijective inside a chunk, ~1/c pairwise collision
rate per row, one coordinate of each chunk per bucket of its region), CSVec
API semantics on the CPU implementation, and heavy-hitter recovery no worse
than the multiply-shift csvec family.  GPU: the HIP encode / query / zeroing
against the CPU implementation (query and zeroing bitwise, encode to fp32
summation order), bitwise run-to-run determinism, chunk-range (sharded)
queries, and the sharded unsketch equal to the replicated one."""
import numpy as np
import pytest
import torch

from commefficient_amd.ops import CSVec
from commefficient_amd.ops import sketch_region
from commefficient_amd.ops.sketch_region import RegionHash, collision_rate, region_geometry

GEOMS = [(1000, 100, 5), (20000, 3000, 5), (50001, 5000, 3), (7, 10, 1), (123457, 20000, 4)]


@pytest.mark.parametrize("d,c,r", GEOMS)
def test_region_structure(d, c, r):
    h = RegionHash(d, c, r, seed=3)
    b, s = h.dense()
    assert b.shape == (r, d) and int(b.min()) >= 0 and int(b.max()) < h.G * h.g * h.m <= c
    assert set(np.unique(s.numpy())) <= {-1.0, 1.0}
    for q in range(h.nch):
        lo, hi = q * h.m, min(d, (q + 1) * h.m)
        for j in range(r):
            bq = b[j, lo:hi]
            assert bq.unique().numel() == hi - lo  # bijective inside a chunk
            assert int(bq.min()) // h.m == int(bq.max()) // h.m == int(h.region[j, q])
    # chunks dealt evenly over the groups; a chunk's regions in its group;
    # a batch's chunks in distinct regions of every row
    assert np.ptp(np.bincount(h.group, minlength=h.G)) <= 1
    assert np.array_equal(h.region // h.g, np.broadcast_to(h.group, h.region.shape))
    for x in range(h.G):
        members = h.lists[h.goffs[x]:h.goffs[x + 1]]
        assert np.all(h.group[members] == x)
        for t0 in range(0, len(members), h.W):
            batch = members[t0:t0 + h.W]
            for j in range(r):
                assert len(np.unique(h.region[j, batch])) == len(batch)


def test_region_geometry_choices():
    assert region_geometry(500000, 5) == (64, 32, 244, 32)
    assert region_geometry(100, 5) == (64, 1, 1, 1)
    assert region_geometry(10, 1) == (10, 1, 1, 1)
    for c, r in ((10 ** 6, 16), (3000, 5), (999983, 7)):
        m, g, G, W = region_geometry(c, r)
        assert r * g * m * 4 <= 160 * 1024 and G * g * m <= c and W <= g and (W <= 16 or W == 32)


def test_collision_rate_is_uniform_like():
    d, c, r = 200000, 20000, 5
    h = RegionHash(d, c, r, seed=1)
    rate = collision_rate(h, pairs=400000)
    assert abs(rate - 1.0 / c) < 0.3 / c, (rate, 1.0 / c)


def test_csvec_region_linearity_and_exact_recovery():
    d, c, r = 30000, 4000, 5
    torch.manual_seed(0)
    a, b = torch.randn(d), torch.randn(d)
    s1 = CSVec(d, c, r, kernel="region")
    s2 = s1.like()
    s12 = s1.like()
    s1.accumulateVec(a)
    s2.accumulateVec(b)
    s12.accumulateVec(a, 1.0, b, 1.0)
    torch.testing.assert_close(s12.table, s1.table + s2.table, rtol=1e-5, atol=1e-5)
    # a sparse vector is recovered exactly unless two of its entries collide in
    # >= 3 of 5 rows (they cannot inside one chunk)
    v = torch.zeros(d)
    hot = torch.tensor([5, 17, 999, 2047, 2048, 29999])
    v[hot] = torch.tensor([3.0, -2.0, 1.5, 7.0, -4.0, 0.5])
    sk = CSVec(d, c, r, kernel="region")
    sk.accumulateVec(v)
    est = sk.query()
    torch.testing.assert_close(est[hot], v[hot])
    idx, vals = sk.unsketch_sparse(4)
    assert sorted(idx.tolist()) == [5, 17, 2047, 2048]


def test_csvec_region_overwrite_and_zero():
    d, c, r = 9000, 1000, 3
    sk = CSVec(d, c, r, kernel="region")
    sk.table.fill_(123.0)
    v = torch.randn(d)
    sk.accumulateVec(v, overwrite=True)
    ref = CSVec(d, c, r, kernel="region")
    ref.accumulateVec(v)
    assert torch.equal(sk.table, ref.table)
    other = ref.table.clone() + 1.0
    idx = torch.tensor([0, 4000, 8999])
    vals = torch.tensor([1.0, 0.0, -2.0])
    ref.zero_heavy_hitters(idx, vals, other)
    b = ref.region.buckets_of(idx)
    for j in range(r):
        for t in (0, 2):  # the nonzero entries' cells, in both tables
            assert ref.table[j, b[j, t]] == 0 and other[j, b[j, t]] == 0


def test_heavy_hitter_recall_matches_csvec_family():
    # heavy-tailed vector: top-k recall of the region family within a few
    # points of the multiply-shift (csvec layout) family at the same geometry
    d, c, r, k = 200000, 20000, 5, 1000
    g = torch.Generator().manual_seed(7)
    v = torch.randn(d, generator=g) * 0.01
    hot = torch.randperm(d, generator=g)[:k]
    v[hot] += torch.randn(k, generator=g).sign() * (0.5 + torch.rand(k, generator=g))
    true = set(torch.topk(v.abs(), k).indices.tolist())
    recall = {}
    for kern in ("region", "planned"):
        sk = CSVec(d, c, r, kernel=kern, numBlocks=20)
        sk.accumulateVec(v)
        idx, _ = sk.unsketch_sparse(k)
        recall[kern] = len(true & set(idx.tolist())) / k
    assert recall["region"] >= recall["planned"] - 0.02, recall
    assert recall["region"] > 0.95, recall


# ------------------------------------------------------------------ GPU
GPU_GEOMS = [(1000, 100, 5), (6568640, 500000, 5), (50001, 5000, 3), (123457, 20000, 4),
             (2000003, 500000, 5)]


def _pair(d, c, r, seed=11):
    cpu = CSVec(d, c, r, kernel="region", seed=seed)
    gpu = CSVec(d, c, r, device="cuda", kernel="region", seed=seed)
    return cpu, gpu


@pytest.mark.gpu
@pytest.mark.parametrize("d,c,r", GPU_GEOMS)
def test_region_gpu_encode_query_zero_match_cpu(d, c, r):
    torch.manual_seed(d % 1000)
    v = torch.randn(d)
    w = torch.randn(d)
    cpu, gpu = _pair(d, c, r)
    cpu.accumulateVec(v, 0.5, w, 0.01)
    gpu.table.fill_(7.0)  # overwrite ignores stale contents, incl. the unused tail
    gpu.accumulateVec(v.cuda(), 0.5, w.cuda(), 0.01, overwrite=True)
    torch.testing.assert_close(gpu.table.cpu(), cpu.table, rtol=1e-5, atol=1e-5)
    gpu.accumulateVec(v.cuda())  # accumulate (+=)
    cpu.accumulateVec(v)
    torch.testing.assert_close(gpu.table.cpu(), cpu.table, rtol=1e-5, atol=1e-5)
    # query / zeroing of one shared table: bitwise
    gpu.table.copy_(cpu.table)
    assert torch.equal(gpu.query().cpu(), cpu.query())
    k = min(1000, d // 3)
    idx = torch.randperm(d)[:k].sort().values
    vals = torch.randn(k)
    vals[::4] = 0
    other_c = cpu.table.clone()
    other_g = other_c.cuda()
    cpu.zero_heavy_hitters(idx, vals, other_c)
    gpu.zero_heavy_hitters(idx.cuda(), vals.cuda(), other_g)
    assert torch.equal(gpu.table.cpu(), cpu.table)
    assert torch.equal(other_g.cpu(), other_c)


@pytest.mark.gpu
def test_region_gpu_deterministic_and_sharded():
    d, c, r = 6568640, 500000, 5
    v = torch.randn(d, device="cuda")
    w = torch.randn(d, device="cuda")
    a = CSVec(d, c, r, device="cuda", kernel="region")
    b = a.like()
    a.accumulateVec(v, 0.3, w, 1e-3, overwrite=True)
    b.accumulateVec(v, 0.3, w, 1e-3, overwrite=True)
    assert torch.equal(a.table, b.table)
    full = a.query()
    k = 50000
    ref_idx, ref_vals = a.unsketch_sparse(k)
    for world in (2, 3, 8):
        bounds = a.shard_bounds(world)
        packs = [a.unsketch_shard(k, q, world, bounds) for q in range(world)]
        for q in range(world):
            lo, hi = bounds[q], bounds[q + 1]
            qb = a.region.chunk_bounds(world)
            est = sketch_region.query(a.region, a.table, qb[q], qb[q + 1])
            assert torch.equal(est[lo:hi], full[lo:hi])
        idx, vals = CSVec.merge_shards(torch.stack(packs).view(world, 2 * k), world, k)
        assert torch.equal(idx, ref_idx) and torch.equal(vals, ref_vals)


@pytest.mark.gpu
@pytest.mark.parametrize("world,rank,et", [(8, 3, "virtual"), (4, 0, "none"), (2, 1, "virtual")])
def test_region_gpu_group_shard_topk_matches_cpu(world, rank, et):
    """The sharded server's query + top-k on one rank's group-major shard
    (G / world groups; with few groups the query runs several blocks per group
    after a separate momentum pass, csrc/sketch_region.hip bpg) equals the CPU
    path: momentum / error feedback bitwise, and the same (index, value) list."""
    d, c, r, k = 6568640, 500000, 5, 50000
    h = RegionHash(d, c, r, seed=5)
    g = torch.Generator().manual_seed(world * 10 + rank)
    E, V, G = (torch.randn(r, c, generator=g) for _ in range(3))
    Gp = h.shard_groups(world)
    g0 = rank * Gp
    shard = lambda t: h.group_major(t, world)[g0:g0 + Gp].contiguous()  # noqa: E731
    Ec, Vc, Gc = shard(E), shard(V), shard(G)
    Eg, Vg, Gg = Ec.cuda(), Vc.cuda(), Gc.cuda()
    src_c, src_g = (Ec, Eg) if et == "virtual" else (Vc, Vg)
    li, lv, cmap = sketch_region.topk(h, src_g, k, None, mom=(Vg, Gg, 0.9, 0.01, et), g0=g0)
    # momentum / error feedback (GPU: fmaf, CPU: two roundings)
    sketch_region.topk(h, src_c, k, None, mom=(Vc, Gc, 0.9, 0.01, et), g0=g0)
    torch.testing.assert_close(Vg.cpu(), Vc, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(Eg.cpu(), Ec, rtol=1e-6, atol=1e-6)
    # the selection on the GPU's updated shard: the CPU query + top-k, bitwise
    ci, cv, _ = sketch_region.topk(h, src_g.cpu(), k, None, g0=g0)
    gi = cmap.long()[li // h.m] * h.m + li % h.m  # compact -> global coordinates
    assert torch.equal(gi.cpu(), ci)
    assert torch.equal(lv.cpu(), cv)


def test_hot_chunks_are_filtered_by_the_median():
    # whole chunks of large values (a layer with big gradients) plus heavy
    # hitters elsewhere: independent per-row region assignments keep the
    # heavy hitters' median estimates as clean as the csvec family's; a shared
    # assignment (every row polluted by the same hot region-mates) measured
    # a 16x larger median error here
    d, c, r = 400000, 40000, 5
    g = torch.Generator().manual_seed(3)
    v = torch.randn(d, generator=g) * 1e-3
    h = RegionHash(d, c, r, seed=1)
    hot = torch.randperm(h.nch, generator=g)[: h.nch // 10].tolist()
    cold = torch.ones(d, dtype=torch.bool)
    for q in hot:
        lo, hi = q * h.m, min(d, (q + 1) * h.m)
        v[lo:hi] = torch.randn(hi - lo, generator=g)
        cold[lo:hi] = False
    cand = torch.nonzero(cold).view(-1)
    heavy = cand[torch.randperm(len(cand), generator=g)[:300]]
    v[heavy] = 3.0 * torch.randn(300, generator=g).sign()
    err = {}
    for kern in ("region", "planned"):
        sk = CSVec(d, c, r, kernel=kern, seed=1, numBlocks=20)
        sk.accumulateVec(v)
        err[kern] = float((sk.query()[heavy] - v[heavy]).abs().median())
    assert err["region"] <= 2 * err["planned"] + 0.005, err


@pytest.mark.gpu
def test_region_fused_topk_matches_query_then_topk():
    # the fused unsketch (query + first top-k histogram in one kernel) selects
    # bitwise what query() followed by the standalone top-k selects, with and
    # without a (stale, too high, too low) hint, on full and chunk ranges
    from commefficient_amd import ops as O
    d, c, r, k = 6568640, 500000, 5, 50000
    sk = CSVec(d, c, r, device="cuda", kernel="region")
    sk.accumulateVec(torch.randn(d, device="cuda") * torch.rand(d, device="cuda") ** 4, overwrite=True)
    est = sk.query()
    ref = O.topk_abs(est, k)
    for hv in (None, 0, 0x3f000000, 0x7f000000):
        hint = None if hv is None else torch.full((1,), hv, dtype=torch.int32, device="cuda")
        idx, vals = sketch_region.topk(sk.region, sk.table, k, hint)
        assert torch.equal(idx, ref[0]) and torch.equal(vals, ref[1])
    qb = sk.region.chunk_bounds(4)
    lo, hi = qb[1] * sk.region.m, qb[2] * sk.region.m
    ref2 = O.topk_abs(est[lo:hi].contiguous(), k)
    idx, vals = sketch_region.topk(sk.region, sk.table, k, None, qb[1], qb[2])
    assert torch.equal(idx, ref2[0]) and torch.equal(vals, ref2[1])


@pytest.mark.gpu
def test_region_encode_zero_vec_clears_the_vector():
    d, c, r = 2000003, 500000, 5
    v = torch.randn(d, device="cuda")
    w = torch.randn(d, device="cuda")
    a = CSVec(d, c, r, device="cuda", kernel="region")
    b = a.like()
    vv = v.clone()
    a.accumulateVec(v, 0.5, w, 1e-3, overwrite=True)
    assert b.accumulateVec(vv, 0.5, w, 1e-3, overwrite=True, zero_vec=True)
    assert torch.equal(a.table, b.table) and int(vv.count_nonzero()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("et", ["virtual", "none"])
def test_region_fused_momentum_matches_separate(et):
    # the server momentum applied inside the query's staging == momentum_ef
    # then the unsketch: selection, V and E bitwise, also for a chunk range
    # (the momentum still covers every region)
    from commefficient_amd import ops as O
    d, c, r, k = 6568640, 500000, 5, 50000
    base = CSVec(d, c, r, device="cuda", kernel="region")
    torch.manual_seed(5)
    V0, E0, G = (torch.randn(r, c, device="cuda") for _ in range(3))
    for q0, q1 in ((0, -1), tuple(base.region.chunk_bounds(3)[1:3])):
        V1, E1 = V0.clone(), E0.clone()
        O.momentum_ef(V1.view(-1), E1.view(-1) if et == "virtual" else None, G.view(-1), 0.9, 0.01, et)
        src1 = E1 if et == "virtual" else V1
        ref = sketch_region.topk(base.region, src1, k, None, q0, q1)
        V2, E2 = V0.clone(), E0.clone()
        src2 = E2 if et == "virtual" else V2
        got = sketch_region.topk(base.region, src2, k, None, q0, q1, mom=(V2, G, 0.9, 0.01, et))
        assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
        m = base.region.G * base.region.g * base.region.m  # the unused tail is never touched
        assert torch.equal(V2[:, :m], V1[:, :m]) and torch.equal(E2[:, :m], E1[:, :m])


@pytest.mark.gpu
@pytest.mark.parametrize("d,c,r", GPU_GEOMS)
def test_region_zero_apply_matches_separate_steps(d, c, r):
    """cs_region_zero_apply = zero_heavy_hitters + sparse_apply (bitwise),
    incl. the last-changed stamps and the change histogram."""
    from commefficient_amd import ops as cops
    torch.manual_seed(d % 997)
    _, gpu = _pair(d, c, r)
    gpu.table.copy_(torch.randn(gpu.table.shape))
    other = torch.randn(gpu.table.shape, device="cuda")
    k = min(1000, d // 3)
    idx = torch.randperm(d)[:k].sort().values.cuda()
    vals = torch.randn(k, device="cuda")
    vals[::4] = 0
    w = torch.randn(d, device="cuda")
    last_mod = torch.randint(-1, 3, (d,), dtype=torch.int32, device="cuda")
    hist = torch.zeros(64, dtype=torch.int32, device="cuda")
    lr_vec = torch.rand(d, device="cuda")
    for lrv in (None, lr_vec):
        t1, t2, w1, lm1, h1 = gpu.table.clone(), other.clone(), w.clone(), last_mod.clone(), hist.clone()
        sep = gpu.like(t1)
        sep.zero_heavy_hitters(idx, vals, t2)
        cops.sparse_apply(w1, idx, vals, 0.3, lrv, lm1, 5, None, h1)
        t3, t4, w2, lm2, h2 = gpu.table.clone(), other.clone(), w.clone(), last_mod.clone(), hist.clone()
        fused = gpu.like(t3)
        assert fused.zero_heavy_hitters_apply(idx, vals, t4, w2, 0.3, lrv, lm2, 5, h2)
        for a, b in ((t1, t3), (t2, t4), (w1, w2), (lm1, lm2), (h1, h2)):
            assert torch.equal(a, b)
