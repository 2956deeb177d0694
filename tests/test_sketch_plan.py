"""The planned (atomic-free) Count-Sketch: plan invariants and a pure-torch
simulation of the four kernels of csrc/sketch_planned.hip (P1/P2 encode,
Q1/Q2 query) driven by the plan, checked against the native CPU encode /
query.  Runs on CPU (the plan builder's hash op has a CPU twin); the GPU
kernels themselves are checked in test_ops.py."""
import pytest
import torch

from commefficient_amd._ext import ops as _ops
from commefficient_amd.ops import CSVec
from commefficient_amd.ops.sketch_plan import build_plan


def _u16(t):
    return t.to(torch.int64) & 0xFFFF


def _plan(d, c, r, nb, seed=3):
    sk = CSVec(d, c, r, device="cpu", numBlocks=nb, seed=seed)
    geo = [int(v) for v in _ops().plan_geometry(d, r, c)]
    plan = build_plan(sk.hashes, sk.blk_off, sk.blk_sign, sk.numBlocks, d, r, c, "cpu")
    return sk, geo, plan


def _gpos_of_slots(geo, plan, d, r):
    """global (segment-order) position of every entry (i, j), via the runs"""
    tile, nt, chunk, nch = geo[:4]
    src_info, _, _, _, base, off, _, _ = plan[:8]
    gpos = torch.empty(d * r, dtype=torch.int64)
    for ch in range(nch):
        i0, i1 = ch * chunk, min(d, (ch + 1) * chunk)
        s = _u16(src_info[i0 * r:i1 * r])
        o = off[ch].to(torch.int64)
        t = torch.searchsorted(o[1:], s, right=True)
        gpos[i0 * r:i1 * r] = base[ch].to(torch.int64)[t] + s - o[t]
    return gpos


def _simulate_encode(geo, plan, vec, r, c):
    tile, nt, chunk, nch = geo[:4]
    src_info, _, perm, csr, _, _, seg, _ = plan[:8]
    p2_src, p2_pos = plan[8].long(), plan[9].long()
    d = vec.numel()
    # P1: chunk-major stage images
    cm = (torch.arange(d) // chunk).repeat_interleave(r) * (chunk * r) + _u16(src_info)
    vals = torch.zeros(nch * chunk * r, dtype=torch.float64)
    vals[cm] = vec.double().repeat_interleave(r)
    # P2: per tile, every chunk's run scattered to its bucket-order slot
    pl = _u16(perm)
    csr = csr.to(torch.int64)
    seg = seg.to(torch.int64)
    table = torch.zeros(r * c, dtype=torch.float64)
    for t in range(nt):
        S = torch.zeros(int(seg[t + 1] - seg[t]), dtype=torch.float64)
        for ch in range(nch):
            a, ln = int(p2_src[t, ch]), int(p2_pos[t, ch + 1] - p2_pos[t, ch])
            x = torch.arange(a, a + ln)
            S[pl[x] & 0x7FFF] = torch.where((pl[x] & 0x8000) != 0, -vals[x], vals[x])
        g1 = min((t + 1) * tile, r * c)
        for gb in range(t * tile, g1):
            table[gb] = S[csr[gb] - seg[t]:csr[gb + 1] - seg[t]].sum()
    return table.view(r, c)


def _simulate_query(geo, plan, table, d, r):
    tile, nt, chunk, nch = geo[:4]
    _, ent_info, _, _, _, _, seg, _ = plan[:8]
    n = d * r
    seg = seg.to(torch.int64)
    tile_of_e = torch.searchsorted(seg[1:], torch.arange(n), right=True)
    info = _u16(ent_info)
    flat = table.reshape(-1)
    v = flat[tile_of_e * tile + (info & (tile - 1))]
    vals = torch.where((info & 0x8000) != 0, -v, v)                                # Q1
    per = vals[_gpos_of_slots(geo, plan, d, r)].view(d, r)                          # Q2
    return per.sort(dim=1).values[:, (r - 1) // 2]


@pytest.mark.parametrize("d,c,r,nb", [(20000, 900, 5, 1), (30011, 2003, 3, 4), (9000, 700, 1, 1),
                                      (50000, 4000, 5, 20)])
def test_plan_invariants_and_simulated_kernels(d, c, r, nb):
    sk, geo, plan = _plan(d, c, r, nb)
    assert geo and plan is not None
    tile, nt, chunk, nch = geo[:4]
    src_info, ent_info, perm, csr, base, off, seg, vals = plan[:8]
    n = d * r
    assert nt * tile >= r * c and nch * chunk >= d
    assert int(seg[-1]) == n and int(csr[-1]) == n
    assert int((seg[1:] - seg[:-1]).max()) <= 32767
    # every chunk's stage slots are a permutation of 0..len-1
    for ch in range(nch):
        i0, i1 = ch * chunk, min(d, (ch + 1) * chunk)
        s = _u16(src_info[i0 * r:i1 * r])
        assert torch.equal(s.sort().values, torch.arange((i1 - i0) * r))
    # global positions are a permutation of 0..n-1
    assert torch.equal(_gpos_of_slots(geo, plan, d, r).sort().values, torch.arange(n))
    # P2's tile-major run metadata agrees with the chunk-major one
    p2_src, p2_pos = plan[8].long(), plan[9].long()
    offl = off.long()
    assert torch.equal(p2_pos[:, 1:] - p2_pos[:, :-1], (offl[:, 1:] - offl[:, :-1]).t())
    assert torch.equal(p2_src, torch.arange(nch).view(1, -1) * chunk * r + offl[:, :nt].t())
    assert torch.equal(p2_pos[:, -1], seg[1:].long() - seg[:-1].long())
    g = torch.Generator().manual_seed(0)
    vec = torch.randn(d, generator=g)
    ref = sk.like()
    ref.accumulateVec(vec)
    sim = _simulate_encode(geo, plan, vec, r, c)
    torch.testing.assert_close(sim.float(), ref.table, rtol=1e-5, atol=1e-5)
    est = _simulate_query(geo, plan, ref.table, d, r)
    assert torch.equal(est, sk.like(ref.table).query())


def _simulate_encode_dense(geo, plan, vec, r, c):
    """Dense plan: P1 as the exact plan, P2 adds each run entry (chunk-major
    in-tile bucket | sign in plan slot 2) into its tile."""
    tile, nt, chunk, nch = geo[:4]
    src_info, _, cm_info = plan[:3]
    p2_src, p2_pos = plan[8].long(), plan[9].long()
    d = vec.numel()
    cm = (torch.arange(d) // chunk).repeat_interleave(r) * (chunk * r) + _u16(src_info)
    vals = torch.zeros(nch * chunk * r, dtype=torch.float64)
    vals[cm] = vec.double().repeat_interleave(r)
    info = _u16(cm_info)
    table = torch.zeros(nt * tile, dtype=torch.float64)
    for t in range(nt):
        for ch in range(nch):
            a, ln = int(p2_src[t, ch]), int(p2_pos[t, ch + 1] - p2_pos[t, ch])
            x = torch.arange(a, a + ln)
            sv = torch.where((info[x] & 0x8000) != 0, -vals[x], vals[x])
            table.index_add_(0, t * tile + (info[x] & (tile - 1)), sv)
    return table[:r * c].view(r, c)


@pytest.mark.parametrize("d,c,r,nb", [(2_000_000, 8000, 5, 20), (300_000, 1000, 3, 1)])
def test_dense_plan_for_many_entries_per_bucket(d, c, r, nb):
    """~250 entries per bucket (GPT-2's ratio): the exact plan's segments do
    not fit in LDS, the dense plan (LDS-atomic encode P2) takes over; the
    query kernels (Q1/Q2) are the exact plan's."""
    sk, geo, plan = _plan(d, c, r, nb)
    assert geo and geo[4] == 1 and geo[0] == 8192 and plan is not None
    g = torch.Generator().manual_seed(0)
    vec = torch.randn(d, generator=g)
    ref = sk.like()
    ref.accumulateVec(vec)
    sim = _simulate_encode_dense(geo, plan, vec, r, c)
    torch.testing.assert_close(sim.float(), ref.table, rtol=1e-4, atol=1e-4)
    est = _simulate_query(geo, plan, ref.table, d, r)
    assert torch.equal(est, sk.like(ref.table).query())


@pytest.mark.gpu
def test_dense_planned_gpu_kernels_match_cpu():
    d, c, r, nb = 3_000_001, 12007, 5, 20
    cpu = CSVec(d, c, r, device="cpu", numBlocks=nb, seed=5)
    gpu = CSVec(d, c, r, device="cuda", numBlocks=nb, seed=5, kernel="planned")
    assert gpu._use_plan()
    g = torch.Generator().manual_seed(1)
    v, w = torch.randn(d, generator=g), torch.randn(d, generator=g)
    cpu.accumulateVec(v, 0.5, w, 1e-2)
    gpu.accumulateVec(v.cuda(), 0.5, w.cuda(), 1e-2, overwrite=True)
    torch.testing.assert_close(gpu.table.cpu(), cpu.table, rtol=1e-4, atol=1e-4)
    gpu.accumulateVec(v.cuda(), 0.5, w.cuda(), 1e-2)  # += path
    torch.testing.assert_close(gpu.table.cpu(), 2 * cpu.table, rtol=1e-4, atol=1e-4)
    assert torch.equal(gpu.like(cpu.table.cuda()).query().cpu(), cpu.query())


@pytest.mark.gpu
@pytest.mark.parametrize("d,c,r,nb", [(20000, 900, 5, 1), (30011, 2003, 3, 4), (9000, 700, 1, 1),
                                      (50000, 4000, 5, 20), (123457, 10007, 4, 2)])
def test_planned_gpu_kernels_match_cpu(d, c, r, nb):
    cpu = CSVec(d, c, r, device="cpu", numBlocks=nb, seed=5)
    gpu = CSVec(d, c, r, device="cuda", numBlocks=nb, seed=5, kernel="planned")
    assert gpu._use_plan()
    g = torch.Generator().manual_seed(1)
    v, w = torch.randn(d, generator=g), torch.randn(d, generator=g)
    cpu.accumulateVec(v, 0.5, w, 1e-2)
    gpu.accumulateVec(v.cuda(), 0.5, w.cuda(), 1e-2)
    torch.testing.assert_close(gpu.table.cpu(), cpu.table, rtol=1e-5, atol=1e-5)
    assert torch.equal(gpu.like(cpu.table.cuda()).query().cpu(), cpu.query())


@pytest.mark.gpu
def test_dense_fixed_point_encode_deterministic_and_accurate():
    """The dense plan's 64-bit fixed-point encode P2: bitwise identical on
    repeats, at least as close to a float64 table as fp32 accumulation, and
    NaN-poisoned by a NaN input."""
    d, c, r, nb = 3_000_001, 12007, 5, 20
    gpu = CSVec(d, c, r, device="cuda", numBlocks=nb, seed=5, kernel="planned")
    assert gpu._use_plan() and len(gpu._plan()) == 11
    g = torch.Generator().manual_seed(2)
    # heavy-tailed values: a few large coordinates among many small ones
    v = torch.randn(d, generator=g) * torch.exp(3 * torch.randn(d, generator=g))
    vc = v.cuda()
    gpu.accumulateVec(vc, 1.0, overwrite=True)
    t1 = gpu.table.clone()
    for _ in range(3):
        gpu.accumulateVec(vc, 1.0, overwrite=True)
        assert torch.equal(gpu.table, t1)
    cpu = CSVec(d, c, r, device="cpu", numBlocks=nb, seed=5)
    cpu.accumulateVec(v, 1.0)
    err = (t1.cpu().double() - cpu.table.double()).abs().max().item()
    assert err <= 1e-4 * cpu.table.abs().max().item()
    bad = vc.clone()
    bad[12345] = float("nan")
    gpu.accumulateVec(bad, 1.0, overwrite=True)
    assert torch.isnan(gpu.table).all()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("shape", [(6568640, 5, 500000), (2_000_003, 5, 100_000)])
def test_sharded_unsketch_equals_replicated_gpu(world, shape):
    """Each rank's shard query + top-k, merged over the ranks' candidate lists,
    is bitwise the replicated unsketch (same indices, same values)."""
    import torch
    from commefficient_amd.ops import CSVec
    d, r, c = shape
    k = 50000
    torch.manual_seed(0)
    sk = CSVec(d, c, r, device="cuda", numBlocks=20, kernel="planned")
    v = torch.randn(d, device="cuda") * torch.rand(d, device="cuda").pow(8)
    sk.accumulateVec(v)
    ref_i, ref_v = sk.unsketch_sparse(k)
    b = sk.shard_bounds(world)
    assert b is not None and b[0] == 0 and b[-1] == d
    packs = [sk.unsketch_shard(k, q, world, b) for q in range(world)]
    idx, vals = CSVec.merge_shards(torch.cat([p.view(1, -1) for p in packs]), world, k)
    assert torch.equal(idx, ref_i)
    assert torch.equal(vals, ref_v)
