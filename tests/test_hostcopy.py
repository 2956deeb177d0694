"""Per-round host staging (csrc/hostcopy.hip): a kernel reads the pinned
ring slot through its device mapping instead of a runtime blit copy."""
import numpy as np
import pytest
import torch

from commefficient_amd import _ext
from commefficient_amd.parallel import dist


def test_host_read_copy_cpu_semantics():
    src = torch.arange(37, dtype=torch.int64)
    dst = torch.empty(37, dtype=torch.int64)
    _ext.ops().host_read_copy(dst, src)
    assert torch.equal(dst, src)


@pytest.mark.gpu
@pytest.mark.parametrize("nbytes", [8, 40, 1000, 4096, 100_008, 1 << 20])
def test_host_read_copy_matches_source(nbytes):
    g = np.random.default_rng(nbytes)
    host = torch.from_numpy(g.integers(0, 255, nbytes, dtype=np.uint8)).pin_memory()
    dst = torch.full((nbytes,), 7, dtype=torch.uint8, device="cuda")
    _ext.ops().host_read_copy(dst, host)
    torch.cuda.synchronize()
    assert torch.equal(dst.cpu(), host)


@pytest.mark.gpu
def test_pinned_ring_slots_stream_ordered():
    """Many rounds through the ring: every device buffer holds its own round's
    array although the slots are reused (event-guarded) and the reads run
    asynchronously behind queued work."""
    outs, refs = [], []
    x = torch.randn(2048, 2048, device="cuda")
    for r in range(100):
        if r % 10 == 0:
            x = x @ x.t() / 2048.0  # keep the stream busy so the reads queue up
        a = np.arange(r, r + 1000, dtype=np.int64) * 3
        outs.append(dist.h2d(a, "cuda"))
        refs.append(a)
    torch.cuda.synchronize()
    for o, a in zip(outs, refs):
        assert np.array_equal(o.cpu().numpy(), a)
    step = torch.zeros(2, dtype=torch.int32, device="cuda")
    dist.h2d_into(step, np.array([5, 9], dtype=np.int32))
    torch.cuda.synchronize()
    assert step.tolist() == [5, 9]
