"""Launch status checks (csrc/launch.h): a kernel launch the runtime rejects
raises a RuntimeError that names the kernel, its grid, block and dynamic LDS
bytes, instead of silently leaving its outputs unwritten."""
import pytest
import torch

from commefficient_amd import _ext


def _probe(out, lds):
    _ext.load()
    torch.ops.commeff.launch_probe(out, lds)


@pytest.mark.skipif(torch.cuda.is_available(), reason="the no-device path (CPU container)")
def test_launch_failure_raises_without_device():
    with pytest.raises(RuntimeError) as ei:
        _probe(torch.zeros(1, dtype=torch.int32), 256)
    msg = str(ei.value)
    assert "launch_probe_kernel" in msg and "dynamic LDS 256 bytes" in msg, msg
    assert "block (64, 1, 1)" in msg, msg


@pytest.mark.gpu
def test_impossible_lds_request_raises_gpu():
    out = torch.zeros(1, dtype=torch.int32, device="cuda")
    _probe(out, 1024)  # a valid launch runs
    torch.cuda.synchronize()
    assert int(out.item()) == 64
    with pytest.raises(RuntimeError) as ei:
        _probe(out, 200 * 1024)  # more LDS than a CU has (160 KB)
    msg = str(ei.value)
    assert "launch_probe_kernel" in msg and "dynamic LDS 204800 bytes" in msg, msg
    # the sticky status was cleared: the next (valid) launch and a PyTorch op run
    out.zero_()
    _probe(out, 1024)
    torch.cuda.synchronize()
    assert int(out.item()) == 64
