"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer run of the CPU codec
kernels (SURVEY.md §5.2 "race detection and sanitizers"): scripts/sanitize_host.sh
builds tests/native/cpu_ops_harness.cpp + csrc/cpu_ops.cpp with
-fsanitize=address,undefined and runs boundary geometries against brute-force
references.  GPU ASan is unavailable on the MI355X pool; device kernels are
covered by the fp32-reference and determinism tests."""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_cpu_codec_kernels_clean_under_asan_ubsan():
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "sanitize_host.sh"), d],
                           capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "OK (0 failures)" in r.stdout
