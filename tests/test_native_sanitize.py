"""Host-code sanitizers: the C++ runtime's paged-KV block pool
under AddressSanitizer + UBSan and ThreadSanitizer, driven by a multi-threaded
random-lifecycle stress test (csrc/runtime/tests/pool_stress.cpp)."""
import shutil
import subprocess

import pytest

from loqa_hub_amd._native.build import build_sanitized

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")


@pytest.mark.parametrize("kind", ["address,undefined", "thread"])
def test_block_pool_under_sanitizer(kind, tmp_path):
    try:
        exe = build_sanitized(kind, str(tmp_path))
    except RuntimeError as e:
        if "cannot find" in str(e) or "No such file" in str(e):
            pytest.skip(f"sanitizer runtime unavailable: {e}")
        raise
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "0 errors" in r.stdout
