"""AddressSanitizer run of the C ABI's host code (tools/asan: every csrc/*.hip built with host-side
-fsanitize=address and linked into abi_host_check.cpp, which sweeps the dispatch planners and the
argument checks; nothing is launched). CPU only; skipped where hipcc is absent."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which("make") is None,
                    reason="hipcc / make not available")
def test_abi_host_code_under_asan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools", "asan"), "run",
                        "-j8"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "asan host check OK" in r.stdout
