"""CPU: the C ABI's host code under AddressSanitizer + UBSan.

`make -C <pkg>/csrc sanitize` builds the library's sources with host-side
sanitizers (device code as usual) into tests/native/abi_host_check.c, which
drives every entry point's argument validation and error text without a
GPU. A sanitizer report or a missing error fails the test. (GPU sanitizers
are not available on this pool; this covers the host half of the ABI.)
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(
    ROOT, "beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd")
BIN = os.path.join(PKG, "lib", "san", "abi_host_check")


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs hipcc")
def test_abi_host_code_under_asan_ubsan():
    jobs = str(min(8, os.cpu_count() or 4))
    r = subprocess.run(["make", "-C", os.path.join(PKG, "csrc"), "sanitize", f"-j{jobs}"],
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "abi host check ok" in out
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out
