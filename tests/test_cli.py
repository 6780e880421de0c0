"""CPU: the driver-facing scripts parse their arguments and every tool
compiles (no GPU needed: nothing here launches a kernel)."""
import os
import py_compile
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_help_lists_the_contract_flags():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    for flag in ("--gpus", "--steps", "--warmup", "--config", "--vertex-order",
                 "--exchange-parts", "--frontier-parts", "--scaling", "--dense-check"):
        assert flag in r.stdout + r.stderr, flag


@pytest.mark.parametrize("name", sorted(f for f in os.listdir(os.path.join(ROOT, "tools"))
                                        if f.endswith(".py")))
def test_tools_compile(name):
    py_compile.compile(os.path.join(ROOT, "tools", name), doraise=True)
