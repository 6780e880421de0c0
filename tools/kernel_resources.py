"""Per-kernel register and scratch use of the built gfx950 code objects.

    python tools/kernel_resources.py [lib/obj/spmm.o ...] [--spills]

Reads the AMDGPU metadata notes of each object's device code (the
.hip_fatbin bundle unpacked with clang-offload-bundler, the notes printed by
llvm-readobj): .vgpr_count, .sgpr_count, .private_segment_fixed_size (bytes
of scratch per lane: register spills). A spilling SpMM kernel writes and
re-reads its spill slots through L2 on every batch; at C4 the two-row kernels'
spills (12-24 B per lane at the 8-wave target) issued 5-12.5M extra 64-B
write requests per launch (profiles/round5/r5c_*), so tests/test_kernel_resources.py
keeps the product kernels spill-free.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(
    ROOT, "beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd")
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def kernels(obj: str) -> dict:
    """{kernel symbol: {"vgpr": n, "sgpr": n, "scratch": bytes per lane}} of
    one host object's gfx950 device code."""
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fb.bin"), os.path.join(td, "dev.co")
        r = subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", obj],
                           capture_output=True)
        if r.returncode != 0 or not os.path.exists(fb):
            return {}   # a host-only object (no device code)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        f"--input={fb}", f"--targets={TARGET}", f"--output={co}"],
                       check=True, capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    out, cur = {}, None
    keys = {".private_segment_fixed_size:": "scratch", ".vgpr_count:": "vgpr",
            ".sgpr_count:": "sgpr"}
    for line in notes.splitlines():
        t = line.strip().split()
        if not t:
            continue
        if t[0] == ".name:" and len(t) > 1:
            cur = out.setdefault(t[1], {})
        elif t[0] in keys and cur is not None and len(t) > 1:
            cur[keys[t[0]]] = int(t[1])
    return {k: v for k, v in out.items() if "scratch" in v}


def product_objects() -> list:
    return sorted(glob.glob(os.path.join(PKG, "lib", "obj", "*.o")))


def main(argv):
    spills_only = "--spills" in argv
    objs = [a for a in argv if not a.startswith("--")] or product_objects()
    for o in objs:
        for name, r in sorted(kernels(o).items()):
            if spills_only and not r["scratch"]:
                continue
            print(f"{os.path.basename(o):8s} vgpr {r.get('vgpr', 0):3d} sgpr {r.get('sgpr', 0):3d} "
                  f"scratch {r['scratch']:3d}  {name}")


if __name__ == "__main__":
    main(sys.argv[1:])
