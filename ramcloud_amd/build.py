"""Build libramcrc.so in-tree (hipcc, gfx950 only).

    python -m ramcloud_amd.build          # or __graft_entry__.build()

The library is plain C ABI (include/ramcrc.h); torch is not linked.  The .so
lands in ramcloud_amd/lib/ (git-ignored, shipped to the GPU box with the
snapshot).
"""
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libramcrc.so")
ARCH = "gfx950"

SOURCES = ["ramcrc_device.hip", "ramcrc_host.cc"]
HEADERS = ["gf2.h"]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the MI355X build needs ROCm")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "ramcrc.h"))
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    if not force and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-fconstexpr-steps=1000000000", "-Wall", "-Wno-unused-function",
           "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
    cmd += [os.path.join(CSRC, s) for s in SOURCES]
    cmd += ["-o", tmp]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
