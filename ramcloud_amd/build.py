"""Build libramcrc.so in-tree (hipcc, gfx950 only).

    python -m ramcloud_amd.build          # or __graft_entry__.build()

The library is plain C ABI (include/ramcrc.h); torch is not linked.  The .so
lands in ramcloud_amd/lib/ (git-ignored, shipped to the GPU box with the
snapshot).
"""
import hashlib
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

SOURCES = ["ramcrc_device.hip", "ramcrc_host.cc", "ramcrc_shard.hip", "ramcrc_fill.hip"]
HEADERS = ["gf2.h", "walk_rules.h", "shard_plan.h",
           # parts of ramcrc_device.hip (one translation unit)
           "dev_common.inc", "dev_chunks.inc", "dev_bins.inc", "dev_entries.inc",
           "dev_plan.inc", "dev_host.inc", "dev_walk.inc", "dev_checks.inc"]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the MI355X build needs ROCm")


SHA_MARKER = b"src_sha="

# Knobs whose non-default values gave wrong results or skipped work in earlier
# rounds' A/B probes.  The knobs are gone from the sources; a variant naming
# one is refused here, and ramcrc.lib() refuses a library whose build_info
# reports one (RAMCRC_LIB), so no bench line or test can run such a build.
UNSAFE_DEFINES = ("RAMCRC_PROBE_", "RAMCRC_WALK_DEBUG", "RAMCRC_BIN_RESCUE", "RAMCRC_NO_CAPTURE")


def unsafe_defines(defines):
    """The entries of `defines` (or a build_info "defines=" list) that name an
    unsafe knob."""
    return [d for d in defines if d.startswith(UNSAFE_DEFINES)]


def _deps():
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "ramcrc.h"))
    return deps


def _flags(defines=()):
    """The compile flags of a build (everything but the file paths)."""
    return ([f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
             "-fconstexpr-steps=1000000000", "-Wall", "-Wno-unused-function", "-ldl"]
            + ["-D" + d for d in defines])


def source_sha(defines=()):
    """sha256 (first 16 hex digits) of every source, header and compile flag
    the library is built from (not of this script: edits that leave the
    flags alone do not change the hash).  Compiled into the library (ramcrc_build_info
    reports it) and read back from the .so to decide staleness, so a shipped
    library can be tied to the tree it came from."""
    h = hashlib.sha256()
    for d in _deps():
        h.update(os.path.relpath(d, ROOT).encode() + b"\0")
        with open(d, "rb") as f:
            h.update(f.read())
    for f in _flags(defines):
        h.update(f.encode() + b"\0")
    return h.hexdigest()[:16]


def built_sha(path=LIB):
    """The source hash embedded in a built library, or None."""
    try:
        with open(path, "rb") as f:
            blob = f.read()
    except OSError:
        return None
    i = blob.find(b"ramcrc gfx950 " + SHA_MARKER)
    if i < 0:
        return None
    i += len(b"ramcrc gfx950 " + SHA_MARKER)
    return blob[i:i + 16].decode("ascii", "replace")


def _stale():
    return built_sha(LIB) != source_sha()


def _compile(out, defines=(), verbose=False):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + ".tmp"
    flags = _flags(defines)
    cmd = [hipcc()] + [f for f in flags if f != "-ldl"]
    cmd += ["-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
    if unsafe_defines(defines):
        raise ValueError(f"refusing a build with unsafe knobs: {unsafe_defines(defines)}")
    cmd += [f'-DRAMCRC_SRC_SHA="{source_sha(defines)}"']
    if defines:
        cmd += [f'-DRAMCRC_DEFINES="{",".join(defines)}"']
    cmd += [os.path.join(CSRC, s) for s in SOURCES]
    cmd += ["-ldl", "-o", tmp]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(tmp, out)
    return out


def build(force=False, verbose=False):
    if not force and not _stale():
        return LIB
    return _compile(LIB, verbose=verbose)


def build_variants(names=None, verbose=False):
    from concurrent.futures import ThreadPoolExecutor
    from .variants import VARIANTS
    names = names or list(VARIANTS)
    outs = {n: os.path.join(LIBDIR, "variants", f"libramcrc_{n}.so") for n in names}
    with ThreadPoolExecutor(max_workers=4) as ex:
        list(ex.map(lambda n: _compile(outs[n], VARIANTS[n], verbose), names))
    return outs


if __name__ == "__main__":
    if "--variants" in sys.argv:
        names = sys.argv[sys.argv.index("--variants") + 1:]
        print(build_variants(names or None, verbose=True))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
