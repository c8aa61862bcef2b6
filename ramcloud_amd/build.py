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
HEADERS = ["gf2.h", "walk_rules.h", "shard_plan.h"]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the MI355X build needs ROCm")


SHA_MARKER = b"src_sha="


def _deps():
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "ramcrc.h"))
    deps.append(os.path.abspath(__file__))
    return deps


def source_sha(defines=()):
    """sha256 (first 16 hex digits) of every source, header and compile flag
    the library is built from.  Compiled into the library (ramcrc_build_info
    reports it) and read back from the .so to decide staleness, so a shipped
    library can be tied to the tree it came from."""
    h = hashlib.sha256()
    for d in _deps():
        h.update(os.path.relpath(d, ROOT).encode() + b"\0")
        with open(d, "rb") as f:
            h.update(f.read())
    for d in defines:
        h.update(b"-D" + d.encode() + b"\0")
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
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-fconstexpr-steps=1000000000", "-Wall", "-Wno-unused-function",
           "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
    cmd += ["-D" + d for d in defines]
    cmd += [f'-DRAMCRC_SRC_SHA="{source_sha(defines)}"']
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


# Tuning variants (A/B on the GPU box: RAMCRC_LIB=<path> python bench.py ...)
VARIANTS = {
    "u4_c18": ["RAMCRC_UNROLL=4", "RAMCRC_CHUNK_SHIFT=18"],
    "u2_c18": ["RAMCRC_UNROLL=2", "RAMCRC_CHUNK_SHIFT=18"],
    "u6_c18": ["RAMCRC_UNROLL=6", "RAMCRC_CHUNK_SHIFT=18"],
    "u4_c19": ["RAMCRC_UNROLL=4", "RAMCRC_CHUNK_SHIFT=19"],
    "u4_c17": ["RAMCRC_UNROLL=4", "RAMCRC_CHUNK_SHIFT=17"],
    "u4_c20": ["RAMCRC_UNROLL=4", "RAMCRC_CHUNK_SHIFT=20"],
    # parallel-walk sync search (k_walk_sync)
    "walkdbg": ["RAMCRC_WALK_DEBUG=1"],
    "fw32": ["RAMCRC_FIX_WIN_KIB=32"],
    "nocap": ["RAMCRC_NO_CAPTURE=1"],
    "ew12": ["RAMCRC_ENT_WAVES=12"],
    "sh4": ["RAMCRC_SYNC_HOPS=4"],
    "sh5": ["RAMCRC_SYNC_HOPS=5"],
    "sh3": ["RAMCRC_SYNC_HOPS=3"],
    "sh4_ss6": ["RAMCRC_SYNC_HOPS=4", "RAMCRC_SYNC_STAGE_KIB=6"],
    "sh3_ss4": ["RAMCRC_SYNC_HOPS=3", "RAMCRC_SYNC_STAGE_KIB=4"],
    "sh7": ["RAMCRC_SYNC_HOPS=7"],
    "sh8": ["RAMCRC_SYNC_HOPS=8"],
    "sh10": ["RAMCRC_SYNC_HOPS=10"],
    "sp16": ["RAMCRC_SYNC_PER=16"],
    "sp4": ["RAMCRC_SYNC_PER=4"],
    "ss6": ["RAMCRC_SYNC_STAGE_KIB=6"],
    "ss16": ["RAMCRC_SYNC_STAGE_KIB=16"],
    "ss8": ["RAMCRC_SYNC_STAGE_KIB=8"],
    "ss12": ["RAMCRC_SYNC_STAGE_KIB=12"],
    "spf0": ["RAMCRC_SYNC_PF=0"],
    "searly": ["RAMCRC_SYNC_EARLY=1"],
    "sstrict0": ["RAMCRC_SYNC_STRICT=0"],
    "ps15": ["RAMCRC_PART_SHIFT=15"],
    "ps17": ["RAMCRC_PART_SHIFT=17"],
    "tv1": ["RAMCRC_TINY_V=1"],
    "notrim": ["RAMCRC_TINY_TRIM=0"],
    "tinyprobe": ["RAMCRC_TINY_PROBE=1", "RAMCRC_TINY_CF=0"],
    "nocf": ["RAMCRC_TINY_CF=0"],
    "bg1": ["RAMCRC_BIN_WGS_PER_CU=1"],
    "bg4": ["RAMCRC_BIN_WGS_PER_CU=4"],
    "evrec": ["RAMCRC_EXT_TIMING=0"],
    "bp2": ["RAMCRC_BIN_PER=2"],
    "bp8": ["RAMCRC_BIN_PER=8"],
    "nosafe": ["RAMCRC_TINY_SAFE=0"],
    "aa": ["RAMCRC_AA_SAME=1"],   # A/A: identical code, separate library
    # k_entries ping-pong depth / waves per CU
    "pu4": ["RAMCRC_PU=4"],
    "ew8": ["RAMCRC_ENT_WAVES=8"],
    # long-phase probes (WRONG results, A/B timing only)
    "pfold0": ["RAMCRC_PROBE_FOLD=1"],
    "pfoldcf": ["RAMCRC_PROBE_FOLD=2"],
    "pmask": ["RAMCRC_PROBE_MASK=1"],
    "pu3": ["RAMCRC_PU=3"],
    # k_entries phase stamps (tools/stamps.py)
    "stamps": ["RAMCRC_STAMPS=1"],
    "stamps_sk0": ["RAMCRC_STAMPS=1", "RAMCRC_AGE_SKEW=0"],
    "sk0": ["RAMCRC_AGE_SKEW=0"],
    "sk30": ["RAMCRC_AGE_SKEW=30"],
    "sk50": ["RAMCRC_AGE_SKEW=50"],
    "oc2": ["RAMCRC_OCTET_COST=2"],
    "sk80": ["RAMCRC_AGE_SKEW=80"],
    "ss7": ["RAMCRC_SYNC_STAGE_KIB=7"],
    "ss9": ["RAMCRC_SYNC_STAGE_KIB=9"],
    "ps15": ["RAMCRC_PART_SHIFT=15"],
    "ps17": ["RAMCRC_PART_SHIFT=17"],
    "fw8": ["RAMCRC_FIX_WIN_KIB=8"],
    "sh5_ss7": ["RAMCRC_SYNC_HOPS=5", "RAMCRC_SYNC_STAGE_KIB=7"],
    "oc6": ["RAMCRC_OCTET_COST=6"],
    "sk120": ["RAMCRC_AGE_SKEW=120"],
    "nobatch": ["RAMCRC_STEP_BATCH=0"],


}


def build_variants(names=None, verbose=False):
    from concurrent.futures import ThreadPoolExecutor
    names = names or list(VARIANTS)
    outs = {n: os.path.join(LIBDIR, "variants", f"libramcrc_{n}.so") for n in names}
    with ThreadPoolExecutor(max_workers=4) as ex:
        list(ex.map(lambda n: _compile(outs[n], VARIANTS[n], verbose), names))
    return outs


if __name__ == "__main__":
    if "--variants" in sys.argv:
        print(build_variants(verbose=True))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
