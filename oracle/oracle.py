"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes bindings for the CPU restatement (oracle/liboracle.so) and, when it has
been built, the reference's own compiled hardware path
(oracle/_ref/libref_crc32c.so).  Imported only by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg -- never by the ramcloud_amd product path.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libref_crc32c.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)

IMPL_SSE42, IMPL_SLICING8, IMPL_BITWISE = 0, 1, 2

_lib = None
_ref = None


def build(with_ref=None):
    """Compile the oracle (and the reference harness when /root/reference exists)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    if with_ref is None:
        with_ref = os.path.isdir("/root/reference/src")
    if with_ref:
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build(with_ref=False)
        L = ctypes.CDLL(LIB_PATH)
        for name in ("oracle_bitwise", "oracle_slicing8", "oracle_sse42"):
            f = getattr(L, name)
            f.restype = ctypes.c_uint32
            f.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_mulmod.restype = ctypes.c_uint32
        L.oracle_mulmod.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_xpow8.restype = ctypes.c_uint32
        L.oracle_xpow8.argtypes = [ctypes.c_uint64]
        L.oracle_shift.restype = ctypes.c_uint32
        L.oracle_shift.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
        L.oracle_splitmix_fill.restype = None
        L.oracle_splitmix_fill.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_entries.restype = None
        L.oracle_entries.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_int, ctypes.c_int]
        L.oracle_segments_mt.restype = ctypes.c_int
        L.oracle_build_object_segment.restype = ctypes.c_uint32
        L.oracle_build_object_segment.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                                  ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_check_metadata.restype = ctypes.c_uint32
        L.oracle_check_metadata.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_verify_objects.restype = ctypes.c_uint64
        L.oracle_verify_objects.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                            ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p]
        L.oracle_segments_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_replay_mt.restype = ctypes.c_int64
        L.oracle_replay_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.oracle_have_sse42.restype = ctypes.c_int
        L.oracle_init()
        _lib = L
    return _lib


def ref_available():
    return os.path.exists(REF_PATH)


def ref():
    """The reference's own intelCrc32C (src/Crc32C.h:39-93), or None if not built."""
    global _ref
    if _ref is None and ref_available():
        R = ctypes.CDLL(REF_PATH)
        R.ref_intel_crc32c.restype = ctypes.c_uint32
        R.ref_intel_crc32c.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
        R.ref_segments_mt.restype = ctypes.c_int
        R.ref_segments_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        R.ref_entries_mt.restype = ctypes.c_int
        R.ref_entries_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int]
        _ref = R
    return _ref


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _as_u8(data):
    if isinstance(data, (bytes, bytearray)):
        return np.frombuffer(bytes(data), dtype=np.uint8)
    return np.ascontiguousarray(data).view(np.uint8).reshape(-1)


def crc_raw(state, data, impl=IMPL_SSE42):
    """Crc32C with result=state, update(data): the raw (pre-inversion) state."""
    buf = _as_u8(data)
    f = (lib().oracle_sse42, lib().oracle_slicing8, lib().oracle_bitwise)[impl]
    return int(f(state & 0xFFFFFFFF, _ptr(buf), buf.size))


def crc32c(data, impl=IMPL_SSE42):
    """Crc32C().update(data).getResult()."""
    return (~crc_raw(0xFFFFFFFF, data, impl)) & 0xFFFFFFFF


def ref_crc_raw(state, data):
    R = ref()
    buf = _as_u8(data)
    return int(R.ref_intel_crc32c(state & 0xFFFFFFFF, _ptr(buf), buf.size))


def mulmod(a, b):
    return int(lib().oracle_mulmod(a & 0xFFFFFFFF, b & 0xFFFFFFFF))


def xpow8(n):
    return int(lib().oracle_xpow8(n))


def shift(state, nbytes):
    return int(lib().oracle_shift(state & 0xFFFFFFFF, nbytes))


def splitmix_bytes(seed, nbytes):
    out = np.empty(nbytes, dtype=np.uint8)
    lib().oracle_splitmix_fill(seed & 0xFFFFFFFFFFFFFFFF, _ptr(out), nbytes)
    return out


def entries(base, off, length, init=None, finalize=True, impl=IMPL_SSE42):
    base = _as_u8(base)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint64)
    n = off.size
    if n and int((off + length).max()) > base.size:
        raise ValueError("entry past end of base buffer")
    out = np.empty(n, dtype=np.uint32)
    init_a = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
    lib().oracle_entries(_ptr(base), _ptr(off), _ptr(length), _ptr(init_a), _ptr(out),
                         n, 1 if finalize else 0, impl)
    return out


def ref_entries(base, off, length, init=None, finalize=True, threads=1, pin=True):
    """The reference's own intelCrc32C (oracle/_ref) once per entry, blocks of
    4096 entries dealt round-robin over `threads` pinned threads."""
    base = _as_u8(base)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint64)
    n = off.size
    if n and int((off + length).max()) > base.size:
        raise ValueError("entry past end of base buffer")
    out = np.empty(n, dtype=np.uint32)
    init_a = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
    rc = ref().ref_entries_mt(_ptr(base), _ptr(off), _ptr(length), _ptr(init_a), _ptr(out), n,
                              threads, 1 if pin else 0, 1 if finalize else 0)
    if rc != 0:
        raise RuntimeError("thread start failed")
    return out


def segments(base, seg_bytes, nseg, threads=1, impl=IMPL_SSE42, pin=True, use_ref=False):
    """getResult() of each whole segment; threads take segments round-robin."""
    base = _as_u8(base)
    if base.size < seg_bytes * nseg:
        raise ValueError("base buffer too small")
    out = np.empty(nseg, dtype=np.uint32)
    if use_ref:
        rc = ref().ref_segments_mt(_ptr(base), seg_bytes, nseg, _ptr(out), threads, 1 if pin else 0)
    else:
        rc = lib().oracle_segments_mt(_ptr(base), seg_bytes, nseg, _ptr(out), threads, impl,
                                      1 if pin else 0)
    if rc != 0:
        raise RuntimeError("thread start failed")
    return out


# ---------------------------------------------------------------- segments
def build_object_segment(seg, value_len, first_key=0):
    """Restated RecoverSegmentBenchmark fill of `seg` (numpy uint8, value bytes
    pre-filled); returns (n_objects, segment_length, checksum)."""
    cl = np.zeros(1, np.uint32)
    cc = np.zeros(1, np.uint32)
    n = lib().oracle_build_object_segment(_ptr(seg), seg.size, value_len, first_key,
                                          _ptr(cl), _ptr(cc))
    return int(n), int(cl[0]), int(cc[0])


def check_metadata(seg, cert_len, cert_crc, segment=0, capacity=None, table_cap=None):
    """Restated Segment::checkMetadataIntegrity.  Returns (flags, checksum,
    n_entries, table uint32[n, 4])."""
    seg = np.ascontiguousarray(seg, dtype=np.uint8)
    capacity = seg.size if capacity is None else capacity
    cap = (capacity // 2 + 1) if table_cap is None else table_cap
    table = np.zeros((max(cap, 1), 4), np.uint32)
    ck = np.zeros(1, np.uint32)
    n = np.zeros(1, np.uint32)
    flags = lib().oracle_check_metadata(_ptr(seg), capacity, cert_len & 0xFFFFFFFF,
                                        cert_crc & 0xFFFFFFFF, segment, _ptr(ck), _ptr(n),
                                        _ptr(table), cap)
    k = min(int(n[0]), cap)
    return int(flags), int(ck[0]), int(n[0]), table[:k].copy()


def verify_objects(base, stride, table, nseg=None, seg_ok=None):
    """Restated Object::computeChecksum comparison over walk records of the
    segments whose metadata check passed (seg_ok: bool[nseg], None = all).
    Returns (bad_total, crc uint32[n], bad_per_segment uint32[nseg])."""
    base = np.ascontiguousarray(base, dtype=np.uint8)
    table = np.ascontiguousarray(table, dtype=np.uint32).reshape(-1, 4)
    n = table.shape[0]
    crc = np.zeros(max(n, 1), np.uint32)
    nseg = (int(table[:, 0].max()) + 1 if n else 1) if nseg is None else nseg
    bad = np.zeros(max(nseg, 1), np.uint32)
    ok = None if seg_ok is None else np.ascontiguousarray(seg_ok, dtype=np.uint8)
    total = lib().oracle_verify_objects(_ptr(base), stride, _ptr(table), n,
                                        None if ok is None else _ptr(ok), _ptr(crc), _ptr(bad))
    return int(total), crc[:n], bad[:nseg]


def replay_mt(base, seg_bytes, nseg, certs, threads=1, pin=True, use_ref=False):
    """Walk + replay checks of nseg object segments (whole segments round-robin
    over threads); with use_ref every CRC byte goes through the reference's
    own intelCrc32C (oracle/_ref).  Returns the number of failed segments."""
    base = _as_u8(base)
    certs = np.ascontiguousarray(certs, dtype=np.uint32).reshape(-1, 2)
    if base.size < seg_bytes * nseg or certs.shape[0] < nseg:
        raise ValueError("buffers too small")
    ext = ctypes.cast(ref().ref_intel_crc32c, ctypes.c_void_p) if use_ref else None
    r = lib().oracle_replay_mt(_ptr(base), seg_bytes, nseg, _ptr(certs), threads,
                               1 if pin else 0, ext)
    if r < 0:
        raise RuntimeError("thread start failed")
    return int(r)
