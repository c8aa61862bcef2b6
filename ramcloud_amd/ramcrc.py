"""Python binding of libramcrc (include/ramcrc.h) -- the product path.

The CRC work happens in the HIP kernels of libramcrc.so; this module only
passes pointers.  There is no CPU fallback for the device entry points: if the
library is missing or a call fails, an exception is raised.

Device memory and streams come from PyTorch (plumbing only): tensors are
passed by data_ptr(), streams by torch.cuda.current_stream().cuda_stream.
"""
import ctypes
import os

import numpy as np

from . import build as _build

_c = ctypes
_lib = None

FINALIZE = 1

_ERRORS = {0: "ok", -1: "invalid argument", -2: "out of memory", -3: "HIP error",
           -4: "no usable device", -5: "RCCL error", -6: "launch refused (scratch too small)",
           -7: "launch refused (inconsistent bin layout)",
           -8: "another shard rank failed"}

ENOMEM = -2
EINTERNAL = -7
EPEER = -8

# ramcrc_ctx_set_option options (include/ramcrc.h)
OPT_SERIAL_WALK = 1
OPT_WALK_PART_SHIFT = 2
OPT_TEST_FAIL_AFTER_COUNT = 3
OPT_TEST_DIRTY_BINS = 4
OPT_TEST_BIN_STRAGGLER = 5
OPT_BIN_ONE = 6
OPT_VERIFY_IN_WALK = 7


class RamcrcError(RuntimeError):
    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


def lib_path():
    # RAMCRC_LIB selects a tuning variant built by `python -m ramcloud_amd.build --variants`
    return os.environ.get("RAMCRC_LIB") or _build.LIB


def lib():
    """Load libramcrc.so; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        raise RamcrcError(f"libramcrc.so not built ({path}); run python -m ramcloud_amd.build")
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7,
    # with the same soname as /opt/rocm's, and whichever is loaded first
    # serves both.  Loading this library first left torch on /opt/rocm's
    # runtime, which then reported no GPU; importing torch first keeps every
    # caller on torch's runtime.
    import torch  # noqa: F401
    L = _c.CDLL(path)
    if path != _build.LIB:
        _check_variant(L, path)
    vp, u32, u64, i32 = _c.c_void_p, _c.c_uint32, _c.c_uint64, _c.c_int
    sig = {
        "ramcrc_update_hw": (u32, [u32, vp, u64]),
        "ramcrc_update_sw": (u32, [u32, vp, u64]),
        "ramcrc_update": (u32, [u32, vp, u64]),
        "ramcrc_cpu_has_hw": (i32, []),
        "ramcrc_shift": (u32, [u32, u64]),
        "ramcrc_combine": (u32, [u32, u32, u64]),
        "ramcrc_ctx_create": (i32, [i32, _c.POINTER(vp)]),
        "ramcrc_ctx_destroy": (i32, [vp]),
        "ramcrc_ctx_reserve": (i32, [vp, u64, u64]),
        "ramcrc_segments_device": (i32, [vp, vp, u64, u64, vp, vp, u32, vp]),
        "ramcrc_batch_device": (i32, [vp, vp, vp, vp, vp, vp, u64, u32, vp]),
        "ramcrc_entries_device": (i32, [vp, vp, vp, vp, vp, vp, u64, u32, vp]),
        "ramcrc_batch_host": (i32, [vp, vp, vp, vp, vp, u64, u32]),
        "ramcrc_stream_host": (i32, [vp, vp, u64, u64, vp, u32, i32, i32]),
        "ramcrc_segment_walk_device": (i32, [vp, vp, u64, u32, u64, vp, vp, vp, u64, vp, vp]),
        "ramcrc_verify_objects_device": (i32, [vp, vp, u64, vp, u64, vp, vp, vp, vp]),
        "ramcrc_replay_verify_device": (i32, [vp, vp, u64, u32, u64, vp, vp, vp, u64, vp, vp, vp]),
        "ramcrc_segments_certify_device": (i32, [vp, vp, u64, u32, u64, vp, vp, vp, vp]),
        "ramcrc_segment_fill_objects": (i32, [vp, u32, u32, u64, _c.POINTER(u32), vp]),
        "ramcrc_assemble_objects_device": (i32, [vp, vp, vp, vp, vp, u64, vp]),
        "ramcrc_assemble_objects_host": (i32, [vp, vp, vp, u64]),
        "ramcrc_ctx_set_timing": (i32, [vp, i32]),
        "ramcrc_ctx_scan_time": (i32, [vp, _c.POINTER(_c.c_double), _c.POINTER(u64)]),
        "ramcrc_ctx_status": (i32, [vp, _c.POINTER(u32)]),
        "ramcrc_ctx_check": (i32, [vp, vp]),
        "ramcrc_ctx_set_option": (i32, [vp, i32, _c.c_int64]),
        "ramcrc_segment_fill_objects_device": (i32, [vp, vp, u64, u32, u64, u32, u64, vp, vp,
                                                     _c.POINTER(u32)]),
        "ramcrc_shard_unique_id": (i32, [vp]),
        "ramcrc_shard_create_all": (i32, [vp, i32, _c.POINTER(vp)]),
        "ramcrc_shard_create_rank": (i32, [vp, i32, i32, i32, _c.POINTER(vp)]),
        "ramcrc_shard_destroy": (i32, [vp]),
        "ramcrc_shard_range": (i32, [u64, i32, i32, _c.POINTER(u64), _c.POINTER(u64)]),
        "ramcrc_shard_local_count": (i32, [vp]),
        "ramcrc_shard_info": (i32, [vp, i32, _c.POINTER(i32), _c.POINTER(i32), _c.POINTER(vp),
                                    _c.POINTER(vp)]),
        "ramcrc_shard_segments": (i32, [vp, vp, u64, u64, vp, u32]),
        "ramcrc_shard_sync": (i32, [vp]),
        "ramcrc_shard_results": (i32, [vp, i32, vp, u64]),
        "ramcrc_stream_create_cu_mask": (i32, [i32, vp, u32, _c.POINTER(vp)]),
        "ramcrc_stream_destroy": (i32, [vp]),
        "ramcrc_ctx_set_cus": (i32, [vp, i32]),
        "ramcrc_strerror": (_c.c_char_p, [i32]),
        "ramcrc_last_hip_error": (i32, []),
        "ramcrc_device_count": (i32, []),
        "ramcrc_build_info": (_c.c_char_p, []),
        "ramcrc_ctx_debug_bins": (i32, [vp, vp, u64, _c.POINTER(u32)]),
    }
    for name, (res, args) in sig.items():
        try:
            f = getattr(L, name)
        except AttributeError:
            if path == _build.LIB:
                raise   # the product library must export the whole header
            continue    # an older A/B variant (RAMCRC_LIB)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def build_defines(info):
    """The -D knobs a library was built with, from its ramcrc_build_info()."""
    if " defines=" not in info:
        return []
    d = info.split(" defines=", 1)[1].split()
    return d[0].split(",") if d and d[0] != "none" else []


def _check_variant(L, path):
    """RAMCRC_LIB: only A/B variants of this tree's table that compute exact
    results (build.UNSAFE_DEFINES) may replace the product library."""
    f = L.ramcrc_build_info
    f.restype = _c.c_char_p
    info = f().decode("ascii", "replace")
    if "src_sha=" not in info:
        raise RamcrcError(f"RAMCRC_LIB={path} is not a libramcrc build")
    bad = _build.unsafe_defines(build_defines(info))
    if bad:
        raise RamcrcError(f"RAMCRC_LIB={path} is a probe build ({bad}); refusing to load it")


def exported_symbols():
    return [n for n in dir(lib()) if n.startswith("ramcrc_")]


def _check(rc, what):
    if rc != 0:
        msg = lib().ramcrc_strerror(rc).decode()
        raise RamcrcError(f"{what} failed: {_ERRORS.get(rc, rc)} ({msg})", rc)


def _buf(data):
    if isinstance(data, (bytes, bytearray, memoryview)):
        a = np.frombuffer(bytes(data), dtype=np.uint8)
    else:
        a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return a, _c.c_void_p(a.ctypes.data)


# ------------------------------------------------------------------ host
def update(state, data):
    """Crc32C::update on the host hardware path; returns the raw state."""
    a, p = _buf(data)
    return int(lib().ramcrc_update(state & 0xFFFFFFFF, p, a.size))


def update_sw(state, data):
    a, p = _buf(data)
    return int(lib().ramcrc_update_sw(state & 0xFFFFFFFF, p, a.size))


def update_hw(state, data):
    a, p = _buf(data)
    return int(lib().ramcrc_update_hw(state & 0xFFFFFFFF, p, a.size))


def crc32c(data):
    """Crc32C().update(data).getResult() on the host."""
    return (~update(0xFFFFFFFF, data)) & 0xFFFFFFFF


def shift(state, nbytes):
    return int(lib().ramcrc_shift(state & 0xFFFFFFFF, nbytes))


def combine(raw_a, raw_b, len_b):
    return int(lib().ramcrc_combine(raw_a & 0xFFFFFFFF, raw_b & 0xFFFFFFFF, len_b))


def cpu_has_hw():
    return bool(lib().ramcrc_cpu_has_hw())


def device_count():
    return int(lib().ramcrc_device_count())


def segment_fill_objects(seg, value_len, first_key=0):
    """Host append path: fill an empty segment (numpy uint8, pre-filled value
    bytes) with RecoverSegmentBenchmark-shaped objects.  Returns
    (n_objects, segment_length, checksum)."""
    if not (isinstance(seg, np.ndarray) and seg.dtype == np.uint8 and seg.flags.c_contiguous):
        raise RamcrcError("segment must be a contiguous numpy uint8 array")
    n = _c.c_uint32(0)
    cert = np.zeros(2, dtype=np.uint32)
    rc = lib().ramcrc_segment_fill_objects(_c.c_void_p(seg.ctypes.data), seg.size, value_len,
                                           first_key, _c.byref(n), _c.c_void_p(cert.ctypes.data))
    _check(rc, "ramcrc_segment_fill_objects")
    return n.value, int(cert[0]), int(cert[1])


# ---------------------------------------------------------------- device
def _ptr(t):
    if t is None:
        return None
    if isinstance(t, int):
        return _c.c_void_p(t)
    return _c.c_void_p(t.data_ptr())


def _stream(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    if isinstance(stream, CuMaskStream):
        return _c.c_void_p(stream.handle)
    if isinstance(stream, int):
        return _c.c_void_p(stream)
    return _c.c_void_p(stream.cuda_stream)


class CuMaskStream:
    """A HIP stream whose kernels run only on the given CUs
    (ramcrc_stream_create_cu_mask).  Pass it as stream= (it converts to the
    raw stream handle); destroy() after the work on it has finished."""

    def __init__(self, device, cus):
        import numpy as np
        mask = np.zeros(8, np.uint32)
        for cu in cus:
            mask[cu // 32] |= np.uint32(1 << (cu % 32))
        words = int(max(cu for cu in cus) // 32 + 1)
        h = _c.c_void_p()
        _check(lib().ramcrc_stream_create_cu_mask(int(device), _c.c_void_p(mask.ctypes.data), words,
                                                  _c.byref(h)), "ramcrc_stream_create_cu_mask")
        self.handle = h.value
        self.ncu = len(set(cus))

    def __int__(self):
        return self.handle

    def destroy(self):
        if self.handle:
            lib().ramcrc_stream_destroy(_c.c_void_p(self.handle))
            self.handle = None


class Context:
    """A libramcrc context on one GPU (scratch + staging).  One per stream/thread."""

    def __init__(self, device=0):
        h = _c.c_void_p()
        _check(lib().ramcrc_ctx_create(int(device), _c.byref(h)), "ramcrc_ctx_create")
        self._h = h
        self.device = int(device)

    def close(self):
        if self._h:
            lib().ramcrc_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_timing(self, enable=True):
        _check(lib().ramcrc_ctx_set_timing(self._h, 1 if enable else 0), "ramcrc_ctx_set_timing")

    def scan_time(self):
        """(summed scan-kernel milliseconds, launches) since the last call."""
        ms = _c.c_double(0)
        n = _c.c_uint64(0)
        _check(lib().ramcrc_ctx_scan_time(self._h, _c.byref(ms), _c.byref(n)), "ramcrc_ctx_scan_time")
        return ms.value, n.value

    def status(self):
        s = _c.c_uint32(0)
        _check(lib().ramcrc_ctx_status(self._h, _c.byref(s)), "ramcrc_ctx_status")
        return s.value

    def check(self, stream=None):
        """Wait for `stream`; raise if any launch of this context was refused
        since the last check (ramcrc_ctx_check)."""
        _check(lib().ramcrc_ctx_check(self._h, _stream(stream)), "ramcrc_ctx_check")

    def set_serial_walk(self, enable=True):
        """Walk segments with one wavefront each (the serial chase) instead of
        the parallel walk (RAMCRC_OPT_SERIAL_WALK)."""
        _check(lib().ramcrc_ctx_set_option(self._h, 1, 1 if enable else 0), "ramcrc_ctx_set_option")

    def set_walk_part_shift(self, shift):
        """log2 of the parallel walk's part size, 13..20, forced for every
        batch; 0 = the default, chosen per batch from the entry density
        (RAMCRC_OPT_WALK_PART_SHIFT)."""
        _check(lib().ramcrc_ctx_set_option(self._h, 2, int(shift)), "ramcrc_ctx_set_option")

    def debug_bins(self):
        """Diagnostics: (count[161], cursor[2][161], hist[2][161], next parity)."""
        buf = np.zeros(5 * 161, np.uint64)
        par = _c.c_uint32(0)
        _check(lib().ramcrc_ctx_debug_bins(self._h, _c.c_void_p(buf.ctypes.data), buf.size,
                                           _c.byref(par)), "ramcrc_ctx_debug_bins")
        return buf[:161], buf[161:483].reshape(2, 161), buf[483:].reshape(2, 161), par.value

    def bin_rescues(self):
        """One-launch binnings of this context that aborted (part of the grid
        not dispatched in time) and completed through the two-launch path."""
        buf = np.zeros(5 * 161 + 1, np.uint64)
        par = _c.c_uint32(0)
        _check(lib().ramcrc_ctx_debug_bins(self._h, _c.c_void_p(buf.ctypes.data), buf.size,
                                           _c.byref(par)), "ramcrc_ctx_debug_bins")
        return int(buf[-1])

    def set_option(self, option, value):
        """ramcrc_ctx_set_option (OPT_* above)."""
        _check(lib().ramcrc_ctx_set_option(self._h, int(option), int(value)), "ramcrc_ctx_set_option")

    def set_cus(self, ncu):
        """Size this context's persistent grids for ncu CUs (0 = all): for
        launches on a CU-masked stream (see cu_mask_stream)."""
        _check(lib().ramcrc_ctx_set_cus(self._h, int(ncu)), "ramcrc_ctx_set_cus")

    def reserve(self, max_chunks, max_entries):
        _check(lib().ramcrc_ctx_reserve(self._h, max_chunks, max_entries), "ramcrc_ctx_reserve")

    # All tensors below are CUDA tensors; outputs are int32 tensors holding the
    # uint32 CRC bit patterns.
    def segments(self, data, seg_bytes, nseg, out, init=None, finalize=True, stream=None):
        rc = lib().ramcrc_segments_device(self._h, _ptr(data), seg_bytes, nseg, _ptr(init),
                                          _ptr(out), FINALIZE if finalize else 0, _stream(stream))
        _check(rc, "ramcrc_segments_device")
        return out

    def batch(self, data, off, length, out, init=None, finalize=True, stream=None):
        n = off.numel()
        fl = FINALIZE if finalize else 0
        rc = lib().ramcrc_batch_device(self._h, _ptr(data), _ptr(off), _ptr(length), _ptr(init),
                                       _ptr(out), n, fl, _stream(stream))
        _check(rc, "ramcrc_batch_device")
        return out

    def entries(self, data, off, length, out, init=None, finalize=True, stream=None):
        n = off.numel()
        fl = FINALIZE if finalize else 0
        rc = lib().ramcrc_entries_device(self._h, _ptr(data), _ptr(off), _ptr(length), _ptr(init),
                                         _ptr(out), n, fl, _stream(stream))
        _check(rc, "ramcrc_entries_device")
        return out

    def segment_walk(self, data, seg_stride, seg_capacity, nseg, certs, status, entries,
                     n_entries, stream=None):
        """Segment::checkMetadataIntegrity on the device.  certs: int32 [nseg, 2]
        (segment_length, checksum); status: int32 [nseg, 4]; entries: int32
        [cap, 4]; n_entries: int64 [1]."""
        cap = 0 if entries is None else entries.shape[0]
        rc = lib().ramcrc_segment_walk_device(self._h, _ptr(data), seg_stride, seg_capacity, nseg,
                                              _ptr(certs), _ptr(status), _ptr(entries), cap,
                                              _ptr(n_entries), _stream(stream))
        _check(rc, "ramcrc_segment_walk_device")
        return status

    def certify(self, data, seg_stride, seg_capacity, nseg, heads, certs, flags=None, stream=None):
        """Segment::getAppendedLength's certificate for nseg rebuilt segments
        (ramcrc_segments_certify_device).  heads: int32 CUDA [nseg]; certs:
        int32 CUDA [nseg, 2] out; flags: int32 CUDA [nseg] out or None."""
        rc = lib().ramcrc_segments_certify_device(self._h, _ptr(data), seg_stride, seg_capacity, nseg,
                                                  _ptr(heads), _ptr(certs), _ptr(flags),
                                                  _stream(stream))
        _check(rc, "ramcrc_segments_certify_device")
        return certs

    def verify_objects(self, data, seg_stride, entries, n_entries, obj_crc, status, stream=None):
        """Object::computeChecksum + comparison for every object record of a walk."""
        rc = lib().ramcrc_verify_objects_device(self._h, _ptr(data), seg_stride, _ptr(entries),
                                                entries.shape[0], _ptr(n_entries), _ptr(obj_crc),
                                                _ptr(status), _stream(stream))
        _check(rc, "ramcrc_verify_objects_device")
        return status

    def replay_verify(self, data, seg_stride, seg_capacity, nseg, certs, status, entries, n_entries,
                      obj_crc, stream=None):
        """segment_walk + verify_objects in one call (ramcrc_replay_verify_device):
        same results; skips the binning pass when every record is a one-window
        object."""
        cap = 0 if entries is None else entries.shape[0]
        rc = lib().ramcrc_replay_verify_device(self._h, _ptr(data), seg_stride, seg_capacity, nseg,
                                               _ptr(certs), _ptr(status), _ptr(entries), cap,
                                               _ptr(n_entries), _ptr(obj_crc), _stream(stream))
        _check(rc, "ramcrc_replay_verify_device")
        return status

    def fill_objects(self, data, seg_stride, capacity, nseg, value_len, first_key=0, certs=None):
        """RecoverSegmentBenchmark-shaped object segments built in place on the
        device (ramcrc_segment_fill_objects_device): returns (objects per
        segment, segment_length, checksum); certs (int32 CUDA [nseg, 2]) gets
        every segment's certificate when given.  Synchronous."""
        cert = np.zeros(2, dtype=np.uint32)
        per = _c.c_uint32(0)
        rc = lib().ramcrc_segment_fill_objects_device(
            self._h, _ptr(data), seg_stride, capacity, nseg, value_len, first_key, _ptr(certs),
            _c.c_void_p(cert.ctypes.data), _c.byref(per))
        _check(rc, "ramcrc_segment_fill_objects_device")
        return per.value, int(cert[0]), int(cert[1])

    def assemble_objects(self, data, off, length, out=None, stream=None):
        """Object::assembleForLog's checksum for serialized objects in `data`
        (uint8 CUDA tensor, modified in place): header.checksum of object i
        (bytes [off[i], off[i]+4)) = Crc32C over bytes [4, length[i])."""
        n = off.numel()
        rc = lib().ramcrc_assemble_objects_device(self._h, _ptr(data), _ptr(off), _ptr(length),
                                                  _ptr(out), n, _stream(stream))
        _check(rc, "ramcrc_assemble_objects_device")
        return out

    def assemble_objects_host(self, objects):
        """Same for host objects (writable contiguous numpy uint8 arrays),
        stamped in place."""
        for o in objects:
            if not (isinstance(o, np.ndarray) and o.dtype == np.uint8 and o.flags.c_contiguous
                    and o.flags.writeable):
                raise RamcrcError("objects must be writable contiguous numpy uint8 arrays")
        n = len(objects)
        ptrs = (_c.c_void_p * max(n, 1))(*[o.ctypes.data for o in objects])
        lens = np.array([o.size for o in objects], dtype=np.uint64)
        rc = lib().ramcrc_assemble_objects_host(self._h, ptrs, _c.c_void_p(lens.ctypes.data), n)
        _check(rc, "ramcrc_assemble_objects_host")

    def batch_host(self, buffers, init=None, finalize=True):
        """CRC a list of host buffers (bytes / numpy) on the GPU; returns np.uint32."""
        arrs = [_buf(b)[0] for b in buffers]
        n = len(arrs)
        ptrs = (_c.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
        lens = np.array([a.size for a in arrs], dtype=np.uint64)
        out = np.zeros(n, dtype=np.uint32)
        init_a = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
        rc = lib().ramcrc_batch_host(self._h, ptrs, _c.c_void_p(lens.ctypes.data),
                                     None if init_a is None else _c.c_void_p(init_a.ctypes.data),
                                     _c.c_void_p(out.ctypes.data), n,
                                     FINALIZE if finalize else 0)
        _check(rc, "ramcrc_batch_host")
        return out

    def stream_host(self, host_segments, seg_bytes, nseg, finalize=True, batch=8, depth=3):
        """Host-to-host streaming CRC (config 5).  host_segments: numpy uint8 or a
        pinned torch CPU tensor; returns np.uint32[nseg]."""
        out = np.zeros(nseg, dtype=np.uint32)
        if hasattr(host_segments, "data_ptr"):
            base = _c.c_void_p(host_segments.data_ptr())
        else:
            base = _c.c_void_p(np.ascontiguousarray(host_segments).ctypes.data)
        rc = lib().ramcrc_stream_host(self._h, base, seg_bytes, nseg, _c.c_void_p(out.ctypes.data),
                                      FINALIZE if finalize else 0, batch, depth)
        _check(rc, "ramcrc_stream_host")
        return out


# ------------------------------------------------------------ multi-GPU shard
def shard_range(nseg, nranks, rank):
    """[lo, hi) of segment indices rank `rank` of `nranks` owns (ramcrc_shard_range)."""
    lo, hi = _c.c_uint64(0), _c.c_uint64(0)
    _check(lib().ramcrc_shard_range(nseg, nranks, rank, _c.byref(lo), _c.byref(hi)),
           "ramcrc_shard_range")
    return lo.value, hi.value


def shard_unique_id():
    """128-byte RCCL unique id for ramcrc_shard_create_rank (bytes)."""
    buf = (_c.c_uint8 * 128)()
    _check(lib().ramcrc_shard_unique_id(buf), "ramcrc_shard_unique_id")
    return bytes(buf)


class _StdoutToStderr:
    """RCCL prints a version banner on stdout at communicator creation; a
    benchmark's stdout carries exactly one JSON line, so point fd 1 at
    stderr for the duration."""

    def __enter__(self):
        import sys
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        os.dup2(self.saved, 1)
        os.close(self.saved)


class Shard:
    """The recovery-scan shard of libramcrc (ramcrc_shard_*): scan of each
    rank's contiguous segment range + one RCCL all-gather of the CRCs.

    Shard(devices=[0, 1, ...])          one process, several GPUs (ncclCommInitAll)
    Shard(uid=..., nranks=N, rank=r, device=d)   one process per GPU (ncclCommInitRank)
    """

    def __init__(self, devices=None, uid=None, nranks=None, rank=None, device=None):
        h = _c.c_void_p()
        if devices is not None:
            arr = (_c.c_int * len(devices))(*devices)
            with _StdoutToStderr():
                rc = lib().ramcrc_shard_create_all(arr, len(devices), _c.byref(h))
            _check(rc, "ramcrc_shard_create_all")
        else:
            if uid is None or len(uid) != 128:
                raise RamcrcError("Shard needs devices=[...] or a 128-byte uid")
            buf = (_c.c_uint8 * 128).from_buffer_copy(uid)
            with _StdoutToStderr():
                rc = lib().ramcrc_shard_create_rank(buf, int(nranks), int(rank), int(device),
                                                    _c.byref(h))
            _check(rc, "ramcrc_shard_create_rank")
        self._h = h
        self.nlocal = int(lib().ramcrc_shard_local_count(h))

    def info(self, k=0):
        """(rank, device, stream handle, ctx handle) of local rank k."""
        r, d = _c.c_int(0), _c.c_int(0)
        st, cx = _c.c_void_p(), _c.c_void_p()
        _check(lib().ramcrc_shard_info(self._h, k, _c.byref(r), _c.byref(d), _c.byref(st),
                                       _c.byref(cx)), "ramcrc_shard_info")
        return r.value, d.value, st.value, cx.value

    def set_timing(self, enable=True, k=0):
        _check(lib().ramcrc_ctx_set_timing(_c.c_void_p(self.info(k)[3]), 1 if enable else 0),
               "ramcrc_ctx_set_timing")

    def scan_time(self, k=0):
        ms, n = _c.c_double(0), _c.c_uint64(0)
        _check(lib().ramcrc_ctx_scan_time(_c.c_void_p(self.info(k)[3]), _c.byref(ms), _c.byref(n)),
               "ramcrc_ctx_scan_time")
        return ms.value, n.value

    def segments(self, shards, seg_bytes, nseg, outs=None, finalize=True):
        """shards[k]: local rank k's segment range (CUDA uint8 tensor); outs[k]
        (int32 CUDA [nseg]) or None for the shard's own buffers."""
        if len(shards) != self.nlocal or (outs is not None and len(outs) != self.nlocal):
            raise RamcrcError("one shard (and output) per local rank")
        sp = (_c.c_void_p * self.nlocal)(*[t.data_ptr() if t is not None else 0 for t in shards])
        op = None if outs is None else (_c.c_void_p * self.nlocal)(*[t.data_ptr() for t in outs])
        _check(lib().ramcrc_shard_segments(self._h, sp, seg_bytes, nseg, op,
                                           FINALIZE if finalize else 0), "ramcrc_shard_segments")

    def sync(self):
        _check(lib().ramcrc_shard_sync(self._h), "ramcrc_shard_sync")

    def results(self, nseg, k=0):
        out = np.zeros(nseg, dtype=np.uint32)
        _check(lib().ramcrc_shard_results(self._h, k, _c.c_void_p(out.ctypes.data), nseg),
               "ramcrc_shard_results")
        return out

    def close(self):
        if self._h:
            lib().ramcrc_shard_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
