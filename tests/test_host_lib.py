"""libramcrc on the CPU: the library loads, exports every symbol include/ramcrc.h
declares, and its host update paths (the Crc32C::update replacement) agree with
the reference known answers and the oracle.  No GPU calls."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def header_symbols():
    text = open(os.path.join(ROOT, "include", "ramcrc.h")).read()
    return sorted(set(re.findall(r"\b(ramcrc_[a-z0-9_]+)\s*\(", text)))


def test_exports_every_declared_symbol(ramcrc):
    lib = ramcrc.lib()
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert len(header_symbols()) >= 15


def test_library_is_in_tree(ramcrc):
    assert os.path.realpath(ramcrc.lib_path()).startswith(os.path.realpath(ROOT))


@pytest.mark.parametrize("path", ["hw", "sw"])
def test_host_known_answers(golden, ramcrc, path):
    f = ramcrc.update_hw if path == "hw" else ramcrc.update_sw
    inp = bytes(golden["crc32c_test"]["input"])
    for i, want in enumerate(golden["crc32c_test"]["crcByLength"]):
        assert (~f(0xFFFFFFFF, inp[:i])) & 0xFFFFFFFF == want
    for c in golden["segment_certificates"] + golden["object_checksums"] + golden["tombstone_checksums"]:
        data = bytes.fromhex(c.get("stream", c.get("bytes")))
        assert (~f(0xFFFFFFFF, data)) & 0xFFFFFFFF == c["checksum"]


@pytest.mark.parametrize("path", ["hw", "sw"])
def test_host_random_cases(golden, golden_base, ramcrc, path):
    f = ramcrc.update_hw if path == "hw" else ramcrc.update_sw
    for off, L, init, raw in golden["random"]["cases"]:
        assert f(init, golden_base[off:off + L]) == raw, (off, L, init)


def test_host_interleaved_path_against_oracle(ramcrc, oracle_mod):
    # lengths around multiples of the 3 x 8 KiB interleave block
    rng = np.random.default_rng(3)
    buf = rng.integers(0, 256, 200000, dtype=np.uint8)
    for L in (24575, 24576, 24577, 49152 + 7, 73728, 150000):
        for off in (0, 1, 3, 7):
            s = int(rng.integers(0, 2 ** 32))
            want = oracle_mod.crc_raw(s, buf[off:off + L])
            assert ramcrc.update_hw(s, buf[off:off + L]) == want
            assert ramcrc.update_sw(s, buf[off:off + L]) == want


def test_shift_and_combine(ramcrc, oracle_mod):
    rng = np.random.default_rng(11)
    for _ in range(100):
        s = int(rng.integers(0, 2 ** 32))
        n = int(rng.integers(0, 1 << 40))
        assert ramcrc.shift(s, n) == oracle_mod.shift(s, n)
    a = rng.integers(0, 256, 5000, dtype=np.uint8)
    b = rng.integers(0, 256, 3333, dtype=np.uint8)
    ra, rb = ramcrc.update(0, a), ramcrc.update(0, b)
    assert ramcrc.combine(ra, rb, b.size) == ramcrc.update(0, np.concatenate([a, b]))


def test_pipeline_entry_points_reject_bad_arguments(ramcrc):
    """ramcrc_stream_create_cu_mask / ramcrc_stream_destroy / ramcrc_ctx_set_cus
    validate their arguments before any HIP call (runs without a GPU)."""
    import ctypes
    L = ramcrc.lib()
    out = ctypes.c_void_p()
    mask = (ctypes.c_uint32 * 9)(*([0xFFFFFFFF] * 9))
    assert L.ramcrc_stream_create_cu_mask(0, None, 1, ctypes.byref(out)) == -1
    assert L.ramcrc_stream_create_cu_mask(0, mask, 0, ctypes.byref(out)) == -1
    assert L.ramcrc_stream_create_cu_mask(0, mask, 9, ctypes.byref(out)) == -1
    assert L.ramcrc_stream_create_cu_mask(0, mask, 1, None) == -1
    assert L.ramcrc_stream_destroy(None) == -1
    assert L.ramcrc_ctx_set_cus(None, 0) == -1
