"""Pin the oracle (oracle/crc32c_oracle.c) before trusting it as the checker.

Known answers come from the reference's own tests (src/Crc32CTest.cc:27-58,
src/SegmentTest.cc:159,369,373, src/ObjectTest.cc:171) and from the reference's
compiled intelCrc32C (oracle/_ref, via tests/golden/make_golden.py).
"""
import numpy as np
import pytest

IMPLS = [0, 1, 2]  # sse4.2 restatement, slicing-by-8 restatement, bitwise


@pytest.mark.parametrize("impl", IMPLS)
def test_crc32c_test_single(golden, oracle_mod, impl):
    inp = bytes(golden["crc32c_test"]["input"])
    crcs = golden["crc32c_test"]["crcByLength"]
    for i in range(len(inp) + 1):
        assert oracle_mod.crc32c(inp[:i], impl) == crcs[i], i


@pytest.mark.parametrize("impl", IMPLS)
def test_crc32c_test_accumulated(golden, oracle_mod, impl):
    inp = bytes(golden["crc32c_test"]["input"])
    crcs = golden["crc32c_test"]["crcByLength"]
    s = 0xFFFFFFFF
    assert (~s) & 0xFFFFFFFF == crcs[0]
    for i in range(len(inp)):
        s = oracle_mod.crc_raw(s, inp[i:i + 1], impl)
        assert (~s) & 0xFFFFFFFF == crcs[i + 1]


@pytest.mark.parametrize("impl", IMPLS)
def test_segment_and_object_goldens(golden, oracle_mod, impl):
    for c in golden["segment_certificates"] + golden["object_checksums"] + golden["tombstone_checksums"]:
        data = bytes.fromhex(c.get("stream", c.get("bytes")))
        assert oracle_mod.crc32c(data, impl) == c["checksum"], c["cite"]


@pytest.mark.parametrize("impl", [0, 1])
def test_random_cases_from_reference(golden, golden_base, oracle_mod, impl):
    for off, L, init, raw in golden["random"]["cases"]:
        assert oracle_mod.crc_raw(init, golden_base[off:off + L], impl) == raw, (off, L, init)


def test_bitwise_random_subset(golden, golden_base, oracle_mod):
    for off, L, init, raw in golden["random"]["cases"][:200]:
        if L <= 20000:
            assert oracle_mod.crc_raw(init, golden_base[off:off + L], 2) == raw


def test_chains_from_reference(golden, golden_base, oracle_mod):
    for ch in golden["chains"]:
        s, pos = 0xFFFFFFFF, ch["offset"]
        for p, want in zip(ch["parts"], ch["raw_states"]):
            s = oracle_mod.crc_raw(s, golden_base[pos:pos + p])
            pos += p
            assert s == want


def test_large_kats(golden, oracle_mod):
    MiB = 1 << 20
    for k in golden["kat"]:
        if k["name"] == "zeros_8MiB":
            assert oracle_mod.crc32c(np.zeros(8 * MiB, np.uint8)) == k["crc"]
        elif k["name"] == "ff_8MiB":
            assert oracle_mod.crc32c(np.full(8 * MiB, 0xFF, np.uint8)) == k["crc"]
        elif k["name"] == "splitmix42_prefixes_0_16":
            buf = oracle_mod.splitmix_bytes(42, 64)
            assert [oracle_mod.crc32c(buf[:i]) for i in range(17)] == k["crcs"]
        elif "seed" in k:
            buf = oracle_mod.splitmix_bytes(k["seed"], k["offset"] + k["len"] + 8)
            assert oracle_mod.crc32c(buf[k["offset"]:k["offset"] + k["len"]]) == k["crc"], k["name"]


def test_linearity_identities(oracle_mod):
    """raw(s, M) = X^|M|(s) ^ raw(0, M);  raw(0, A||B) = X^|B|(raw(0,A)) ^ raw(0,B)."""
    rng = np.random.default_rng(7)
    for _ in range(50):
        a = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8)
        b = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8)
        s = int(rng.integers(0, 2 ** 32))
        assert oracle_mod.crc_raw(s, a) == oracle_mod.shift(s, a.size) ^ oracle_mod.crc_raw(0, a)
        ab = np.concatenate([a, b])
        assert oracle_mod.crc_raw(0, ab) == (oracle_mod.shift(oracle_mod.crc_raw(0, a), b.size)
                                             ^ oracle_mod.crc_raw(0, b))


def test_oracle_against_compiled_reference(oracle_mod):
    if not oracle_mod.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(99)
    buf = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    for _ in range(300):
        off = int(rng.integers(0, 64))
        L = int(rng.integers(0, 70000))
        s = int(rng.integers(0, 2 ** 32))
        want = oracle_mod.ref_crc_raw(s, buf[off:off + L])
        assert oracle_mod.crc_raw(s, buf[off:off + L], 0) == want
        assert oracle_mod.crc_raw(s, buf[off:off + L], 1) == want


def test_segments_mt_matches_serial(oracle_mod):
    seg = 1 << 16
    buf = oracle_mod.splitmix_bytes(5, 24 * seg)
    serial = [oracle_mod.crc32c(buf[i * seg:(i + 1) * seg]) for i in range(24)]
    assert list(oracle_mod.segments(buf, seg, 24, threads=4)) == serial
    if oracle_mod.ref_available():
        assert list(oracle_mod.segments(buf, seg, 24, threads=3, use_ref=True)) == serial
