"""Segment metadata walk and object checksums: the oracle against the
reference's golden values, and the product's host append path against the
oracle (CPU).  The GPU walk/verify is compared with the oracle in
tests/test_gpu_segments.py."""
import numpy as np
import pytest

from ramcloud_amd import segments, workloads

import segment_cases


def _entry(hdr, length_bytes, payload):
    return bytes([hdr]) + length_bytes + payload


@pytest.mark.parametrize("content,cert", [
    (b"", (0, 0x48674BC7)),        # src/SegmentTest.cc:366-370 (empty segment)
    (b"hi", (4, 0x87A632E2)),      # src/SegmentTest.cc:159-162, 189
    (b"yo!", (5, 0x62F2F7F6)),     # src/SegmentTest.cc:371-374
])
def test_oracle_metadata_goldens(oracle_mod, content, cert):
    seg = np.zeros(64, np.uint8)
    if content:
        e = _entry(0x02, bytes([len(content)]), content)   # LOG_ENTRY_TYPE_OBJ, 1 length byte
        seg[:len(e)] = np.frombuffer(e, np.uint8)
    flags, ck, n, table = oracle_mod.check_metadata(seg, cert[0], cert[1])
    assert flags == segments.SEG_OK
    assert ck == cert[1]
    assert n == (1 if content else 0)
    bad_flags, _, _, _ = oracle_mod.check_metadata(seg, cert[0], cert[1] ^ 1)
    assert bad_flags == segments.SEG_BAD_CHECKSUM


def test_oracle_object_golden(oracle_mod, golden):
    """src/ObjectTest.cc:171: the object's checksum is 0xBB68333C."""
    g = golden["object_checksums"][0]
    body = bytes.fromhex(g["bytes"])
    obj = np.uint32(g["checksum"]).tobytes() + body
    seg = np.zeros(256, np.uint8)
    e = _entry(0x02, bytes([len(obj)]), obj)
    seg[:len(e)] = np.frombuffer(e, np.uint8)
    _, ck, n, table = oracle_mod.check_metadata(seg, len(e), 0)
    assert n == 1 and table[0, 2] == len(obj)
    bad, crc, per = oracle_mod.verify_objects(seg, 256, table)
    assert bad == 0 and crc[0] == g["checksum"]
    seg[len(e) - 1] ^= 1
    bad, _, per = oracle_mod.verify_objects(seg, 256, table)
    assert bad == 1 and per[0] == 1


def test_benchmark_segment_counts():
    """Objects per 8 MiB segment of RecoverSegmentBenchmark."""
    expect = {64: 83055, 128: 50840, 256: 28532, 512: 15252, 1024: 7898, 2048: 4021, 8192: 1019}
    for v, n in expect.items():
        assert segments.objects_per_segment(8 << 20, v) == n


@pytest.mark.parametrize("value_len", [0, 1, 64, 100, 1000, 8192, 70000])
def test_fill_objects_matches_oracle(ramcrc, oracle_mod, value_len):
    cap = 256 * 1024
    base = workloads.splitmix_bytes_np(77 + value_len, cap)
    a = base.copy()
    b = base.copy()
    n, length, ck = ramcrc.segment_fill_objects(a, value_len, first_key=5)
    n2, length2, ck2 = oracle_mod.build_object_segment(b, value_len, first_key=5)
    assert (n, length, ck) == (n2, length2, ck2)
    assert np.array_equal(a, b)
    assert n == segments.objects_per_segment(cap, value_len)
    flags, ck3, nw, table = oracle_mod.check_metadata(a, length, ck)
    assert flags == segments.SEG_OK and ck3 == ck and nw == n
    bad, _, _ = oracle_mod.verify_objects(a, cap, table)
    assert bad == 0


def test_fill_objects_8mib_1k_values(ramcrc, oracle_mod):
    """One full RecoverSegmentBenchmark segment (valueLen 1024: 7,898 objects)."""
    cap = 8 << 20
    seg = workloads.splitmix_bytes_np(segments.REPLAY_SEED, cap)
    n, length, ck = ramcrc.segment_fill_objects(seg, 1024)
    assert n == 7898
    flags, ck2, nw, table = oracle_mod.check_metadata(seg, length, ck)
    assert flags == segments.SEG_OK and nw == 7898
    assert oracle_mod.verify_objects(seg, cap, table)[0] == 0


def test_oracle_damage_cases(oracle_mod):
    """Every damaged segment of the GPU parity batch fails in the expected way."""
    buf, certs, cases = segment_cases.build_batch(oracle_mod)
    status, table, crc = segment_cases.oracle_walk(oracle_mod, buf, certs, len(cases))
    for i, (kind, v) in enumerate(cases):
        f, bad = int(status[i, 0]), int(status[i, 3])
        if kind in ("clean", "empty", "nonobj", "tail_header"):
            assert f == segments.SEG_OK and bad == 0, (kind, v, f, bad)
        elif kind in ("flip_value", "flip_checksum"):
            assert f == segments.SEG_OK and bad >= 1, (kind, v, f, bad)
        elif kind == "bad_cert":
            assert f == segments.SEG_BAD_CHECKSUM, (kind, v, f)
        elif kind == "short_cert":
            assert f == segments.SEG_PAST_LENGTH, (kind, v, f)
        elif kind == "overrun":
            assert f == segments.SEG_PAST_CAPACITY, (kind, v, f)
        elif kind == "wrap":
            rows = table[table[:, 0] == i]
            assert rows[0, 3] & 0x100   # overlong; the walk went on at offset 2
        elif kind == "cycle":
            assert f == segments.SEG_CYCLE, (kind, f)
        elif kind == "tiny_obj":
            assert f == segments.SEG_OK and bad == 1, (kind, f, bad)


def test_oracle_tombstone_golden(oracle_mod, golden):
    """src/ObjectTest.cc:913: the tombstone's checksum is 0x5D60E8EF; replay
    (src/ObjectManager.cc:752-758) checks it over header [0, 28) + key."""
    t = golden["tombstone_checksums"][0]
    tb = bytes.fromhex(t["bytes"])
    tomb = tb[:28] + int(t["checksum"]).to_bytes(4, "little") + tb[28:]
    seg = np.zeros(256, np.uint8)
    e = segment_cases._log_entry(segments.LOG_ENTRY_TYPE_OBJTOMB, tomb)
    seg[:len(e)] = np.frombuffer(e, np.uint8)
    _, ck, n, table = oracle_mod.check_metadata(seg, len(e), 0)
    bad, crc, _ = oracle_mod.verify_objects(seg, 256, table)
    assert n == 1 and bad == 0 and crc[0] == t["checksum"]
    seg[len(e) - 1] ^= 1   # last key byte
    bad, _, _ = oracle_mod.verify_objects(seg, 256, table)
    assert bad == 1


def test_oracle_replay_mix(oracle_mod, golden):
    """Objects, tombstones and safe versions, valid and damaged, plus an
    unchecked type: the oracle's replay checks fail exactly the damaged ones."""
    buf, certs, bad, checked = segment_cases.build_replay_mix(oracle_mod, golden)
    status, table, crc = segment_cases.oracle_walk(oracle_mod, buf, certs, certs.shape[0])
    assert (status[:, 0] == segments.SEG_OK).all()
    assert np.array_equal(status[:, 3], bad)
    assert bad.sum() > 0 and (checked > bad).all()


def test_walk_cu_split_is_even():
    """The replay pipeline's walk CUs (bench._walk_cu_list): the same share of
    every XCD under both CU-id layouts (id % 8 and id // 32)."""
    import importlib.util
    import pathlib
    spec = importlib.util.spec_from_file_location(
        "bench_mod", pathlib.Path(__file__).resolve().parents[1] / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for walk in (64, 128):
        cus = bench._walk_cu_list(256, walk)
        assert len(set(cus)) == walk and max(cus) < 256
        assert np.all(np.bincount(np.array(cus) % 8, minlength=8) == walk // 8)
        assert np.all(np.bincount(np.array(cus) // 32, minlength=8) == walk // 8)
