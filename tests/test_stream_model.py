"""The lane-level model of the ordered-stream kernels (tools/stream_model.py,
the data flow of ramcloud_amd/csrc/stream.h) against a bitwise CRC32C on
random log-ordered batches: empty runs, entries around the 128-byte step,
gaps, spans of more than 64 entries (window refill), entries crossing one or
many spans (the fix-up chain) and raw output.  A design check of the
algorithm the GPU kernels implement; the kernels themselves are checked
against the oracle in tests/test_gpu_ordered.py."""
import os
import random
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import stream_model  # noqa: E402


@pytest.fixture(scope="module")
def tables():
    return stream_model.Tables()


@pytest.mark.parametrize("seed", range(12))
def test_model_matches_crc(tables, seed):
    rnd = random.Random(seed)
    for _ in range(15):
        n = rnd.randint(1, 160)
        pick = rnd.choice([[0, 1, 2, 3, 4, 5], [100, 127, 128, 129], [0, 3, 128, 300, 1000, 2500],
                           [0, 0, 0, 7]])
        lens = [rnd.choice(pick) for _ in range(n)]
        gaps = [rnd.choice([0, 0, 0, 1, 5, 130, 4095]) if rnd.random() < 0.3 else 0
                for _ in range(n)]
        pos, off = rnd.randint(0, 300), []
        for i in range(n):
            pos += gaps[i]
            off.append(pos)
            pos += lens[i]
        data = bytes(rnd.getrandbits(8) for _ in range(pos + 64))
        fin = rnd.random() < 0.8
        got, refused = stream_model.model(data, 0, off, lens, nspan=rnd.choice([1, 2, 3, 8, 40]),
                                          finalize=fin, T=tables)
        assert not refused
        for i in range(n):
            raw = stream_model.crc32c(data[off[i]:off[i] + lens[i]])
            want = (~raw & 0xFFFFFFFF) if fin else raw
            assert got[i] == want, (seed, i, off[i], lens[i])


@pytest.mark.parametrize("nspan", [2, 3, 7, 16])
def test_model_entries_on_span_starts(tables, nspan):
    """Entries of whole steps from a 128-byte aligned start, several of them
    longer than a span: starts fall exactly on span starts (the group injects
    the initial state there, the fix-up chains from that span)."""
    rnd = random.Random(nspan)
    lens = [128 * rnd.choice([0, 1, 2, 5, 9]) for _ in range(30)]
    off, pos = [], 256
    for ln in lens:
        off.append(pos)
        pos += ln
    data = bytes(rnd.getrandbits(8) for _ in range(pos + 64))
    got, refused = stream_model.model(data, 0, off, lens, nspan=nspan, T=tables)
    assert not refused
    for i in range(len(off)):
        assert got[i] == (~stream_model.crc32c(data[off[i]:off[i] + lens[i]])) & 0xFFFFFFFF, i


def test_model_refuses_unordered(tables):
    data = bytes(range(256)) * 40
    assert stream_model.model(data, 0, [0, 50], [100, 10], 4, T=tables)[1]      # overlap
    assert stream_model.model(data, 0, [0, 5000], [100, 10], 4, T=tables)[1]    # 4 KiB gap
