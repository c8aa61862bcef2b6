"""The reference's own walk scenarios (src/SegmentTest.cc:598-648,
src/SegmentIteratorTest.cc:44-186) rebuilt from the committed fixture
tests/golden/segment_walk_ref.json (made by tests/golden/make_segment_ref.py)."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "segment_walk_ref.json")


def load():
    with open(FIXTURE) as f:
        return json.load(f)


def flag_value(name):
    return load()["_flags"][name]


def build(case, oracle):
    """The case's segment: capacity bytes, zeroed or splitmix64-filled, with
    the case's writes applied in order."""
    cap = case["capacity"]
    fill = case["fill"]
    if fill == "zero":
        seg = np.zeros(cap, np.uint8)
    else:
        seed = int(fill.split(":")[1])
        seg = np.array(oracle.splitmix_bytes(seed, cap), dtype=np.uint8)
    for off, hexbytes in case["writes"]:
        b = np.frombuffer(bytes.fromhex(hexbytes), np.uint8)
        seg[off:off + b.size] = b
    return seg


def batches(oracle):
    """Cases grouped by capacity: {cap: (cases, buf, certs uint32[n, 2])}."""
    out = {}
    for c in load()["cases"]:
        out.setdefault(c["capacity"], []).append(c)
    res = {}
    for cap, cases in out.items():
        buf = np.concatenate([build(c, oracle) for c in cases])
        certs = np.array([c["cert"] for c in cases], dtype=np.uint32)
        res[cap] = (cases, buf, certs)
    return res


def records_of(table):
    """[offset, type, length] of walk records (segment, offset, length, header)."""
    return [[int(r[1]), int(r[3]) & 0x3F, int(r[2])] for r in table]
