"""Generate tests/golden/crc32c_golden.json (run in the build container only).

Every expected value in the fixture comes from the reference itself:
  * `crc32c_test` -- the input array and 82 CRCs held by the reference's own
    unit test, src/Crc32CTest.cc:27-58 (parsed from the file as data);
  * `segment_certificates` / `object_checksums` -- the golden constants held by
    src/SegmentTest.cc:159,369,373 and src/ObjectTest.cc:171,321,913, with the byte
    strings those tests checksum, rebuilt from the formats in src/Segment.cc:197-228,
    :672-684 (EntryHeader + length bytes + SegmentCertificate.segmentLength)
    and src/Object.cc:770-819 (header bytes [4,24) + keysAndValue);
  * everything else (`kat_*`, `random`, `chains`) -- outputs of
    oracle/_ref/libref_crc32c.so, i.e. RAMCloud::intelCrc32C compiled from
    /root/reference/src/Crc32C.h (see oracle/Makefile).

The reference never travels to the GPU box: only this JSON does.
Usage:  python tests/golden/make_golden.py
"""
import json
import os
import re
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle import oracle  # noqa: E402

REF_TEST = "/root/reference/src/Crc32CTest.cc"
MiB = 1 << 20


def parse_crc32c_test():
    text = open(REF_TEST).read()
    inp = re.search(r"input\[81\]\s*=\s*\{(.*?)\};", text, re.S).group(1)
    crcs = re.search(r"crcByLength\[sizeof\(input\) \+ 1\]\s*=\s*\{(.*?)\};", text, re.S).group(1)
    inp = [int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]+", inp)]
    crcs = [int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]+", crcs)]
    assert len(inp) == 81 and len(crcs) == 82
    return inp, crcs


def ref_raw(state, data):
    return oracle.ref_crc_raw(state, data)


def ref_result(data, state=0xFFFFFFFF):
    return (~ref_raw(state, data)) & 0xFFFFFFFF


def entry_bytes(type_, length):
    # EntryHeader (src/Segment.h:114-195): low 6 bits type, high 2 bits = lengthBytes-1
    nb = 1 if length < 0x100 else 2 if length < 0x10000 else 3 if length < 0x1000000 else 4
    return bytes([type_ | ((nb - 1) << 6)]) + struct.pack("<I", length)[:nb]


def segment_cert_stream(payloads):
    """Bytes Segment's running checksum covers, then certificate.segmentLength."""
    LOG_ENTRY_TYPE_OBJ = 2  # src/LogEntryTypes.h:29-35
    stream, head = b"", 0
    for p in payloads:
        hdr = entry_bytes(LOG_ENTRY_TYPE_OBJ, len(p))
        stream += hdr
        head += len(hdr) + len(p)
    return stream + struct.pack("<I", head), head


def main():
    if not oracle.ref_available():
        oracle.build(with_ref=True)
    inp, crcs = parse_crc32c_test()
    out = {"_source": __doc__.strip().splitlines()[0],
           "crc32c_test": {"input": inp, "crcByLength": crcs,
                           "cite": "src/Crc32CTest.cc:27-58"}}
    # sanity: the compiled reference reproduces its own unit-test table
    for i in range(82):
        assert ref_result(bytes(inp[:i])) == crcs[i], i

    certs = []
    for payloads, golden, cite in (([], 0x48674BC7, "src/SegmentTest.cc:369"),
                                   ([b"hi"], 0x87A632E2, "src/SegmentTest.cc:159,189"),
                                   ([b"yo!"], 0x62F2F7F6, "src/SegmentTest.cc:373")):
        stream, head = segment_cert_stream(payloads)
        assert ref_result(stream) == golden, (payloads, hex(ref_result(stream)))
        certs.append({"stream": stream.hex(), "segmentLength": head, "checksum": golden,
                      "cite": cite})
    out["segment_certificates"] = certs

    # Object checksum (src/Object.cc:805-819): CRC over header bytes [4,24)
    # {timestamp u32, version u64, tableId u64} then keysAndValue:
    # KeyCount(1B)=3, CumulativeKeyLength(u16)x3 = {3,6,9}, keys "ha\0" "hi\0"
    # "ho\0", value "YO!\0" (src/ObjectTest.cc:60-110 fixture; golden :171).
    hdr = struct.pack("<IQQ", 723, 75, 57)
    kv = bytes([3]) + struct.pack("<HHH", 3, 6, 9) + b"ha\0hi\0ho\0" + b"YO!\0"
    assert ref_result(hdr + kv) == 0xBB68333C
    # single-key object (src/ObjectTest.cc:117 fixture, golden :321): key "ha\0"
    # of table 57, value "YO!\0", version 75, timestamp 723
    kv1 = bytes([1]) + struct.pack("<H", 3) + b"ha\0" + b"YO!\0"
    assert ref_result(hdr + kv1) == 0xE86291D1
    out["object_checksums"] = [{"bytes": (hdr + kv).hex(), "checksum": 0xBB68333C,
                                "cite": "src/ObjectTest.cc:171"},
                               {"bytes": (hdr + kv1).hex(), "checksum": 0xE86291D1,
                                "cite": "src/ObjectTest.cc:321"}]
    # ObjectTombstone::computeChecksum (src/Object.cc:1042-1057): header bytes
    # before the trailing checksum {tableId u64, segmentId u64, objectVersion
    # u64, timestamp u32} (src/Object.h:301-336), then the key; fixture
    # src/ObjectTest.cc:843-866 (key "key!\0", table 572, segment 925, version
    # 58, timestamp 335), golden :913
    tomb = struct.pack("<QQQI", 572, 925, 58, 335) + b"key!\0"
    assert ref_result(tomb) == 0x5D60E8EF
    out["tombstone_checksums"] = [{"bytes": tomb.hex(), "checksum": 0x5D60E8EF,
                                   "cite": "src/ObjectTest.cc:913"}]

    kats = []
    for name, data in (("zeros_8MiB", np.zeros(8 * MiB, np.uint8)),
                       ("ff_8MiB", np.full(8 * MiB, 0xFF, np.uint8))):
        kats.append({"name": name, "crc": ref_result(data)})
    s42 = oracle.splitmix_bytes(42, 8 * MiB + 64)
    kats.append({"name": "splitmix42_first_8MiB", "seed": 42, "offset": 0, "len": 8 * MiB,
                 "crc": ref_result(s42[:8 * MiB])})
    kats.append({"name": "splitmix42_off1_8MiB_minus3", "seed": 42, "offset": 1,
                 "len": 8 * MiB - 3, "crc": ref_result(s42[1:1 + 8 * MiB - 3])})
    kats.append({"name": "splitmix42_prefixes_0_16", "seed": 42,
                 "crcs": [ref_result(s42[:i]) for i in range(17)]})
    # bench segment seeds (seed = 0x52414D43 + i per segment)
    for i in range(4):
        seg = oracle.splitmix_bytes(0x52414D43 + i, 8 * MiB)
        kats.append({"name": f"bench_segment_{i}", "seed": 0x52414D43 + i, "offset": 0,
                     "len": 8 * MiB, "crc": ref_result(seg)})
    out["kat"] = kats

    # randomized (offset, len, init) cases over one splitmix64 buffer
    seed = 0xC0FFEE
    base = oracle.splitmix_bytes(seed, 300000)
    rng = np.random.default_rng(1234)
    lens = list(range(0, 80)) + [95, 96, 97, 100, 127, 128, 129, 255, 256, 257, 1000,
                                 1023, 1024, 1025, 2047, 2048, 2049, 4095, 4096, 4097,
                                 8191, 8192, 16383, 65535, 65536, 65537, 131072, 262143,
                                 262144, 262145]
    lens += [int(x) for x in rng.integers(0, 20000, 60)]
    cases = []
    for L in lens:
        for _ in range(2):
            off = int(rng.integers(0, 32)) if L > 200000 else int(rng.integers(0, 300000 - L))
            init = [0xFFFFFFFF, 0, int(rng.integers(0, 2 ** 32))][int(rng.integers(0, 3))]
            raw = ref_raw(init, base[off:off + L])
            cases.append([off, L, init, raw])
    out["random"] = {"seed": seed, "base_len": 300000, "cases": cases,
                     "fields": ["offset", "len", "init", "raw_state"]}

    # chained updates (accumulatedVaried-style splits, src/Crc32CTest.cc:84-109)
    chains = []
    for _ in range(40):
        off = int(rng.integers(0, 1000))
        parts = [int(x) for x in rng.integers(0, 3000, int(rng.integers(1, 6)))]
        state = 0xFFFFFFFF
        pos = off
        states = []
        for p in parts:
            state = ref_raw(state, base[pos:pos + p])
            pos += p
            states.append(state)
        chains.append({"offset": off, "parts": parts, "raw_states": states})
    out["chains"] = chains

    with open(os.path.join(HERE, "crc32c_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "crc32c_golden.json"))


if __name__ == "__main__":
    main()
