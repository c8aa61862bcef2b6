"""Generate tests/golden/segment_walk_ref.json (run in the build container only).

The byte layouts and expected outcomes of the reference's own walk tests,
as data:
  * src/SegmentTest.cc:598-620 (checkMetadataIntegrity_simple) and :622-648
    (checkMetadataIntegrity_badLength), once per segment size the test is
    instantiated with (:75-88: Segment::DEFAULT_SEGMENT_SIZE = 8 MiB, and the
    "extraFragmented" 66,560 bytes; seglets do not change the bytes a walk
    reads);
  * src/SegmentIteratorTest.cc:44-186 (certificates of empty segments and of
    buffers, isDone / next / getType / getLength record expectations).

Each case gives the segment capacity, the bytes written (offset, hex) over a
zeroed or splitmix64-filled background, the certificate the test checks
against, the outcome the reference test expects (OK / BAD_CHECKSUM /
PAST_LENGTH / PAST_CAPACITY, from its EXPECT_TRUE / EXPECT_FALSE and the
WARNING text it matches, src/Segment.cc:777-797) and, where the test pins
them, the entries the walk must find (offset, type, length).  Certificates
are computed as Segment::getAppendedLength does (src/Segment.cc:672-684:
the running checksum over every appended entry's header and length bytes,
src/Segment.cc:211,218, then the 4 head bytes) with RAMCloud::intelCrc32C
compiled from the reference (oracle/_ref), and the three the reference
states as constants (src/SegmentTest.cc:159,369,373) are checked against it.

Geometry: the device walkers take capacities that are multiples of 16.  The
SegmentIteratorTest buffers of 4 bytes (:85, :93) are given capacity 16
(bytes 4..15 random); their certificates end at or before byte 4, where the
walk stops, so the capacity rule (offset > capacity) cannot differ.  The
length-0 buffers of :67, :72 and :117 are given capacity 8192 (the test's
buf[8192], uninitialized there, random here); a certificate of length 0
walks nothing.

Usage:  python tests/golden/make_segment_ref.py
"""
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle import oracle  # noqa: E402

OBJ, OBJTOMB = 2, 3      # src/LogEntryTypes.h:35,38
MiB = 1 << 20
DEFAULT_SEGMENT_SIZE = 8 * MiB   # src/Segment.h (Segment::DEFAULT_SEGMENT_SIZE)
EXTRA_FRAGMENTED = 66560         # src/SegmentTest.cc:80-83


def header(etype, length):
    """EntryHeader(type, length) (src/Segment.h:134-149) + its length bytes."""
    nb = 1 if length < 0x100 else 2 if length < 0x10000 else 3 if length < 0x1000000 else 4
    return bytes([etype | ((nb - 1) << 6)]), struct.pack("<I", length)[:nb]


def result(data, state=0xFFFFFFFF):
    return (~oracle.ref_crc_raw(state, data)) & 0xFFFFFFFF


class Seg:
    """The append path's bytes and running checksum (src/Segment.cc:197-228)."""

    def __init__(self):
        self.meta = b""      # what Segment::checksum has covered
        self.writes = []
        self.head = 0
        self.records = []

    def append(self, etype, payload):
        h, lb = header(etype, len(payload))
        self.writes.append([self.head, (h + lb + payload).hex()])
        self.records.append([self.head, etype, len(payload)])
        self.meta += h + lb
        self.head += len(h) + len(lb) + len(payload)
        return self

    def cert(self, head=None):
        head = self.head if head is None else head
        return [head, result(self.meta + struct.pack("<I", head))]


def case(name, cite, cap, writes, cert, expect, records=None, fill="zero", head=None,
         certify=None):
    c = {"name": name, "cite": cite, "capacity": cap, "fill": fill, "writes": writes,
         "cert": cert, "expect": expect}
    if records is not None:
        c["records"] = records
    if head is not None:
        c["head"] = head                 # ramcrc_segments_certify_device input
        c["certify"] = certify           # {"cert": [...] or None, "flags": ...}
    return c


def segment_test_cases(cap, tag):
    out = []
    empty = Seg()
    out.append(case(f"simple_empty_{tag}", "src/SegmentTest.cc:603-605", cap, [], empty.cert(),
                    "OK", records=[], head=0, certify={"cert": empty.cert(), "flags": "OK"}))
    s = Seg().append(OBJ, b"asdfhasdf\0")
    cert = s.cert()
    out.append(case(f"simple_append_{tag}", "src/SegmentTest.cc:606-608", cap, s.writes, cert,
                    "OK", records=s.records, head=s.head, certify={"cert": cert, "flags": "OK"}))
    # payload scribble (:611): same metadata, same certificate
    scr = [[0, s.writes[0][1][:4] + b"ASDFHASDF\0".hex()]]
    out.append(case(f"simple_scribble_payload_{tag}", "src/SegmentTest.cc:610-612", cap, scr,
                    cert, "OK", records=s.records))
    # metadata scribble (:615-616): EntryHeader(OBJTOMB, 10) over byte 0
    h, _ = header(OBJTOMB, 10)
    meta = [[0, h.hex() + scr[0][1][2:]]]
    out.append(case(f"simple_scribble_metadata_{tag}", "src/SegmentTest.cc:614-619", cap, meta,
                    cert, "BAD_CHECKSUM"))
    # bad length (:627-637): EntryHeader(OBJ, 1 GiB) then the 4 length bytes
    # (segmentSize - 100), head = 1, certificate from a checksum that covers
    # no entry (nothing was appended)
    h, _ = header(OBJ, 1 << 30)
    c1 = [1, result(struct.pack("<I", 1))]
    w = [[0, (h + struct.pack("<I", cap - 100)).hex()]]
    out.append(case(f"badlength_past_length_{tag}", "src/SegmentTest.cc:627-637", cap, w, c1,
                    "PAST_LENGTH", head=1, certify={"cert": None, "flags": "PAST_LENGTH"}))
    w = [[0, (h + struct.pack("<I", cap)).hex()]]
    out.append(case(f"badlength_past_capacity_{tag}", "src/SegmentTest.cc:639-647", cap, w, c1,
                    "PAST_CAPACITY", head=1, certify={"cert": None, "flags": "PAST_CAPACITY"}))
    return out


def iterator_test_cases():
    out = []
    rnd = "splitmix:%d"
    empty = Seg()
    ce = empty.cert()
    assert ce == [0, 0x48674BC7]   # src/SegmentIteratorTest.cc:46-47, src/SegmentTest.cc:369
    out.append(case("iter_segment_empty", "src/SegmentIteratorTest.cc:44-50",
                    DEFAULT_SEGMENT_SIZE, [], ce, "OK", records=[]))
    out.append(case("iter_buffer_default_certificate", "src/SegmentIteratorTest.cc:65-70", 8192,
                    [], [0, 0], "BAD_CHECKSUM", fill=rnd % 1))
    out.append(case("iter_buffer_empty_certificate", "src/SegmentIteratorTest.cc:71-74", 8192,
                    [], ce, "OK", records=[], fill=rnd % 2))
    hi = Seg().append(OBJ, b"hi")
    ch = hi.cert()
    assert ch == [4, 0x87A632E2]   # src/SegmentTest.cc:159,189
    out.append(case("iter_buffer_old_certificate", "src/SegmentIteratorTest.cc:82-88", 16,
                    hi.writes, ce, "OK", records=[], fill=rnd % 3))
    out.append(case("iter_buffer_new_certificate", "src/SegmentIteratorTest.cc:90-100", 16,
                    hi.writes, ch, "OK", records=hi.records, fill=rnd % 4, head=4,
                    certify={"cert": ch, "flags": "OK"}))
    out.append(case("iter_buffer_longer_than_contents", "src/SegmentIteratorTest.cc:102-113",
                    8192, hi.writes, ch, "OK", records=hi.records, fill=rnd % 5))
    out.append(case("iter_buffer_null", "src/SegmentIteratorTest.cc:116-120", 16, [], ce, "OK",
                    records=[]))
    yo = Seg().append(OBJ, b"yo\0")
    assert yo.cert() == [5, 0x62F2F7F6]   # src/SegmentTest.cc:373
    out.append(case("iter_isDone", "src/SegmentIteratorTest.cc:122-135", DEFAULT_SEGMENT_SIZE,
                    yo.writes, yo.cert(), "OK", records=yo.records, head=5,
                    certify={"cert": yo.cert(), "flags": "OK"}))
    blam = Seg().append(OBJ, b"blam\0")
    assert blam.head == 7   # src/SegmentIteratorTest.cc:156
    out.append(case("iter_next", "src/SegmentIteratorTest.cc:137-165", DEFAULT_SEGMENT_SIZE,
                    blam.writes, blam.cert(), "OK", records=blam.records, head=7,
                    certify={"cert": blam.cert(), "flags": "OK"}))
    tg = Seg().append(OBJ, b"hi\0").append(OBJTOMB, b"hi\0")
    out.append(case("iter_getType", "src/SegmentIteratorTest.cc:167-176", DEFAULT_SEGMENT_SIZE,
                    tg.writes, tg.cert(), "OK", records=tg.records, head=tg.head,
                    certify={"cert": tg.cert(), "flags": "OK"}))
    gl = Seg().append(OBJ, b"hi\0").append(OBJTOMB, b"hihi\0")
    assert [r[2] for r in gl.records] == [3, 5]   # src/SegmentIteratorTest.cc:183-185
    out.append(case("iter_getLength", "src/SegmentIteratorTest.cc:178-186", DEFAULT_SEGMENT_SIZE,
                    gl.writes, gl.cert(), "OK", records=gl.records, head=gl.head,
                    certify={"cert": gl.cert(), "flags": "OK"}))
    return out


def main():
    if not oracle.ref_available():
        oracle.build(with_ref=True)
    cases = (segment_test_cases(DEFAULT_SEGMENT_SIZE, "8MiB")
             + segment_test_cases(EXTRA_FRAGMENTED, "66560")
             + iterator_test_cases())
    out = {"_source": __doc__.strip().splitlines()[0],
           "_flags": {"OK": 1, "PAST_CAPACITY": 2, "PAST_LENGTH": 4, "BAD_CHECKSUM": 8},
           "cases": cases}
    path = os.path.join(HERE, "segment_walk_ref.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(cases)} cases to {path}")


if __name__ == "__main__":
    main()
