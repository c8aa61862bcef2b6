"""Segment batches for the walk/verify parity tests (CPU oracle vs GPU path).

Segments are built by the product's host append path and then damaged in the
ways Segment::checkMetadataIntegrity (src/Segment.cc:758-800) and
ObjectManager::replaySegment (src/ObjectManager.cc:659-669) detect.
"""
import numpy as np

from ramcloud_amd import ramcrc, segments, workloads

CAPACITY = 256 * 1024


def _seg(buf, i, cap=CAPACITY):
    return buf[i * cap:(i + 1) * cap]


def _set_u32(a, off, v):
    a[off:off + 4] = np.frombuffer(np.uint32(v & 0xFFFFFFFF).tobytes(), np.uint8)


def build_batch(oracle, seed=1234):
    """Returns (buf uint8[nseg*CAPACITY], certs uint32[nseg, 2], cases).  Crafted
    segments marked `recert` get a certificate that matches their (damaged)
    metadata, so the object verify still runs on them."""
    value_lens = [0, 1, 64, 100, 1000, 1024, 4000, 8192, 20000, 70000, 100000, 200000]
    rng = np.random.default_rng(seed)
    cases = []
    for v in value_lens:
        cases.append(("clean", v))
    for v in (64, 1024, 70000):
        cases += [("flip_value", v), ("flip_checksum", v), ("bad_cert", v),
                  ("short_cert", v), ("overrun", v)]
    cases += [("wrap", 1024), ("cycle", 1024), ("empty", 0), ("nonobj", 64), ("tiny_obj", 0),
              ("tail_header", 64)]
    nseg = len(cases)
    buf = np.empty(nseg * CAPACITY, np.uint8)
    certs = np.zeros((nseg, 2), np.uint32)
    recert = {"wrap", "nonobj", "tiny_obj", "tail_header"}
    for i, (kind, v) in enumerate(cases):
        s = _seg(buf, i)
        s[:] = workloads.splitmix_bytes_np(seed + i, CAPACITY)
        n, length, ck = ramcrc.segment_fill_objects(s, v, first_key=1000 * i)
        certs[i] = (length, ck)
        eb = segments.entry_bytes(v)
        lb = eb - 1 - (segments.OBJECT_OVERHEAD + v)
        if kind == "flip_value" and n:
            for k in rng.choice(n, size=min(3, n), replace=False):
                p = int(k) * eb + 1 + lb + segments.OBJECT_OVERHEAD + max(v - 1, 0)
                s[p] ^= 0x5A
        elif kind == "flip_checksum" and n:
            s[1 + lb] ^= 1   # first object's stored checksum
        elif kind == "bad_cert":
            certs[i, 1] ^= 0x1
        elif kind == "short_cert":
            certs[i, 0] = max(int(certs[i, 0]) - 3, 0)
        elif kind == "overrun" and n > 1:
            # second entry's length field claims more bytes than the segment has
            off = eb
            hdr = int(s[off])
            lbx = (hdr >> 6) + 1
            s[off + 1:off + 1 + lbx] = 0xFF
        elif kind == "wrap":
            # uint32 offset wrap: entry 0 claims 2^32 - 3 bytes, so the
            # reference's offset wraps to 2 and it keeps walking from there
            s[0] = 0x02 | (3 << 6)
            _set_u32(s, 1, (1 << 32) - 3)
        elif kind == "cycle":
            # entry 1 wraps back to offset 0: the reference would loop forever
            s[eb] = 0x02 | (3 << 6)
            _set_u32(s, eb + 1, (1 << 32) - eb - 5)
        elif kind == "empty":
            s[:] = 0
            certs[i] = (0, 0x48674BC7)   # src/SegmentTest.cc:369
        elif kind == "nonobj":
            s[0] = (s[0] & 0xC0) | 4     # first entry becomes a LOGDIGEST (replay checks no CRC)
        elif kind == "tiny_obj":
            # an OBJ entry shorter than Object::Header (length 5): counts as bad
            s[:8] = np.array([0x02, 5, 1, 2, 3, 4, 5, 0], np.uint8)
            s[7:] = 0
            certs[i] = (7, 0)
        elif kind == "tail_header":
            # certificate length past the last entry: the walk meets a header in
            # the zeroed tail (type 0, length 0) until the length
            certs[i, 0] = int(certs[i, 0]) + 16
        if kind in recert:
            _, ck, _, _ = oracle.check_metadata(s, int(certs[i, 0]), 0, segment=i)
            certs[i, 1] = ck
    return buf, certs, cases


def oracle_walk(oracle, buf, certs, nseg, cap=CAPACITY):
    """Per-segment (flags, checksum, entries) and the concatenated record table."""
    status = np.zeros((nseg, 4), np.uint32)
    tables = []
    for i in range(nseg):
        f, ck, n, t = oracle.check_metadata(_seg(buf, i, cap), int(certs[i, 0]), int(certs[i, 1]),
                                            segment=i, capacity=cap, table_cap=cap + 1)
        status[i, :3] = (f, ck, n)
        tables.append(t)
    table = np.concatenate(tables) if tables else np.zeros((0, 4), np.uint32)
    ok = (status[:, 0] & segments.SEG_OK) != 0
    bad_total, crc, bad = oracle.verify_objects(buf, cap, table, nseg, seg_ok=ok)
    status[:, 3] = bad
    return status, table, crc


def _log_entry(etype, payload):
    """EntryHeader + little-endian length + payload (src/Segment.h:114-195)."""
    n = len(payload)
    lb = 1 if n < 1 << 8 else 2 if n < 1 << 16 else 3 if n < 1 << 24 else 4
    return bytes([etype | ((lb - 1) << 6)]) + n.to_bytes(lb, "little") + payload


def replay_mix_entries(oracle, golden, seed):
    """Entries of every type ObjectManager::replaySegment checksums, valid and
    damaged: [(entry bytes, expect_ok)] with expect_ok None for types it does
    not checksum.  Anchored on the reference goldens: the object of
    src/ObjectTest.cc:171 and the tombstone of src/ObjectTest.cc:913."""
    rng = np.random.default_rng(seed)
    u32 = lambda v: int(v).to_bytes(4, "little")
    g = golden["object_checksums"][0]
    obj = u32(g["checksum"]) + bytes.fromhex(g["bytes"])
    t = golden["tombstone_checksums"][0]
    tb = bytes.fromhex(t["bytes"])
    tomb = tb[:28] + u32(t["checksum"]) + tb[28:]

    def flip(b, i):
        b = bytearray(b)
        b[i] ^= 0x40
        return bytes(b)

    def tomb_of(key):
        hdr = rng.integers(0, 256, 28, dtype=np.uint8).tobytes()
        return hdr + u32(oracle.crc32c(np.frombuffer(hdr + key, np.uint8))) + key

    def safe_of(ver, extra=b""):
        h = int(ver).to_bytes(8, "little")
        return h + u32(oracle.crc32c(np.frombuffer(h, np.uint8))) + extra

    def rand(n):
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()

    def crc(b):
        return u32(oracle.crc32c(np.frombuffer(b, np.uint8)))

    # PreparedOp (src/PreparedOp.h:63-100, src/PreparedOp.cc:177-190): 32-byte
    # header, checksum at [28, 32) over [0, 28) and the object from its byte 4
    def prep_of(o):
        h = rand(28)
        return h + crc(h + o[4:]) + o

    # PreparedOpTombstone (src/PreparedOp.h:142-185, src/PreparedOp.cc:271-282)
    def preptomb_of():
        h = rand(40)
        return h + crc(h)

    # TxDecisionRecord (src/TxDecisionRecord.h:62-128, .cc:209-223): participants
    # through Buffer::Iterator, uint32 24 * count clipped to the entry
    def txdec_of(count, present):
        h = rand(36) + u32(count) + rand(4)
        parts = rand(24 * present)
        tail = min((24 * count) & 0xFFFFFFFF, len(parts))
        return h + crc(h + parts[:tail]) + parts

    # ParticipantList (src/ParticipantList.h:81-113, .cc:96-110)
    def txplist_of(count):
        h = rand(16) + u32(count)
        parts = rand(24 * count)
        return h + crc(h + parts) + parts

    big = u32(0) + bytes.fromhex(g["bytes"])[:20] + rand(int(rng.integers(1500, 2500)))
    key = rng.integers(0, 256, int(rng.integers(300, 700)), dtype=np.uint8).tobytes()
    e = [
        (_log_entry(segments.LOG_ENTRY_TYPE_OBJ, obj), True),
        (_log_entry(segments.LOG_ENTRY_TYPE_OBJTOMB, tomb), True),
        (_log_entry(segments.LOG_ENTRY_TYPE_OBJTOMB, flip(tomb, 33)), False),   # key byte
        (_log_entry(segments.LOG_ENTRY_TYPE_OBJTOMB, flip(tomb, 29)), False),   # stored checksum
        (_log_entry(segments.LOG_ENTRY_TYPE_OBJTOMB, flip(tomb, 3)), False),    # header byte
        (_log_entry(segments.LOG_ENTRY_TYPE_OBJTOMB, tomb_of(key)), True),      # 2 length bytes
        (_log_entry(segments.LOG_ENTRY_TYPE_OBJTOMB, tomb_of(b"")), True),      # empty key
        (_log_entry(segments.LOG_ENTRY_TYPE_OBJTOMB, tomb[:20]), False),        # shorter than its header
        (_log_entry(segments.LOG_ENTRY_TYPE_SAFEVERSION, safe_of(rng.integers(1 << 62))), True),
        (_log_entry(segments.LOG_ENTRY_TYPE_SAFEVERSION, flip(safe_of(7), 2)), False),
        (_log_entry(segments.LOG_ENTRY_TYPE_SAFEVERSION, safe_of(9)[:8]), False),
        (_log_entry(segments.LOG_ENTRY_TYPE_SAFEVERSION, safe_of(11, b"\x01\x02\x03\x04")), True),
        (_log_entry(4, rng.integers(0, 256, 40, dtype=np.uint8).tobytes()), None),   # LOGDIGEST
        (_log_entry(segments.LOG_ENTRY_TYPE_OBJ, flip(obj, len(obj) - 1)), False),
        (_log_entry(segments.LOG_ENTRY_TYPE_PREP, prep_of(obj)), True),            # golden object inside
        (_log_entry(segments.LOG_ENTRY_TYPE_PREP, prep_of(big)), True),            # 2 length bytes
        (_log_entry(segments.LOG_ENTRY_TYPE_PREP, flip(prep_of(obj), 33)), True),  # object's own checksum: not covered
        (_log_entry(segments.LOG_ENTRY_TYPE_PREP, flip(prep_of(obj), 40)), False),  # object header byte
        (_log_entry(segments.LOG_ENTRY_TYPE_PREP, flip(prep_of(big), 32 + 24 + 1000)), False),
        (_log_entry(segments.LOG_ENTRY_TYPE_PREP, flip(prep_of(obj), 30)), False),  # stored checksum
        (_log_entry(segments.LOG_ENTRY_TYPE_PREP, prep_of(obj)[:50]), False),      # shorter than its headers
        (_log_entry(segments.LOG_ENTRY_TYPE_PREPTOMB, preptomb_of()), True),
        (_log_entry(segments.LOG_ENTRY_TYPE_PREPTOMB, flip(preptomb_of(), 39)), False),
        (_log_entry(segments.LOG_ENTRY_TYPE_PREPTOMB, preptomb_of()[:43]), False),
        (_log_entry(segments.LOG_ENTRY_TYPE_TXDECISION, txdec_of(3, 3)), True),
        (_log_entry(segments.LOG_ENTRY_TYPE_TXDECISION, txdec_of(0, 0)), True),
        (_log_entry(segments.LOG_ENTRY_TYPE_TXDECISION, txdec_of(5, 2)), True),     # count past the entry: clipped
        (_log_entry(segments.LOG_ENTRY_TYPE_TXDECISION, txdec_of(0xAAAAAAAB, 1)), True),  # 24 * count wraps to 8
        (_log_entry(segments.LOG_ENTRY_TYPE_TXDECISION, txdec_of(2, 2) + rand(5)), True),  # bytes past the list
        (_log_entry(segments.LOG_ENTRY_TYPE_TXDECISION, flip(txdec_of(3, 3), 100)), False),
        (_log_entry(segments.LOG_ENTRY_TYPE_TXDECISION, flip(txdec_of(3, 3), 37)), False),  # count byte
        (_log_entry(segments.LOG_ENTRY_TYPE_TXDECISION, txdec_of(0, 0)[:47]), False),
        (_log_entry(segments.LOG_ENTRY_TYPE_TXPLIST, txplist_of(4)), True),
        (_log_entry(segments.LOG_ENTRY_TYPE_TXPLIST, txplist_of(0)), True),
        (_log_entry(segments.LOG_ENTRY_TYPE_TXPLIST, flip(txplist_of(4), 60)), False),
        (_log_entry(segments.LOG_ENTRY_TYPE_TXPLIST, txplist_of(4)[:-1]), False),   # list past the entry
        (_log_entry(segments.LOG_ENTRY_TYPE_TXPLIST, txplist_of(1)[:23]), False),
        (_log_entry(7, rand(60)), None),                                            # RPCRESULT: not checked
    ]
    order = rng.permutation(len(e))
    return [e[i] for i in order]


def replay_crc_mask(buf, cap, table):
    """Records the replay checks leave a computed CRC for: those of a checked
    type holding their header, not OVERLONG, and (ParticipantList) whose list
    fits in the entry."""
    typ = table[:, 3] & 0x3F
    hdr = np.array([segments.REPLAY_HEADER_BYTES.get(int(t), 1 << 32) for t in typ], np.int64)
    m = (table[:, 2] >= hdr) & ((table[:, 3] & 0x100) == 0)
    for i in np.nonzero(m & (typ == segments.LOG_ENTRY_TYPE_TXPLIST))[0]:
        seg, off, ln, h = (int(v) for v in table[i])
        p = seg * cap + off + 1 + ((h >> 6) & 3) + 1
        count = int.from_bytes(bytes(buf[p + 16:p + 20]), "little")
        m[i] = (24 * count) & 0xFFFFFFFF <= ln - 24
    return m


def build_replay_mix(oracle, golden, nseg=8, seed=77, cap=CAPACITY):
    """nseg segments filled with replay_mix_entries groups; certificates from
    the oracle's metadata checksum.  Returns (buf, certs, expected bad per
    segment, expected checked records per segment)."""
    buf = np.zeros(nseg * cap, np.uint8)
    certs = np.zeros((nseg, 2), np.uint32)
    bad = np.zeros(nseg, np.uint32)
    checked = np.zeros(nseg, np.uint32)
    for i in range(nseg):
        s = _seg(buf, i, cap)
        pos, k = 0, 0
        while True:
            group = replay_mix_entries(oracle, golden, seed * 1000 + i * 100 + k)
            size = sum(len(b) for b, _ in group)
            if pos + size > cap - 64 or k == 3 + i:
                break
            for b, ok in group:
                s[pos:pos + len(b)] = np.frombuffer(b, np.uint8)
                pos += len(b)
                if ok is not None:
                    checked[i] += 1
                    bad[i] += 0 if ok else 1
            k += 1
        _, ck, _, _ = oracle.check_metadata(s, pos, 0)
        certs[i] = (pos, ck)
    return buf, certs, bad, checked


def tombstone_segments(oracle, nseg, cap, seed=99):
    """nseg segments packed with ObjectTombstones of empty keys -- 34-byte
    entries (EntryHeader, 1 length byte, 32-byte ObjectTombstone::Header,
    src/Object.h:285-338), smaller than any object entry -- each with a valid
    checksum (src/Object.cc:1042-1057).  Returns (buf, certs, counts)."""
    rng = np.random.default_rng(seed)
    buf = np.zeros(nseg * cap, np.uint8)
    certs = np.zeros((nseg, 2), np.uint32)
    counts = np.zeros(nseg, np.uint32)
    for i in range(nseg):
        s = _seg(buf, i, cap)
        pos = 0
        while pos + 34 <= cap:
            hdr = rng.integers(0, 256, 28, dtype=np.uint8).tobytes()
            tomb = hdr + int(oracle.crc32c(np.frombuffer(hdr, np.uint8))).to_bytes(4, "little")
            e = _log_entry(segments.LOG_ENTRY_TYPE_OBJTOMB, tomb)
            s[pos:pos + len(e)] = np.frombuffer(e, np.uint8)
            pos += len(e)
            counts[i] += 1
        _, ck, _, _ = oracle.check_metadata(s, pos, 0)
        certs[i] = (pos, ck)
    return buf, certs, counts


def mixed_segments(oracle, nseg, cap, seed=4242, fill=0.97):
    """nseg segments of log entries with random sizes and types: objects of
    24 B .. 200 KiB (tiny, 100 B-ish, 1 and 4 KiB, tens of KiB and larger
    than a 64 KiB part of the parallel walk), tombstones and safe versions,
    all payload bytes random (junk headers everywhere for the walk's
    synchronisation).  Entries fill `fill` of the capacity; the certificate
    matches the metadata.  Returns (buf, certs, counts)."""
    rng = np.random.default_rng(seed)
    buf = np.zeros(nseg * cap, np.uint8)
    certs = np.zeros((nseg, 2), np.uint32)
    counts = np.zeros(nseg, np.uint32)
    kinds = np.array([0, 1, 2, 3, 4, 5, 6])
    regimes = [np.array([0.20, 0.30, 0.20, 0.14, 0.08, 0.02, 0.06]),   # everything
               np.array([0.40, 0.45, 0.05, 0.02, 0.00, 0.00, 0.08]),   # dense small entries
               np.array([0.05, 0.10, 0.40, 0.40, 0.03, 0.00, 0.02]),   # 1-4 KiB objects
               np.array([0.10, 0.10, 0.05, 0.05, 0.30, 0.35, 0.05])]   # large entries
    for i in range(nseg):
        probs = regimes[i % len(regimes)]
        s = _seg(buf, i, cap)
        parts = []
        pos = 0
        while True:
            k = int(rng.choice(kinds, p=probs))
            if k == 0:
                n, t = int(rng.integers(24, 64)), segments.LOG_ENTRY_TYPE_OBJ
            elif k == 1:
                n, t = int(rng.integers(64, 200)), segments.LOG_ENTRY_TYPE_OBJ
            elif k == 2:
                n, t = int(rng.integers(900, 1200)), segments.LOG_ENTRY_TYPE_OBJ
            elif k == 3:
                n, t = int(rng.integers(3500, 4700)), segments.LOG_ENTRY_TYPE_OBJ
            elif k == 4:
                n, t = int(rng.integers(10000, 60000)), segments.LOG_ENTRY_TYPE_OBJ
            elif k == 5:
                n, t = int(rng.integers(70000, 200000)), segments.LOG_ENTRY_TYPE_OBJ
            else:
                n, t = int(rng.integers(32, 80)), int(rng.choice([segments.LOG_ENTRY_TYPE_OBJTOMB, 9]))
            e = _log_entry(t, rng.integers(0, 256, n, dtype=np.uint8).tobytes())
            if pos + len(e) > int(cap * fill):
                break
            parts.append(e)
            pos += len(e)
        blob = b"".join(parts)
        s[:len(blob)] = np.frombuffer(blob, np.uint8)
        counts[i] = len(parts)
        _, ck, _, _ = oracle.check_metadata(s, pos, 0, capacity=cap, table_cap=cap + 1)
        certs[i] = (pos, ck)
    return buf, certs, counts
