"""Recovery-segment verification on the GPU.

What a backup's RecoverySegmentBuilder::build and a recovery master's
ObjectManager::replaySegment do per replica, batched over many segments:

  1. Segment::checkMetadataIntegrity (src/Segment.cc:758-800) -- walk the
     length-prefixed entries, checksum their headers and lengths plus the
     certificate length, compare with the SegmentCertificate;
  2. for every object entry, Object::computeChecksum (src/Object.cc:805-819)
     compared with the checksum stored in its header
     (src/ObjectManager.cc:659-669).

Both run in libramcrc's kernels (ramcrc_segment_walk_device,
ramcrc_verify_objects_device); this module only allocates the tables and
builds synthetic segments shaped like nanobenchmarks/RecoverSegmentBenchmark.cc
(objects with 8-byte counter keys and splitmix64 value bytes) through the
host append path ramcrc_segment_fill_objects.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import ramcrc, workloads

SEG_OK = 1
SEG_PAST_CAPACITY = 2
SEG_PAST_LENGTH = 4
SEG_BAD_CHECKSUM = 8
SEG_TABLE_FULL = 16
SEG_CYCLE = 32
LOG_ENTRY_TYPE_OBJ = 2          # src/LogEntryTypes.h:35
LOG_ENTRY_TYPE_OBJTOMB = 3      # src/LogEntryTypes.h:38
LOG_ENTRY_TYPE_SAFEVERSION = 5  # src/LogEntryTypes.h:44
LOG_ENTRY_TYPE_PREP = 8         # src/LogEntryTypes.h:53
LOG_ENTRY_TYPE_PREPTOMB = 9     # src/LogEntryTypes.h:56
LOG_ENTRY_TYPE_TXDECISION = 10  # src/LogEntryTypes.h:59
LOG_ENTRY_TYPE_TXPLIST = 11     # src/LogEntryTypes.h:62
# Bytes a replayed record of each checked type must hold (ObjectManager::replaySegment,
# src/ObjectManager.cc:659-1100): Object::Header, ObjectTombstone::Header,
# ObjectSafeVersion::Header, PreparedOp::Header + Object::Header,
# PreparedOpTombstone::Header, TxDecisionRecord::Header, ParticipantList::Header.
REPLAY_HEADER_BYTES = {LOG_ENTRY_TYPE_OBJ: 24, LOG_ENTRY_TYPE_OBJTOMB: 32,
                       LOG_ENTRY_TYPE_SAFEVERSION: 12, LOG_ENTRY_TYPE_PREP: 56,
                       LOG_ENTRY_TYPE_PREPTOMB: 44, LOG_ENTRY_TYPE_TXDECISION: 48,
                       LOG_ENTRY_TYPE_TXPLIST: 24}

REPLAY_SEED = 0x5245504C   # "REPL": value bytes of segment i use seed REPLAY_SEED + i
OBJECT_OVERHEAD = 24 + 1 + 2 + 8   # Object::Header + KeyCount + CumulativeKeyLength + key
MIN_REPLAY_ENTRY = 1 + 1 + 12      # EntryHeader + 1 length byte + ObjectSafeVersion::Header


def entry_bytes(value_len):
    obj = OBJECT_OVERHEAD + value_len
    lb = 1 if obj < 1 << 8 else 2 if obj < 1 << 16 else 3 if obj < 1 << 24 else 4
    return 1 + lb + obj


def objects_per_segment(capacity, value_len):
    return capacity // entry_bytes(value_len)


def fill_segments_host(buf, nseg, capacity, value_len, first_key=0, stride=None, threads=8):
    """Turn nseg pre-filled segments of `buf` (numpy uint8; segment i at
    i*stride) into object segments.  Keys continue across segments as in
    RecoverSegmentBenchmark::run.  Returns certs uint32[nseg, 2] and the
    object counts."""
    stride = capacity if stride is None else stride
    per = objects_per_segment(capacity, value_len)
    certs = np.zeros((nseg, 2), np.uint32)
    counts = np.zeros(nseg, np.uint32)

    def one(i):
        seg = buf[i * stride: i * stride + capacity]
        n, length, ck = ramcrc.segment_fill_objects(seg, value_len, first_key + i * per)
        certs[i] = (length, ck)
        counts[i] = n

    with ThreadPoolExecutor(max_workers=max(1, threads)) as ex:
        list(ex.map(one, range(nseg)))
    return certs, counts


def object_segments_host(nseg, capacity, value_len, seed=REPLAY_SEED, threads=8):
    """numpy buffer of nseg object segments (values = splitmix64 bytes of seed + i)."""
    buf = np.empty(nseg * capacity, np.uint8)

    def gen(i):
        buf[i * capacity:(i + 1) * capacity] = workloads.splitmix_bytes_np(seed + i, capacity)

    with ThreadPoolExecutor(max_workers=max(1, threads)) as ex:
        list(ex.map(gen, range(nseg)))
    certs, counts = fill_segments_host(buf, nseg, capacity, value_len, threads=threads)
    return buf, certs, counts


class RecoveryVerify:
    """Device tables for walking and verifying batches of segments on one GPU.

    verify(d_segments, certs) returns the per-segment status tensor
    (int32 [nseg, 4]: flags, checksum, entries, bad_objects -- failed object,
    tombstone and safe-version checks) after both
    kernels ran on the current stream."""

    def __init__(self, ctx, nseg, capacity, stride=None, entries_cap=None, min_entry=None):
        self.ctx = ctx
        self.nseg = nseg
        self.capacity = capacity
        self.stride = capacity if stride is None else stride
        # Table sizing.  Every replayed record is at least a header byte, a
        # length byte and its type's header; the smallest is a safe version
        # (12 B, src/Object.h:402-427), so capacity // 14 + 1 records per
        # segment hold any segment -- but that worst case costs ~32 B of table
        # and scan scratch per 14 segment bytes (~15 GB for 512 x 8 MiB).
        #   entries_cap  fixed table; a walk that overflows it marks the
        #                segment TABLE_FULL (never OK) and check() raises;
        #   min_entry    fixed table sized for entries of at least that size;
        #   neither      a table for 128-byte entries on average that verify()
        #                grows (and walks again) when a walk finds more
        #                records -- at most once per batch shape.  verify() then
        #                waits for the walk's record count on every call, with
        #                or without check=True: no segment is left TABLE_FULL.
        self.grow = entries_cap is None and min_entry is None
        if entries_cap is None:
            per = self.GROW_START_ENTRY if self.grow else min_entry
            entries_cap = nseg * (capacity // per + 1)
        self._alloc(entries_cap)

    GROW_START_ENTRY = 128

    def _alloc(self, entries_cap):
        import torch
        dev = torch.device("cuda", self.ctx.device)
        self.entries = torch.zeros((entries_cap, 4), dtype=torch.int32, device=dev)
        self.n_entries = torch.zeros(1, dtype=torch.int64, device=dev)
        self.obj_crc = torch.zeros(entries_cap, dtype=torch.int32, device=dev)
        self.status = torch.zeros((self.nseg, 4), dtype=torch.int32, device=dev)

    def walk(self, d_segments, d_certs, stream=None):
        self.ctx.segment_walk(d_segments, self.stride, self.capacity, self.nseg, d_certs,
                              self.status, self.entries, self.n_entries, stream=stream)
        return self.status

    def verify_objects(self, d_segments, stream=None):
        self.ctx.verify_objects(d_segments, self.stride, self.entries, self.n_entries,
                                self.obj_crc, self.status, stream=stream)
        return self.status

    def verify(self, d_segments, d_certs, stream=None, check=False):
        """Walk + per-record verify.  check=True waits for the stream and raises
        if the record table overflowed (some segment not verified) or a launch
        was refused.  A growing table (no entries_cap / min_entry given) always
        reads the walked record count back (a host sync), and when the walk
        found more records than the table holds it is enlarged and the batch
        walked again, so that verify(check=False) never returns segments left
        TABLE_FULL; fixed tables never sync unless check=True, and take the
        fused walk + verify call (ramcrc_replay_verify_device)."""
        if not self.grow:
            st = self.ctx.replay_verify(d_segments, self.stride, self.capacity, self.nseg, d_certs,
                                        self.status, self.entries, self.n_entries, self.obj_crc,
                                        stream=stream)
            if check:
                self.check(stream)
            return st
        self.walk(d_segments, d_certs, stream)
        self.ctx.check(stream)
        n = int(self.n_entries.item())
        if n > self.entries.shape[0]:
            self._alloc(n + n // 8 + self.nseg)
            self.walk(d_segments, d_certs, stream)
        st = self.verify_objects(d_segments, stream)
        if check:
            self.check(stream)
        return st

    def check(self, stream=None):
        self.ctx.check(stream)
        n = int(self.n_entries.item())
        if n > self.entries.shape[0]:
            raise ramcrc.RamcrcError(
                f"segment walk found {n} records but the table holds {self.entries.shape[0]}: "
                "segments marked TABLE_FULL were not verified")
