"""GPU segment walk + object verify (ramcrc_segment_walk_device,
ramcrc_verify_objects_device) against the oracle's restatement of
Segment::checkMetadataIntegrity and Object::computeChecksum, bit for bit:
per-segment flags, metadata checksum, entry count and bad-object count, the
walked entry table, and every object CRC."""
import numpy as np
import pytest

from ramcloud_amd import segments

import segment_cases


def _sorted(table, extra=None):
    order = np.lexsort((table[:, 2], table[:, 1], table[:, 0]))
    return table[order], (None if extra is None else extra[order])


def _run(ramcrc, buf, certs, nseg, cap, entries_cap, serial=False, part_shift=0):
    import torch

    ctx = ramcrc.Context(0)
    if serial:
        ctx.set_serial_walk(True)
    if part_shift:
        ctx.set_walk_part_shift(part_shift)
    d = torch.from_numpy(buf).cuda()
    dc = torch.from_numpy(np.ascontiguousarray(certs).view(np.int32)).cuda()
    rv = segments.RecoveryVerify(ctx, nseg, cap, entries_cap=entries_cap)
    st = rv.verify(d, dc)
    torch.cuda.synchronize()
    n = int(rv.n_entries.item())
    k = min(n, entries_cap)
    table = rv.entries[:k].cpu().numpy().view(np.uint32)
    crc = rv.obj_crc[:k].cpu().numpy().view(np.uint32)
    return st.cpu().numpy().view(np.uint32), n, table, crc


@pytest.mark.gpu
@pytest.mark.parametrize("serial", [False, True], ids=["parallel_walk", "serial_walk"])
def test_walk_verify_damage_batch(ramcrc, oracle_mod, serial):
    """Clean segments of value lengths 0 .. 200000 (entries larger than the
    parallel walk's 64 KiB parts included), flipped values and checksums, bad
    and short certificates, overruns, a uint32_t offset wrap, a cycle, an
    empty segment, non-object and short-object entries, a certificate past
    the last entry: every status, record and object CRC equals the oracle's,
    with the parallel and the serial walker."""
    buf, certs, cases = segment_cases.build_batch(oracle_mod)
    nseg, cap = len(cases), segment_cases.CAPACITY
    exp_status, exp_table, exp_crc = segment_cases.oracle_walk(oracle_mod, buf, certs, nseg)
    status, n, table, crc = _run(ramcrc, buf, certs, nseg, cap, nseg * (cap + 1), serial)
    for i, c in enumerate(cases):
        assert np.array_equal(status[i], exp_status[i]), (c, status[i], exp_status[i])
    assert n == exp_table.shape[0]
    t_dev, c_dev = _sorted(table, crc)
    t_exp, c_exp = _sorted(exp_table, exp_crc)
    assert np.array_equal(t_dev, t_exp)
    ok_seg = (exp_status[:, 0] & segments.SEG_OK) != 0
    live = ((t_exp[:, 3] & 0x13F) == segments.LOG_ENTRY_TYPE_OBJ) & (t_exp[:, 2] >= 24) & ok_seg[t_exp[:, 0]]
    assert live.sum() > 1000
    assert np.array_equal(c_dev[live], c_exp[live])


@pytest.mark.gpu
def test_walk_verify_clean_1mib(ramcrc, oracle_mod):
    """64 x 1 MiB segments of 1 KiB-value objects: all pass, counts exact."""
    cap, nseg = 1 << 20, 64
    buf, certs, counts = segments.object_segments_host(nseg, cap, 1024)
    status, n, table, crc = _run(ramcrc, buf, certs, nseg, cap, nseg * 1024)
    assert (status[:, 0] == segments.SEG_OK).all()
    assert (status[:, 3] == 0).all()
    assert np.array_equal(status[:, 2], counts)
    assert np.array_equal(status[:, 1], certs[:, 1])
    assert n == counts.sum()


@pytest.mark.gpu
def test_walk_verify_strided_high_addresses(ramcrc, oracle_mod):
    """Segments spread over 4.5 GiB of device memory (stride 72 MiB): window
    and object addresses whose low 32 bits have bit 31 set, or that cross a
    4 GiB boundary, must be formed correctly (64-bit scalar addresses)."""
    import torch

    cap, nseg, stride = 256 * 1024, 64, 72 << 20
    buf, certs, counts = segments.object_segments_host(nseg, cap, 1000)
    d = torch.zeros(nseg * stride, dtype=torch.uint8, device="cuda")
    for i in range(nseg):
        d[i * stride:i * stride + cap].copy_(torch.from_numpy(buf[i * cap:(i + 1) * cap]))
    ctx = ramcrc.Context(0)
    dc = torch.from_numpy(np.ascontiguousarray(certs).view(np.int32)).cuda()
    rv = segments.RecoveryVerify(ctx, nseg, cap, stride=stride, entries_cap=int(counts.sum()) + 1)
    st = rv.verify(d, dc)
    torch.cuda.synchronize()
    status = st.cpu().numpy().view(np.uint32)
    assert (status[:, 0] == segments.SEG_OK).all()
    assert (status[:, 3] == 0).all()
    assert np.array_equal(status[:, 2], counts)
    n = int(rv.n_entries.item())
    table = rv.entries[:n].cpu().numpy().view(np.uint32)
    _, crc_exp, _ = oracle_mod.verify_objects(buf, cap, table, nseg)
    assert np.array_equal(rv.obj_crc[:n].cpu().numpy().view(np.uint32), crc_exp)


@pytest.mark.gpu
def test_walk_table_full_flag(ramcrc, oracle_mod):
    """A table too small for the walk: records dropped and flagged, count still
    exact; a segment that lost records is never reported OK (it was not
    verified), the others are, and RecoveryVerify.check raises."""
    import torch
    cap, nseg = 1 << 18, 4
    buf, certs, counts = segments.object_segments_host(nseg, cap, 100)
    status, n, table, crc = _run(ramcrc, buf, certs, nseg, cap, 100)
    assert n == counts.sum()
    full = (status[:, 0] & segments.SEG_TABLE_FULL) != 0
    assert full.any()
    assert ((status[full, 0] & segments.SEG_OK) == 0).all()
    assert (status[~full, 0] == segments.SEG_OK).all()
    assert np.array_equal(status[:, 1], certs[:, 1])   # the metadata checksum is still reported
    ctx = ramcrc.Context(0)
    rv = segments.RecoveryVerify(ctx, nseg, cap, entries_cap=100)
    d = torch.from_numpy(buf).cuda()
    dc = torch.from_numpy(np.ascontiguousarray(certs).view(np.int32)).cuda()
    with pytest.raises(ramcrc.RamcrcError):
        rv.verify(d, dc, check=True)


@pytest.mark.gpu
def test_walk_tombstone_only_default_table(ramcrc, oracle_mod, golden):
    """Segments packed with short tombstones (34-byte entries, below the object
    minimum the round-1 default table assumed) with the default table: every
    record is walked and verified, no segment is TABLE_FULL."""
    import torch
    cap, nseg = 1 << 16, 8
    buf, certs, counts = segment_cases.tombstone_segments(oracle_mod, nseg, cap)
    ctx = ramcrc.Context(0)
    rv = segments.RecoveryVerify(ctx, nseg, cap)
    d = torch.from_numpy(buf).cuda()
    dc = torch.from_numpy(np.ascontiguousarray(certs).view(np.int32)).cuda()
    st = rv.verify(d, dc, check=True).cpu().numpy().view(np.uint32)
    assert (st[:, 0] == segments.SEG_OK).all()
    assert np.array_equal(st[:, 2], counts)
    assert (st[:, 3] == 0).all()
    exp_status, _, _ = segment_cases.oracle_walk(oracle_mod, buf, certs, nseg, cap=cap)
    assert np.array_equal(st, exp_status)


@pytest.mark.gpu
def test_walk_small_records_default_table_no_check(ramcrc, oracle_mod):
    """Segments of 64-byte-value objects (101-byte entries, below the 128 bytes
    the growing table starts from) with the default table and check=False:
    verify() itself grows the table and walks again, so every segment is
    verified (OK, exact counts), none is left TABLE_FULL."""
    import torch
    cap, nseg = 1 << 18, 8
    buf, certs, counts = segments.object_segments_host(nseg, cap, 64)
    ctx = ramcrc.Context(0)
    rv = segments.RecoveryVerify(ctx, nseg, cap)
    assert rv.entries.shape[0] < counts.sum()
    d = torch.from_numpy(buf).cuda()
    dc = torch.from_numpy(np.ascontiguousarray(certs).view(np.int32)).cuda()
    st = rv.verify(d, dc).cpu().numpy().view(np.uint32)
    assert (st[:, 0] == segments.SEG_OK).all()
    assert np.array_equal(st[:, 2], counts)
    assert (st[:, 3] == 0).all()
    rv.check()


@pytest.mark.gpu
@pytest.mark.parametrize("value_len", [64, 128, 256, 1024, 8192, 100000])
def test_parallel_walk_8mib_vs_oracle(ramcrc, oracle_mod, value_len):
    """8 MiB object segments (128 parts of the parallel walk) at the
    RecoverSegmentBenchmark value sizes: entries from 101 B to larger than a
    part (128 B values: objects of two windows, the multi-window tiny phase's
    ring, and a layout that holds a same-stride junk chain; 256 B: three
    windows); one segment with a damaged length in its middle (the chain
    derails: every later part misguessed) and one with a wrong certificate.
    Status, records and object CRCs equal the oracle's and the serial
    walker's."""
    import torch
    cap, nseg = 8 << 20, 6
    buf, certs, counts = segments.object_segments_host(nseg, cap, value_len, threads=8)
    eb = segments.entry_bytes(value_len)
    mid = (counts[1] // 2) * eb + cap   # segment 1: an entry in the middle claims 3 bytes more
    lbx = (int(buf[mid]) >> 6) + 1
    ln = int.from_bytes(bytes(buf[mid + 1:mid + 1 + lbx]), "little") + 3
    buf[mid + 1:mid + 1 + lbx] = np.frombuffer(ln.to_bytes(4, "little")[:lbx], np.uint8)
    certs[2, 1] ^= 0x10
    exp_status, exp_table, exp_crc = segment_cases.oracle_walk(oracle_mod, buf, certs, nseg, cap=cap)
    got = {}
    for serial, shift in ((False, 0), (False, 13), (True, 0)):
        status, n, table, crc = _run(ramcrc, buf, certs, nseg, cap, int(counts.sum()) * 2 + 1024,
                                     serial, shift)
        assert np.array_equal(status, exp_status), (serial, status, exp_status)
        assert n == exp_table.shape[0]
        t_dev, c_dev = _sorted(table, crc)
        t_exp, c_exp = _sorted(exp_table, exp_crc)
        assert np.array_equal(t_dev, t_exp)
        ok_seg = (exp_status[:, 0] & segments.SEG_OK) != 0
        live = ((t_exp[:, 3] & 0x13F) == segments.LOG_ENTRY_TYPE_OBJ) & (t_exp[:, 2] >= 24) & ok_seg[t_exp[:, 0]]
        assert np.array_equal(c_dev[live], c_exp[live])
        got[serial] = status
    assert (exp_status[[0, 3, 4, 5], 0] == segments.SEG_OK).all()
    torch.cuda.synchronize()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [4242, 77])
def test_parallel_walk_mixed_sizes_vs_oracle(ramcrc, oracle_mod, seed):
    """8 MiB segments of random-size entries (objects of 24 B .. 200 KiB,
    tombstones, prepared-op tombstones) with random payloads: junk headers
    everywhere, parts holding hundreds of entries (their records spill), parts
    inside an entry (jumped over), guesses that meet the chain after a few
    entries or never.  One segment gets a damaged length in its middle.
    Status, records and object CRCs equal the oracle's, with both walkers."""
    import torch
    cap, nseg = 8 << 20, 6
    buf, certs, counts = segment_cases.mixed_segments(oracle_mod, nseg, cap, seed=seed)
    # segment 3: an entry near the middle claims 5 bytes more (the chain derails)
    s3 = buf[3 * cap:4 * cap]
    _, _, _, t3 = oracle_mod.check_metadata(s3, int(certs[3, 0]), int(certs[3, 1]), segment=3,
                                            capacity=cap, table_cap=cap + 1)
    mid = int(t3[len(t3) // 2, 1])
    lbx = (int(s3[mid]) >> 6) + 1
    ln = int.from_bytes(bytes(s3[mid + 1:mid + 1 + lbx]), "little") + 5
    s3[mid + 1:mid + 1 + lbx] = np.frombuffer(ln.to_bytes(4, "little")[:lbx], np.uint8)
    exp_status, exp_table, exp_crc = segment_cases.oracle_walk(oracle_mod, buf, certs, nseg, cap=cap)
    for serial, shift in ((False, 0), (False, 13), (False, 14), (False, 17), (True, 0)):
        status, n, table, crc = _run(ramcrc, buf, certs, nseg, cap, int(counts.sum()) * 2 + 4096,
                                     serial, shift)
        assert np.array_equal(status, exp_status), (serial, status, exp_status)
        assert n == exp_table.shape[0]
        t_dev, c_dev = _sorted(table, crc)
        t_exp, c_exp = _sorted(exp_table, exp_crc)
        assert np.array_equal(t_dev, t_exp)
        ok_seg = (exp_status[:, 0] & segments.SEG_OK) != 0
        live = ((t_exp[:, 3] & 0x13F) == segments.LOG_ENTRY_TYPE_OBJ) & (t_exp[:, 2] >= 24) & ok_seg[t_exp[:, 0]]
        assert np.array_equal(c_dev[live], c_exp[live])
    assert (exp_status[[0, 1, 2, 4, 5], 0] & segments.SEG_OK).all()
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_walk_verify_replay_mix(ramcrc, oracle_mod, golden):
    """Tombstones (src/ObjectManager.cc:752-758), safe versions (:873-880) and
    the transaction records (prepared ops and their tombstones, decision
    records, participant lists: :956-1084) beside objects, valid and damaged: per-segment failure counts, the record
    table and every computed CRC equal the oracle's."""
    buf, certs, bad, _ = segment_cases.build_replay_mix(oracle_mod, golden)
    nseg, cap = certs.shape[0], segment_cases.CAPACITY
    exp_status, exp_table, exp_crc = segment_cases.oracle_walk(oracle_mod, buf, certs, nseg)
    assert np.array_equal(exp_status[:, 3], bad)
    status, n, table, crc = _run(ramcrc, buf, certs, nseg, cap, nseg * 4096)
    assert np.array_equal(status, exp_status)
    assert n == exp_table.shape[0]
    t_dev, c_dev = _sorted(table, crc)
    t_exp, c_exp = _sorted(exp_table, exp_crc)
    assert np.array_equal(t_dev, t_exp)
    typ = t_exp[:, 3] & 0x3F
    live = segment_cases.replay_crc_mask(buf, cap, t_exp)
    for t in (segments.LOG_ENTRY_TYPE_OBJTOMB, segments.LOG_ENTRY_TYPE_PREP,
              segments.LOG_ENTRY_TYPE_TXDECISION, segments.LOG_ENTRY_TYPE_TXPLIST):
        assert (typ[live] == t).sum() > 10
    assert np.array_equal(c_dev[live], c_exp[live])


@pytest.mark.gpu
def test_walk_verify_on_cu_masked_streams(ramcrc, oracle_mod, golden):
    """The replay pipeline's plumbing: the walk on one CU-masked stream, the
    object verify on the complementary mask with a context sized for those
    CUs (ramcrc_stream_create_cu_mask / ramcrc_ctx_set_cus) give the same
    status, records and CRCs as the oracle."""
    import torch
    buf, certs, bad, _ = segment_cases.build_replay_mix(oracle_mod, golden)
    nseg, cap = certs.shape[0], segment_cases.CAPACITY
    exp_status, exp_table, exp_crc = segment_cases.oracle_walk(oracle_mod, buf, certs, nseg)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    walk_cus = [c for c in range(ncu) if (c // 8) % 4 == 0]
    rest = [c for c in range(ncu) if (c // 8) % 4 != 0]
    s_walk, s_scan = ramcrc.CuMaskStream(0, walk_cus), ramcrc.CuMaskStream(0, rest)
    ctx_walk, ctx_scan = ramcrc.Context(0), ramcrc.Context(0)
    ctx_scan.set_cus(len(rest))
    try:
        d = torch.from_numpy(buf).cuda()
        dc = torch.from_numpy(np.ascontiguousarray(certs).view(np.int32)).cuda()
        rv = segments.RecoveryVerify(ctx_scan, nseg, cap, entries_cap=nseg * 4096)
        torch.cuda.synchronize()
        ctx_walk.segment_walk(d, rv.stride, rv.capacity, nseg, dc, rv.status, rv.entries,
                              rv.n_entries, stream=s_walk)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.ExternalStream(s_walk.handle))
        torch.cuda.ExternalStream(s_scan.handle).wait_event(ev)
        rv.verify_objects(d, stream=s_scan)
        torch.cuda.synchronize()
        status = rv.status.cpu().numpy().view(np.uint32)
        n = int(rv.n_entries.item())
        table = rv.entries[:n].cpu().numpy().view(np.uint32)
        crc = rv.obj_crc[:n].cpu().numpy().view(np.uint32)
    finally:
        s_walk.destroy()
        s_scan.destroy()
    assert np.array_equal(status, exp_status)
    assert np.array_equal(status[:, 3], bad)
    t_dev, c_dev = _sorted(table, crc)
    t_exp, c_exp = _sorted(exp_table, exp_crc)
    assert np.array_equal(t_dev, t_exp)
    live = segment_cases.replay_crc_mask(buf, cap, t_exp)
    assert np.array_equal(c_dev[live], c_exp[live])
