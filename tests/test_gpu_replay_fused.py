"""ramcrc_replay_verify_device: the walk and the replay checks in one call.

It must give exactly what ramcrc_segment_walk_device followed by
ramcrc_verify_objects_device gives (status words, record table, object CRCs),
on RecoverSegmentBenchmark-shaped segments
(nanobenchmarks/RecoverSegmentBenchmark.cc:123-146) of 64-byte values -- where
every record is a one-window object and the fused call skips the binning pass
-- with one object's value damaged (bad_objects) and one certificate damaged
(the whole segment fails, its records are inactive); and on a batch whose
records are not all one-window objects (1 KiB values), where it takes the
binned path.  Expected statuses come from the fill's certificate and the
damage, independently of either device path."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

MiB = 1 << 20
SEG = 8 * MiB


def _batch(ramcrc, ctx, nseg, vlen, first_seed=0x5A17):
    from ramcloud_amd import workloads
    d = torch.empty(nseg * SEG, dtype=torch.uint8, device="cuda")
    certs = torch.zeros((nseg, 2), dtype=torch.int32, device="cuda")
    workloads.splitmix_fill_segments(d, SEG, first_seed)
    per, length, ck = ctx.fill_objects(d, SEG, SEG, nseg, vlen, first_key=0, certs=certs)
    torch.cuda.synchronize()
    return d, certs, per, ck


def _run(ramcrc, ctx, d, certs, nseg, cap, fused):
    from ramcloud_amd import segments
    rv = segments.RecoveryVerify(ctx, nseg, SEG, entries_cap=cap)
    if fused:
        st = rv.verify(d, certs, check=True)   # fixed table: the fused call
    else:
        rv.walk(d, certs)
        st = rv.verify_objects(d)
        rv.check()
    torch.cuda.synchronize()
    n = int(rv.n_entries.item())
    table = rv.entries[:n].cpu().numpy().view(np.uint32)
    crc = rv.obj_crc[:n].cpu().numpy().view(np.uint32)
    # records come out in increasing order within a segment, in no fixed
    # order across segments (include/ramcrc.h): compare by (segment, offset)
    order = np.lexsort((table[:, 1], table[:, 0]))
    return st.cpu().numpy().view(np.uint32).copy(), n, table[order], crc[order]


def test_fused_equals_split_small_values(ramcrc):
    from ramcloud_amd import segments
    nseg, vlen = 16, 64
    ctx = ramcrc.Context(0)
    ctx.set_option(ramcrc.OPT_VERIFY_IN_WALK, 0)   # the binned verify's direct tiny path
    try:
        d, certs, per, ck = _batch(ramcrc, ctx, nseg, vlen)
        eb = segments.entry_bytes(vlen)
        # segment 2: one byte of object 1000's value flipped (its checksum fails)
        d[2 * SEG + 1000 * eb + eb - 3] ^= 0x40
        # segment 5: a wrong certificate (the segment fails, its records are inactive)
        certs[5, 1] ^= 0x100
        cap = nseg * per + 1024
        fs, fn, ft, fc = _run(ramcrc, ctx, d, certs, nseg, cap, fused=True)
        # the shortcut was taken: the count pass put every record in bin 1
        # (the binned path would have counted segment 5's records as inactive)
        _, _, hist, par_next = ctx.debug_bins()
        assert int(hist[par_next ^ 1][1]) == fn
        ss, sn, st, sc = _run(ramcrc, ctx, d, certs, nseg, cap, fused=False)
        assert fn == sn == nseg * per
        assert np.array_equal(fs, ss)
        assert np.array_equal(ft, st)
        assert np.array_equal(fc, sc)
        ok = np.ones(nseg, bool)
        ok[5] = False
        assert (fs[ok, 0] == segments.SEG_OK).all()
        assert fs[5, 0] & segments.SEG_BAD_CHECKSUM and not fs[5, 0] & segments.SEG_OK
        assert (fs[:, 2] == per).all()
        bad = np.zeros(nseg, np.uint32)
        bad[2] = 1
        assert np.array_equal(fs[:, 3], bad)
    finally:
        ctx.close()


def test_fused_equals_split_mixed_values(ramcrc):
    """1 KiB values: records span several windows, so the fused call bins."""
    from ramcloud_amd import segments
    nseg, vlen = 8, 1024
    ctx = ramcrc.Context(0)
    try:
        d, certs, per, ck = _batch(ramcrc, ctx, nseg, vlen, first_seed=0x77)
        eb = segments.entry_bytes(vlen)
        d[3 * SEG + 17 * eb + 100] ^= 1
        cap = nseg * per + 1024
        fs, fn, ft, fc = _run(ramcrc, ctx, d, certs, nseg, cap, fused=True)
        ss, sn, st, sc = _run(ramcrc, ctx, d, certs, nseg, cap, fused=False)
        assert fn == sn == nseg * per
        assert np.array_equal(fs, ss) and np.array_equal(ft, st) and np.array_equal(fc, sc)
        assert (fs[:, 0] == segments.SEG_OK).all()
        assert list(fs[:, 3]) == [0, 0, 0, 1, 0, 0, 0, 0]
    finally:
        ctx.close()


@pytest.mark.parametrize("vlen", [128, 256])
def test_fused_multi_window_direct(ramcrc, vlen):
    """128 B and 256 B values: every object spans two (three) windows, so the
    fused call's summary sends the batch to the direct multi-window path --
    the count pass puts every record in bin 2 without reading the table and
    nothing is scattered -- with one damaged object and one damaged
    certificate; identical to the split calls (which bin the records)."""
    from ramcloud_amd import segments
    nseg = 12
    ctx = ramcrc.Context(0)
    ctx.set_option(ramcrc.OPT_VERIFY_IN_WALK, 0)   # the binned verify's direct multi-window path
    try:
        d, certs, per, ck = _batch(ramcrc, ctx, nseg, vlen, first_seed=0x1281 + vlen)
        eb = segments.entry_bytes(vlen)
        d[4 * SEG + 333 * eb + eb - 5] ^= 0x08
        certs[7, 1] ^= 0x200
        cap = nseg * per + 1024
        fs, fn, ft, fc = _run(ramcrc, ctx, d, certs, nseg, cap, fused=True)
        _, _, hist, par_next = ctx.debug_bins()
        assert int(hist[par_next ^ 1][2]) == fn   # the shortcut: all records in bin 2
        ss, sn, st, sc = _run(ramcrc, ctx, d, certs, nseg, cap, fused=False)
        assert fn == sn == nseg * per
        assert np.array_equal(fs, ss)
        assert np.array_equal(ft, st)
        assert np.array_equal(fc, sc)
        bad = np.zeros(nseg, np.uint32)
        bad[4] = 1
        assert np.array_equal(fs[:, 3], bad)
        assert fs[7, 0] & segments.SEG_BAD_CHECKSUM and not fs[7, 0] & segments.SEG_OK
    finally:
        ctx.close()


@pytest.mark.parametrize("viw", [0, 1])
def test_fused_mixed_two_and_three_window_values(ramcrc, viw):
    """One batch of 128 B-value segments (two-window objects) and 256 B-value
    segments (three windows): the summary must send it to the general
    multi-window loop, not the two-window ring, which reads only two windows
    (the in-place check refuses k > kK).  With and without verify-in-walk:
    identical to the split calls, one damaged object in each half."""
    from ramcloud_amd import segments
    half = 6
    nseg = 2 * half
    ctx = ramcrc.Context(0)
    ctx.set_option(ramcrc.OPT_VERIFY_IN_WALK, viw)
    try:
        d = torch.empty(nseg * SEG, dtype=torch.uint8, device="cuda")
        certs = torch.zeros((nseg, 2), dtype=torch.int32, device="cuda")
        lo, hi = d[:half * SEG], d[half * SEG:]
        from ramcloud_amd import workloads
        workloads.splitmix_fill_segments(d, SEG, 0x2563)
        p128, _, _ = ctx.fill_objects(lo, SEG, SEG, half, 128, first_key=0, certs=certs[:half])
        p256, _, _ = ctx.fill_objects(hi, SEG, SEG, half, 256, first_key=0, certs=certs[half:])
        torch.cuda.synchronize()
        e128, e256 = segments.entry_bytes(128), segments.entry_bytes(256)
        d[1 * SEG + 77 * e128 + e128 - 5] ^= 0x10   # value bytes (as above)
        d[(half + 2) * SEG + 91 * e256 + e256 - 5] ^= 0x01
        cap = half * (p128 + p256) + 1024
        fs, fn, ft, fc = _run(ramcrc, ctx, d, certs, nseg, cap, fused=True)
        ss, sn, st, sc = _run(ramcrc, ctx, d, certs, nseg, cap, fused=False)
        assert fn == sn == half * (p128 + p256)
        assert np.array_equal(fs, ss) and np.array_equal(ft, st) and np.array_equal(fc, sc)
        assert (fs[:, 0] == segments.SEG_OK).all()
        bad = np.zeros(nseg, np.uint32)
        bad[1] = bad[half + 2] = 1
        assert np.array_equal(fs[:, 3], bad)
    finally:
        ctx.close()


def _hist_empty(ctx, n):
    """The verify-in-walk mode was taken: the binned verify's count pass
    exited with an empty histogram although the table holds n records."""
    _, _, hist, par_next = ctx.debug_bins()
    return n > 0 and int(hist[par_next ^ 1].sum()) == 0


@pytest.mark.parametrize("vlen", [64, 100, 128])
def test_verify_in_walk_small_values(ramcrc, vlen):
    """Verify in the walk (RAMCRC_OPT_VERIFY_IN_WALK, the default for small
    entries): k_walk_copyv checks every object from LDS while it copies the
    records, and the binned scan has nothing left.  RecoverSegmentBenchmark
    segments with a damaged object value, a damaged stored checksum and a
    damaged certificate; status words, record table and object CRCs equal to
    the split calls' (which bin and scan)."""
    from ramcloud_amd import segments
    nseg = 12
    ctx = ramcrc.Context(0)
    try:
        d, certs, per, ck = _batch(ramcrc, ctx, nseg, vlen, first_seed=0xF00D + vlen)
        eb = segments.entry_bytes(vlen)
        d[1 * SEG + 77 * eb + eb - 2] ^= 0x10           # a value byte
        d[6 * SEG + 5000 * eb + 2 + 1] ^= 0x01          # the stored checksum (payload byte 1)
        certs[9, 1] ^= 0x4000                           # the whole segment fails
        cap = nseg * per + 1024
        fs, fn, ft, fc = _run(ramcrc, ctx, d, certs, nseg, cap, fused=True)
        assert _hist_empty(ctx, fn)
        ss, sn, st, sc = _run(ramcrc, ctx, d, certs, nseg, cap, fused=False)
        assert fn == sn == nseg * per
        assert np.array_equal(fs, ss)
        assert np.array_equal(ft, st)
        assert np.array_equal(fc, sc)
        bad = np.zeros(nseg, np.uint32)
        bad[1] = bad[6] = 1
        assert np.array_equal(fs[:, 3], bad)
        assert fs[9, 0] & segments.SEG_BAD_CHECKSUM and not fs[9, 0] & segments.SEG_OK
    finally:
        ctx.close()


@pytest.mark.parametrize("seed", [4242, 17])
def test_verify_in_walk_forced_mixed(ramcrc, oracle_mod, seed):
    """The verify-in-walk mode forced (2) on segments of every entry kind
    (objects of 24 B .. 200 KiB, tombstones, safe versions; junk headers in
    the payloads, so parts are misguessed and records are written by the
    fix-up's re-walks): objects too long for the stage or the leftover list
    send the whole table to the binned verify (kHardFull), the other types go
    to k_left.  One damaged entry.  Equal to the split calls and to the
    oracle."""
    import segment_cases
    cap, nseg = 1 << 20, 8
    buf, certs, counts = segment_cases.mixed_segments(oracle_mod, nseg, cap, seed=seed)
    buf[3 * cap + cap // 2] ^= 0x20
    d = torch.from_numpy(buf).cuda()
    dc = torch.from_numpy(certs.view(np.int32)).cuda()
    exp_status, exp_table, exp_crc = segment_cases.oracle_walk(oracle_mod, buf, certs, nseg, cap=cap)
    from ramcloud_amd import segments
    got = {}
    for mode in (2, 0):
        ctx = ramcrc.Context(0)
        try:
            ctx.set_option(ramcrc.OPT_VERIFY_IN_WALK, mode)
            rv = segments.RecoveryVerify(ctx, nseg, cap, entries_cap=int(counts.sum()) + 4096)
            st = rv.verify(d, dc, check=True)
            torch.cuda.synchronize()
            n = int(rv.n_entries.item())
            table = rv.entries[:n].cpu().numpy().view(np.uint32)
            crc = rv.obj_crc[:n].cpu().numpy().view(np.uint32)
            o = np.lexsort((table[:, 1], table[:, 0]))
            got[mode] = (st.cpu().numpy().view(np.uint32).copy(), table[o], crc[o])
        finally:
            ctx.close()
    for k in range(3):
        assert np.array_equal(got[2][k], got[0][k]), k
    assert np.array_equal(got[2][0], exp_status)
    assert np.array_equal(got[2][1], exp_table)
    mask = segment_cases.replay_crc_mask(buf, cap, exp_table)
    assert np.array_equal(got[2][2][mask], exp_crc[mask])


def test_verify_in_walk_replay_mix(ramcrc, oracle_mod, golden):
    """The replay mix (objects, tombstones, safe versions, prepared ops and
    their tombstones, decision records, participant lists; valid and damaged)
    with the verify-in-walk mode forced: the other types go through k_left.
    Equal to the split calls."""
    import segment_cases
    buf, certs, bad_exp, _ = segment_cases.build_replay_mix(oracle_mod, golden)
    nseg, cap = certs.shape[0], segment_cases.CAPACITY
    d = torch.from_numpy(buf).cuda()
    dc = torch.from_numpy(np.ascontiguousarray(certs).view(np.int32)).cuda()
    from ramcloud_amd import segments
    got = {}
    for mode in (2, 0):
        ctx = ramcrc.Context(0)
        try:
            ctx.set_option(ramcrc.OPT_VERIFY_IN_WALK, mode)
            rv = segments.RecoveryVerify(ctx, nseg, cap, entries_cap=nseg * (cap // 14 + 1))
            st = rv.verify(d, dc, check=True)
            torch.cuda.synchronize()
            n = int(rv.n_entries.item())
            table = rv.entries[:n].cpu().numpy().view(np.uint32)
            crc = rv.obj_crc[:n].cpu().numpy().view(np.uint32)
            o = np.lexsort((table[:, 1], table[:, 0]))
            got[mode] = (st.cpu().numpy().view(np.uint32).copy(), table[o], crc[o])
        finally:
            ctx.close()
    for k in range(3):
        assert np.array_equal(got[2][k], got[0][k]), k
    assert np.array_equal(got[2][0][:, 3], bad_exp) and int(bad_exp.sum()) > 0


@pytest.mark.parametrize("vlen", [2048, 3072])
def test_repeated_calls_pool_blocks(ramcrc, oracle_mod, vlen):
    """The same batch verified four times on one context, as a replay thread
    does batch after batch: 2 and 3 KiB values walk in 256 KiB parts of 83 ..
    125 entries, so parts keep records in pool blocks and the fix-up re-walks
    some of them.  Every call's records and object CRCs equal the first call's
    and, for the first segments, the oracle's walk (round 6: a block map kept
    from the previous call replaced one part's pool block by another's)."""
    from ramcloud_amd import segments
    nseg, check = 256, 6
    ctx = ramcrc.Context(0)
    try:
        d, certs, per, ck = _batch(ramcrc, ctx, nseg, vlen, first_seed=0x3C3C + vlen)
        host = d[:check * SEG].cpu().numpy()
        cn = certs.cpu().numpy().view(np.uint32)
        want = np.concatenate([oracle_mod.check_metadata(host[s * SEG:(s + 1) * SEG], int(cn[s, 0]),
                                                         int(cn[s, 1]), segment=s, capacity=SEG)[3]
                               for s in range(check)])
        rv = segments.RecoveryVerify(ctx, nseg, SEG, entries_cap=nseg * per + nseg)
        first = None
        for call in range(4):
            st = rv.verify(d, certs, check=True)
            torch.cuda.synchronize()
            n = int(rv.n_entries.item())
            t = rv.entries[:n].cpu().numpy().view(np.uint32).reshape(-1, 4)
            c = rv.obj_crc[:n].cpu().numpy().view(np.uint32)
            o = np.lexsort((t[:, 1], t[:, 0]))
            t, c = t[o], c[o]
            s = st.cpu().numpy().view(np.uint32)
            assert (s[:, 0] == segments.SEG_OK).all() and (s[:, 3] == 0).all(), call
            assert n == nseg * per, call
            assert np.array_equal(t[t[:, 0] < check], want), call
            if first is None:
                first = (t, c)
            else:
                assert np.array_equal(t, first[0]) and np.array_equal(c, first[1]), call
    finally:
        ctx.close()
