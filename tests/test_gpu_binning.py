"""The small-entry binning sequence (k_bin_count -> k_bin_scatter -> k_entries,
or k_bin_one -> k_entries for batches of at most one tile per resident
workgroup) across failed and corrupted launches.

Round 2 recorded a GPU hang in k_entries whose cause was a bin layout that
disagreed with the slots the scatter had written (stale slots, an octet of
padding only: the interior loop bound Kmin - 1 then wrapped to 2^32).  The
counters are now per-sequence copies (BinCounters), flipped only once
k_bin_count is enqueued, and k_entries refuses a launch whose layout does not
match what was scattered.  These tests drive exactly those paths through the
C ABI's test hooks (RAMCRC_OPT_TEST_FAIL_AFTER_COUNT, RAMCRC_OPT_TEST_DIRTY_BINS)
and check every later call bit-exact against the oracle.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def run(ctx, api, base, offs, lens, init=None, out=None):
    n = len(offs)
    if out is None:
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
    off_t = dev(np.asarray(offs, dtype=np.uint64).view(np.int64))
    len_t = dev(np.asarray(lens, dtype=np.uint64).view(np.int64))
    init_t = None if init is None else dev(np.asarray(init, dtype=np.uint32).view(np.int32))
    getattr(ctx, api)(base, off_t, len_t, out, init=init_t)
    return out


def host_u32(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


def alignment_case(oracle_mod, seed=4242, with_long=True):
    host = oracle_mod.splitmix_bytes(seed, 1 << 20)
    lens = list(range(0, 300, 3)) + ([1023, 1024, 1025, 4095, 4096, 9000] if with_long else [])
    offs, ls = [], []
    for s in range(0, 128, 5):
        for L in lens:
            offs.append(1024 + s + 128 * ((s * 7 + L) % 64))
            ls.append(L)
    rng = np.random.default_rng(seed)
    init = rng.integers(0, 2 ** 32, len(offs), dtype=np.uint64).astype(np.uint32)
    return host, offs, ls, init


@pytest.fixture()
def ctx(ramcrc):
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    c = ramcrc.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("api", ["entries", "batch"])
@pytest.mark.parametrize("fails", [1, 2, 3])
def test_failed_sequence_then_init_call(ctx, ramcrc, oracle_mod, api, fails):
    """A sequence abandoned right after its histogram pass (the early return
    of a failed later launch) must not leak into the next calls -- the
    round-2 hang was the first call with an initial-state array after such a
    hand-off."""
    host, offs, ls, init = alignment_case(oracle_mod)
    base = dev(host)
    ctx.set_option(ramcrc.OPT_TEST_FAIL_AFTER_COUNT, fails)
    for _ in range(fails):
        with pytest.raises(ramcrc.RamcrcError) as e:
            run(ctx, api, base, offs, ls, init)
        assert e.value.code == -3
    for it in (init, None, init):
        got = host_u32(run(ctx, api, base, offs, ls, it))
        want = oracle_mod.entries(host, offs, ls, init=it)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, [(offs[i] % 128, ls[i]) for i in bad[:8]]
    ctx.check()


@pytest.mark.parametrize("api", ["entries", "batch"])
@pytest.mark.parametrize("bin_, add", [(1, 3), (2, 1), (9, 5), (40, 7), (160, 2)])
def test_dirty_histogram_is_refused(ctx, ramcrc, oracle_mod, api, bin_, add):
    """A histogram that disagrees with the scatter (as a stale one would):
    the launch writes nothing and ramcrc_ctx_check reports RAMCRC_EINTERNAL;
    the next call is exact."""
    host, offs, ls, init = alignment_case(oracle_mod, seed=7)
    base = dev(host)
    sentinel = torch.full((len(offs),), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    ctx.set_option(ramcrc.OPT_TEST_DIRTY_BINS, (bin_ << 16) | add)
    run(ctx, api, base, offs, ls, init, out=sentinel)
    with pytest.raises(ramcrc.RamcrcError) as e:
        ctx.check()
    assert e.value.code == ramcrc.EINTERNAL
    got = host_u32(sentinel)
    # small entries are not written (large ones on the batch path are k_chunks')
    small = np.array([L < 65536 for L in ls])
    assert np.all(got[small] == 0x5A5A5A5A)
    ctx.check()   # the sticky bits were taken
    got = host_u32(run(ctx, api, base, offs, ls, init))
    assert np.array_equal(got, oracle_mod.entries(host, offs, ls, init=init))
    ctx.check()


def test_histogram_past_capacity_is_refused(ramcrc, oracle_mod):
    """A histogram asking for more sorted slots than the context holds: the
    scatter writes nothing (no out-of-bounds slot), the launch is refused."""
    c = ramcrc.Context(0)
    try:
        host = oracle_mod.splitmix_bytes(3, 1 << 16)
        offs = [17 * i for i in range(200)]
        ls = [100] * 200
        base = dev(host)
        sentinel = torch.full((200,), 0x1234, dtype=torch.int32, device="cuda")
        c.set_option(ramcrc.OPT_TEST_DIRTY_BINS, (1 << 16) | 0xFFFF)
        run(c, "entries", base, offs, ls, out=sentinel)
        with pytest.raises(ramcrc.RamcrcError) as e:
            c.check()
        assert e.value.code == ramcrc.EINTERNAL
        assert np.all(host_u32(sentinel) == 0x1234)
        got = host_u32(run(c, "entries", base, offs, ls))
        assert np.array_equal(got, oracle_mod.entries(host, offs, ls))
    finally:
        c.close()


def test_plan_skip_alternating(ctx, oracle_mod):
    """The batch path skips its chunk kernels when the count pass finds no
    buffer of >= 64 KiB: alternate batches with and without large buffers (and
    with and without initial states) on one context."""
    rng = np.random.default_rng(99)
    total = 8 << 20
    host = oracle_mod.splitmix_bytes(11, total)
    base = dev(host)
    for k in range(6):
        big = k % 2 == 1
        lens = [int(x) for x in rng.integers(0, 5000, 2000)]
        if big:
            lens += [65536, 65537, 300000, 1 << 20]
        offs = [int(rng.integers(0, total - L + 1)) for L in lens]
        init = None if k % 3 == 0 else rng.integers(0, 2 ** 32, len(lens),
                                                   dtype=np.uint64).astype(np.uint32)
        got = host_u32(run(ctx, "batch", base, offs, lens, init))
        want = oracle_mod.entries(host, offs, lens, init=init)
        assert np.array_equal(got, want), k
    ctx.check()


@pytest.mark.parametrize("api", ["entries", "batch"])
def test_all_tiny_batch_direct_path(ctx, ramcrc, oracle_mod, api):
    """A batch whose every entry fits one 128-byte window (100-byte log
    entries, 0-3 byte ones, every alignment) takes the direct tiny path:
    nothing is scattered, the tiny phase reads the caller's table in place.
    Bit-exact with and without initial states, raw and finalized; then a mixed
    batch on the same context (the layout switches back)."""
    rng = np.random.default_rng(123)
    host = oracle_mod.splitmix_bytes(99, 1 << 20)
    base = dev(host)
    n = 70000
    lens = rng.integers(0, 113, n)
    offs = rng.integers(0, (1 << 20) - 4000, n)
    lens[:200] = np.arange(200) % 4          # bytewise entries
    offs[200:400] = 1024 + np.arange(200)    # every alignment
    lens[200:400] = 128 - (offs[200:400] % 16)   # ending exactly at the window end
    init = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    for it in (None, init):
        got = host_u32(run(ctx, api, base, offs, lens, it))
        want = oracle_mod.entries(host, offs, lens, init=it)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, [(int(offs[i]) % 16, int(lens[i])) for i in bad[:8]]
    lens2 = lens.copy()
    lens2[::97] = 3000
    got = host_u32(run(ctx, api, base, offs, lens2))
    assert np.array_equal(got, oracle_mod.entries(host, offs, lens2))
    got = host_u32(run(ctx, api, base, offs, lens))
    assert np.array_equal(got, oracle_mod.entries(host, offs, lens))
    ctx.check()


@pytest.mark.parametrize("api", ["entries", "batch"])
def test_direct_path_long_windows(ctx, ramcrc, oracle_mod, api):
    """All-tiny batches whose windows mostly end at >= 96 bytes, where the
    tiny loop skips the tail masks of dwords 0-2 (RAMCRC_TINY_T3, a ballot
    per q): entries of 81-112 bytes at every alignment, then 60-112 bytes so
    that waves mix the masked and unmasked window bodies, with and without
    initial states."""
    rng = np.random.default_rng(8196)
    host = oracle_mod.splitmix_bytes(41, 1 << 20)
    base = dev(host)
    n = 50000
    offs = rng.integers(0, (1 << 20) - 4000, n)
    for lo in (81, 60):
        lens = rng.integers(lo, 113, n)
        lens = np.minimum(lens, 128 - (offs % 16))   # one window each: E - (S & ~15) <= 128
        init = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        for it in (None, init):
            got = host_u32(run(ctx, api, base, offs, lens, it))
            want = oracle_mod.entries(host, offs, lens, init=it)
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, [(int(offs[i]) % 16, int(lens[i])) for i in bad[:8]]
    ctx.check()


@pytest.mark.parametrize("api", ["entries", "batch"])
def test_one_launch_threshold(ctx, ramcrc, oracle_mod, api):
    """Batches either side of the one-launch binning limit (one 4,096-entry
    tile per 1,024-thread workgroup, one workgroup per CU -- half of the two a
    CU holds: 1,048,576 entries on 256 CUs)
    and a few small ones: k_bin_one and the two-launch path give the same,
    exact CRCs, with and without initial states."""
    ctx.set_option(ramcrc.OPT_BIN_ONE, 1)   # (the default since round 6 is the two-launch path)
    rng = np.random.default_rng(5150)
    total = 4 << 20
    host = oracle_mod.splitmix_bytes(31, total)
    base = dev(host)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    lim = ncu * 4096
    for n in (1, 1023, 1025, lim - 1, lim, lim + 1):
        lens = rng.integers(0, 600, n)
        lens[::7] = rng.integers(600, 9000, lens[::7].size)
        offs = rng.integers(0, total - 9000, n)
        init = None if n % 2 else rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        got = host_u32(run(ctx, api, base, offs, lens, init))
        want = oracle_mod.entries(host, offs, lens, init=init)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (n, [(int(offs[i]) % 128, int(lens[i])) for i in bad[:8]])
    ctx.check()


@pytest.mark.parametrize("api", ["entries", "batch"])
def test_one_launch_binning_gives_up(ctx, ramcrc, oracle_mod, api):
    """k_bin_one's grid-wide arrival is a vote: if part of the grid never
    arrives (forced here by the straggler hook: one workgroup more than
    launched), the waiters abort after their stall period, nothing is
    scattered by k_bin_one, and the guarded scatter behind it bins the batch
    the two-launch way -- the call completes exact, with and without initial
    states, and counts one rescue."""
    host, offs, ls, init = alignment_case(oracle_mod, seed=13)
    base = dev(host)
    ctx.set_option(ramcrc.OPT_BIN_ONE, 1)
    r0 = ctx.bin_rescues()
    for it in (init, None):
        ctx.set_option(ramcrc.OPT_TEST_BIN_STRAGGLER, 1)
        got = host_u32(run(ctx, api, base, offs, ls, it))
        ctx.check()
        bad = np.nonzero(got != oracle_mod.entries(host, offs, ls, init=it))[0]
        assert bad.size == 0, [(offs[i] % 128, ls[i]) for i in bad[:8]]
    assert ctx.bin_rescues() == r0 + 2
    got = host_u32(run(ctx, api, base, offs, ls, init))   # and the vote goes through again
    assert np.array_equal(got, oracle_mod.entries(host, offs, ls, init=init))
    assert ctx.bin_rescues() == r0 + 2
    ctx.check()


@pytest.mark.parametrize("bin_one", [0, 1])
def test_concurrent_contexts_config3(ramcrc, oracle_mod, bin_one):
    """Four contexts on four streams, one host thread each (the deployment
    include/ramcrc.h prescribes: one context per launching thread; the
    reference replays from 1-16 threads, nanobenchmarks/RecoverSegmentBenchmark.cc:88-118),
    each submitting BASELINE config-3 batches (1M Zipf entries, the one-launch
    binning's size) back to back while the others run.  Grids of different
    contexts then compete for the CUs, so some k_bin_one votes may abort;
    every call must still complete: no RAMCRC_EINTERNAL (or any error) and
    every CRC bit-exact against the oracle."""
    import threading
    from ramcloud_amd import workloads
    lens = workloads.entry_lengths(1_000_000)
    offs = workloads.packed_offsets(lens)
    host = workloads.splitmix_bytes_np(workloads.ENTRY_SEED, int(lens.sum()))
    want = oracle_mod.entries(host, offs, lens)
    base = dev(host)
    off_t = dev(np.asarray(offs, dtype=np.uint64).view(np.int64))
    len_t = dev(np.asarray(lens, dtype=np.uint64).view(np.int64))
    nctx, iters = 4, 6
    ctxs = [ramcrc.Context(0) for _ in range(nctx)]
    for c in ctxs:
        c.set_option(ramcrc.OPT_BIN_ONE, bin_one)
    streams = [torch.cuda.Stream() for _ in range(nctx)]
    outs = [[torch.zeros(len(lens), dtype=torch.int32, device="cuda") for _ in range(iters)]
            for _ in range(nctx)]
    torch.cuda.synchronize()
    errors = []
    start = threading.Barrier(nctx)

    def worker(k):
        try:
            start.wait()
            for i in range(iters):
                api = ctxs[k].entries if (i + k) % 2 == 0 else ctxs[k].batch
                api(base, off_t, len_t, outs[k][i], stream=streams[k])
            ctxs[k].check(streams[k])
        except Exception as e:   # noqa: BLE001 -- reported below
            errors.append((k, repr(e)))

    try:
        th = [threading.Thread(target=worker, args=(k,)) for k in range(nctx)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in th), "a worker did not finish"
        assert not errors, errors
        torch.cuda.synchronize()
        for k in range(nctx):
            for i in range(iters):
                got = outs[k][i].cpu().numpy().view(np.uint32)
                bad = np.nonzero(got != want)[0]
                assert bad.size == 0, (k, i, bad.size, bad[:8])
        rescues = [c.bin_rescues() for c in ctxs]
        print(f"k_bin_one rescues per context: {rescues} of {iters} batches each")
    finally:
        for c in ctxs:
            c.close()


def test_long_phase_sparse_batches(ctx, oracle_mod):
    """Batches of a few long entries (0.5-60 KiB) among tiny ones: the long
    phase's static age-weighted shares (k_entries) then give
    most workgroups and waves an empty or partial range, and the role split
    sends most workgroups to the tiny phase.  Every CRC must be exact, with
    and without initial states, over many batches on one context.  (Written
    for round 5's work-stealing deques, whose failing steal once claimed
    octets past the table; the static shares that replaced them keep the
    same edge cases.)"""
    rng = np.random.default_rng(77)
    total = 8 << 20
    host = oracle_mod.splitmix_bytes(5, total)
    base = dev(host)
    for k in range(24):
        n = int(rng.integers(1, 300))
        lens = rng.integers(0, 120, n)
        nlong = int(rng.integers(1, 12))
        lens[rng.integers(0, n, nlong)] = rng.integers(500, 60000, nlong)
        offs = rng.integers(0, total - 60000, n)
        init = None if k % 2 else rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        for api in ("entries", "batch"):
            got = host_u32(run(ctx, api, base, offs, lens, init))
            want = oracle_mod.entries(host, offs, lens, init=init)
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (k, api, [(int(offs[i]) % 128, int(lens[i])) for i in bad[:8]])
    ctx.check()


@pytest.mark.parametrize("api", ["entries", "batch"])
def test_two_window_table_direct_path(ctx, ramcrc, oracle_mod, api):
    """Table batches whose every entry spans exactly two 128-byte windows
    (1M x 160 B log entries; here 129 .. 256-byte spans at every start
    alignment) take the direct multi-window path: nothing is scattered and the
    two-window ring reads the caller's (off, len, init) in place.  Exact with
    and without initial states, raw and finalized, on both binning launches;
    then a batch with one three-window entry (the layout switches back) and
    the two-window batch again."""
    rng = np.random.default_rng(2626)
    total = 2 << 20
    host = oracle_mod.splitmix_bytes(262, total)
    base = dev(host)
    n = 60000
    offs = rng.integers(0, total - 512, n)
    lens = rng.integers(100, 257, n)
    a = offs & 15
    keep = (a + lens > 128) & (a + lens <= 256)
    offs, lens = offs[keep], lens[keep]
    offs[:256] = 4096 + np.arange(256)                 # every alignment
    lens[:256] = 256 - (offs[:256] % 16)               # ending exactly at the second window's end
    lens[256:512] = 129 - (offs[256:512] % 16)         # one byte into the second window
    init = rng.integers(0, 2 ** 32, offs.size, dtype=np.uint64).astype(np.uint32)
    for one in (0, 1):
        ctx.set_option(ramcrc.OPT_BIN_ONE, one)
        for it in (None, init):
            for fin in (True, False):
                off_t = dev(np.asarray(offs, dtype=np.uint64).view(np.int64))
                len_t = dev(np.asarray(lens, dtype=np.uint64).view(np.int64))
                init_t = None if it is None else dev(np.asarray(it, dtype=np.uint32).view(np.int32))
                out = torch.zeros(offs.size, dtype=torch.int32, device="cuda")
                getattr(ctx, api)(base, off_t, len_t, out, init=init_t, finalize=fin)
                got = host_u32(out)
                want = oracle_mod.entries(host, offs, lens, init=it, finalize=fin)
                bad = np.nonzero(got != want)[0]
                assert bad.size == 0, (one, fin, [(int(offs[i]) % 16, int(lens[i])) for i in bad[:8]])
        # the shortcut was taken: the layout holds no slot
        count, _, _, _ = ctx.debug_bins()
        assert int(count.sum()) == 0
        lens3 = lens.copy()
        lens3[offs.size // 2] = 300
        got = host_u32(run(ctx, api, base, offs, lens3))
        assert np.array_equal(got, oracle_mod.entries(host, offs, lens3))
        got = host_u32(run(ctx, api, base, offs, lens, init))
        assert np.array_equal(got, oracle_mod.entries(host, offs, lens, init=init))
    ctx.check()
