"""Parity of the MI355X kernels (through the C ABI) with the oracle and the
reference's known answers.  Bit-exact: CRC is integer arithmetic.

Cases follow the reference's tests (src/Crc32CTest.cc prefixes/chaining, the
Segment/Object goldens) plus what a batch path adds: empty and 1-3 byte
buffers, unaligned starts and ends, lengths around the 64 KiB small/large
threshold and the 256 KiB chunk and 1 KiB block boundaries, caller-supplied
initial states (chaining), raw vs finalized output, and the full 1024 x 8 MiB
headline batch.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

MiB = 1 << 20


@pytest.fixture(scope="module")
def ctx(ramcrc):
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    c = ramcrc.Context(0)
    yield c
    c.close()


def dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def u32(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


def i32_from_u32(a):
    return dev(np.asarray(a, dtype=np.uint32).view(np.int32))


def oracle_entries(oracle_mod, base, off, length, init, finalize):
    return oracle_mod.entries(base, off, length, init=init, finalize=finalize)


def run_api(ctx, api, base_t, off, length, init, finalize):
    n = len(off)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    off_t = dev(np.asarray(off, dtype=np.uint64).view(np.int64))
    len_t = dev(np.asarray(length, dtype=np.uint64).view(np.int64))
    init_t = None if init is None else i32_from_u32(init)
    getattr(ctx, api)(base_t, off_t, len_t, out, init=init_t, finalize=finalize)
    return u32(out)


@pytest.mark.parametrize("api", ["entries", "batch"])
def test_reference_random_cases(ctx, golden, golden_base, api):
    cases = golden["random"]["cases"]
    off = [c[0] for c in cases]
    length = [c[1] for c in cases]
    init = [c[2] for c in cases]
    want = np.array([c[3] for c in cases], dtype=np.uint32)
    got = run_api(ctx, api, dev(golden_base), off, length, init, finalize=False)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(cases[i], hex(got[i])) for i in bad[:5]]


@pytest.mark.parametrize("api", ["entries", "batch"])
def test_crc32c_test_prefixes(ctx, golden, api):
    inp = np.array(golden["crc32c_test"]["input"], dtype=np.uint8)
    want = np.array(golden["crc32c_test"]["crcByLength"], dtype=np.uint32)
    n = inp.size + 1
    got = run_api(ctx, api, dev(inp), [0] * n, list(range(n)), None, finalize=True)
    assert np.array_equal(got, want)


def test_crc32c_test_accumulated_chain(ctx, golden):
    """Byte-at-a-time chaining through raw states (src/Crc32CTest.cc:77-82):
    each launch continues from the previous launch's raw output."""
    inp = np.array(golden["crc32c_test"]["input"], dtype=np.uint8)
    want = golden["crc32c_test"]["crcByLength"]
    base = dev(inp)
    state = 0xFFFFFFFF
    for i in range(inp.size):
        got = run_api(ctx, "batch", base, [i], [1], [state], finalize=False)
        state = int(got[0])
        assert (~state) & 0xFFFFFFFF == want[i + 1]


def test_segment_and_object_goldens(ctx, golden):
    items = [bytes.fromhex(c.get("stream", c.get("bytes")))
             for c in golden["segment_certificates"] + golden["object_checksums"] + golden["tombstone_checksums"]]
    want = [c["checksum"] for c in golden["segment_certificates"] + golden["object_checksums"] + golden["tombstone_checksums"]]
    blob = b"".join(items)
    off = np.cumsum([0] + [len(x) for x in items[:-1]])
    got = run_api(ctx, "batch", dev(np.frombuffer(blob, np.uint8)), off, [len(x) for x in items],
                  None, finalize=True)
    assert list(got) == want


def _bench_segments(nseg, seg_bytes=8 * MiB, extra=0):
    from ramcloud_amd import workloads
    t = torch.empty(nseg * seg_bytes + extra, dtype=torch.uint8, device="cuda")
    workloads.splitmix_fill_segments(t[:nseg * seg_bytes], seg_bytes, workloads.SEGMENT_SEED)
    return t


def test_segments_aligned_kats(ctx, golden, oracle_mod):
    nseg = 8
    data = _bench_segments(nseg)
    out = torch.zeros(nseg, dtype=torch.int32, device="cuda")
    ctx.segments(data, 8 * MiB, nseg, out)
    got = u32(out)
    kats = {k["name"]: k["crc"] for k in golden["kat"] if "crc" in k}
    for i in range(4):
        assert got[i] == kats[f"bench_segment_{i}"], i
    host = data.cpu().numpy()
    assert np.array_equal(got, oracle_mod.segments(host, 8 * MiB, nseg, threads=8))


def test_segments_init_and_raw(ctx, oracle_mod):
    nseg = 5
    data = _bench_segments(nseg)
    rng = np.random.default_rng(1)
    init = rng.integers(0, 2 ** 32, nseg, dtype=np.uint64).astype(np.uint32)
    out = torch.zeros(nseg, dtype=torch.int32, device="cuda")
    ctx.segments(data, 8 * MiB, nseg, out, init=i32_from_u32(init), finalize=False)
    host = data.cpu().numpy()
    off = np.arange(nseg, dtype=np.uint64) * 8 * MiB
    want = oracle_mod.entries(host, off, np.full(nseg, 8 * MiB, np.uint64), init=init,
                              finalize=False)
    assert np.array_equal(u32(out), want)


@pytest.mark.parametrize("shift,seg_bytes", [
    (0, 256 * 1024), (0, 512 * 1024 + 1024), (1, 8 * MiB), (13, 300001), (5, 65536),
    (3, 65535), (7, 4), (2, 3), (0, 1), (11, 262144 * 3 - 1), (0, 1024 * 1024 + 17)])
def test_segments_unaligned_and_odd_sizes(ctx, oracle_mod, shift, seg_bytes):
    nseg = max(2, min(9, (24 * MiB) // max(seg_bytes, 1)))
    total = shift + nseg * seg_bytes
    host = oracle_mod.splitmix_bytes(shift * 1000 + seg_bytes, total)
    base = dev(host)
    out = torch.zeros(nseg, dtype=torch.int32, device="cuda")
    ctx.segments(base[shift:], seg_bytes, nseg, out)
    off = shift + np.arange(nseg, dtype=np.uint64) * seg_bytes
    want = oracle_mod.entries(host, off, np.full(nseg, seg_bytes, np.uint64))
    assert np.array_equal(u32(out), want)


def test_batch_mixed_lengths_and_overlaps(ctx, oracle_mod):
    rng = np.random.default_rng(2024)
    total = 24 * MiB
    host = oracle_mod.splitmix_bytes(77, total)
    special = [0, 1, 2, 3, 4, 5, 15, 16, 17, 1023, 1024, 1025, 65535, 65536, 65537,
               262143, 262144, 262145, 524288 + 3, 1 << 20, 3 * MiB + 5]
    lens = special + [int(x) for x in rng.integers(0, 200000, 300)] + \
        [int(x) for x in rng.integers(0, 4 * MiB, 20)]
    offs = [int(rng.integers(0, total - L + 1)) for L in lens]
    init = rng.integers(0, 2 ** 32, len(lens), dtype=np.uint64).astype(np.uint32)
    base = dev(host)
    for finalize in (True, False):
        got = run_api(ctx, "batch", base, offs, lens, init, finalize)
        want = oracle_mod.entries(host, offs, lens, init=init, finalize=finalize)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, [(offs[i], lens[i]) for i in bad[:5]]
    # default init
    got = run_api(ctx, "batch", base, offs, lens, None, True)
    assert np.array_equal(got, oracle_mod.entries(host, offs, lens))


@pytest.mark.parametrize("api", ["entries", "batch"])
def test_entries_every_alignment(ctx, oracle_mod, api):
    """Every start offset within a 128-byte line x every length up to three
    windows (plus a few longer): the small-entry kernels' window geometry
    (one window, entry ending exactly at a window end, init bytes crossing a
    line) is exercised at each alignment."""
    host = oracle_mod.splitmix_bytes(4242, 1 << 20)
    lens = list(range(0, 400)) + [511, 512, 513, 1023, 1024, 1025, 4095, 4096, 4097]
    offs, ls = [], []
    for s in range(128):
        for L in lens:
            offs.append(1024 + s + 128 * ((s * 7 + L) % 64))
            ls.append(L)
    rng = np.random.default_rng(77)
    init = rng.integers(0, 2 ** 32, len(offs), dtype=np.uint64).astype(np.uint32)
    base = dev(host)
    for it in (None, init):
        got = run_api(ctx, api, base, offs, ls, it, True)
        want = oracle_mod.entries(host, offs, ls, init=it)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, [(offs[i] % 128, ls[i]) for i in bad[:8]]


def test_entries_config3_sample(ctx, oracle_mod):
    from ramcloud_amd import workloads
    lens = workloads.entry_lengths(60000)
    offs = workloads.packed_offsets(lens)
    host = workloads.splitmix_bytes_np(workloads.ENTRY_SEED, int(lens.sum()))
    base = dev(host)
    for api in ("entries", "batch"):
        got = run_api(ctx, api, base, offs, lens, None, True)
        assert np.array_equal(got, oracle_mod.entries(host, offs, lens)), api


def test_empty_batches(ctx):
    out = torch.zeros(1, dtype=torch.int32, device="cuda")
    base = torch.zeros(16, dtype=torch.uint8, device="cuda")
    e = torch.zeros(0, dtype=torch.int64, device="cuda")
    ctx.batch(base, e, e, out)
    ctx.entries(base, e, e, out)
    ctx.segments(base, 8, 0, out)
    assert u32(out)[0] == 0


def test_batch_host_and_stream_host(ctx, oracle_mod):
    rng = np.random.default_rng(5)
    bufs = [oracle_mod.splitmix_bytes(i, int(rng.integers(0, 300000))) for i in range(40)]
    bufs += [b"", b"a", b"ab", b"abc"]
    got = ctx.batch_host(bufs)
    assert list(got) == [oracle_mod.crc32c(b) for b in bufs]
    seg = 1 * MiB
    nseg = 37
    host = oracle_mod.splitmix_bytes(9, seg * nseg)
    got = ctx.stream_host(host, seg, nseg, batch=4, depth=3)
    assert np.array_equal(got, oracle_mod.segments(host, seg, nseg, threads=8))


def test_full_headline_batch(ctx, oracle_mod):
    """BASELINE config 2 at full size: 1024 x 8 MiB, every CRC checked against
    the oracle (8 GiB copied back to the host), and the batch-API (planned)
    path agrees with the aligned recovery-scan path on the same bytes."""
    nseg = 1024
    data = _bench_segments(nseg)
    out = torch.zeros(nseg, dtype=torch.int32, device="cuda")
    ctx.segments(data, 8 * MiB, nseg, out)
    got = u32(out)
    off = torch.arange(nseg, dtype=torch.int64, device="cuda") * (8 * MiB)
    ln = torch.full((nseg,), 8 * MiB, dtype=torch.int64, device="cuda")
    out2 = torch.zeros(nseg, dtype=torch.int32, device="cuda")
    ctx.batch(data, off, ln, out2)
    assert np.array_equal(got, u32(out2))
    host = data.cpu().numpy()
    del data
    want = oracle_mod.segments(host, 8 * MiB, nseg, threads=16)
    assert np.array_equal(got, want)


def test_entries_config3_full(ctx, oracle_mod):
    """BASELINE config 3 at its stated size: the 1,000,000-entry Zipf table
    (100 B / 1 KiB / 4 KiB, packed unaligned), every CRC against the oracle,
    through the small-entry path and the general batch path; plus the
    per-object (off + 4, len - 4) variant replay uses."""
    from ramcloud_amd import workloads
    lens = workloads.entry_lengths(1_000_000)
    offs = workloads.packed_offsets(lens)
    host = workloads.splitmix_bytes_np(workloads.ENTRY_SEED, int(lens.sum()))
    base = dev(host)
    want = oracle_mod.entries(host, offs, lens)
    for api in ("entries", "batch"):
        assert np.array_equal(run_api(ctx, api, base, offs, lens, None, True), want), api
    want4 = oracle_mod.entries(host, offs + 4, lens - 4)
    assert np.array_equal(run_api(ctx, "entries", base, offs + 4, lens - 4, None, True), want4)
    ctx.check()


def test_stream_host_config5_8mib(ctx, oracle_mod):
    """BASELINE config 5 shape: 64 pinned 8 MiB host segments streamed through
    the GPU (H2D on the copy stream overlapped with the kernels), CRCs back
    in host memory, against the oracle; also a ragged last batch."""
    seg, nseg = 8 * MiB, 64
    host = torch.empty(nseg * seg, dtype=torch.uint8).pin_memory()
    host.numpy()[:] = oracle_mod.splitmix_bytes(21, seg * nseg)
    want = oracle_mod.segments(host.numpy(), seg, nseg, threads=16)
    got = ctx.stream_host(host, seg, nseg, batch=8, depth=3)
    assert np.array_equal(got, want)
    got = ctx.stream_host(host, seg, 61, batch=8, depth=2)
    assert np.array_equal(got, want[:61])


def test_unknown_flag_bits_refused(ctx, ramcrc):
    """Flag bits other than RAMCRC_FINALIZE are EINVAL (2 was round 4's
    RAMCRC_ORDERED, removed; include/ramcrc.h RAMCRC_ABI_VERSION)."""
    import ctypes
    L = ramcrc.lib()
    data = torch.zeros(1024, dtype=torch.uint8, device="cuda")
    off = dev(np.array([0, 100], dtype=np.int64))
    ln = dev(np.array([100, 200], dtype=np.int64))
    out = torch.zeros(2, dtype=torch.int32, device="cuda")
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    for fl in (2, 4, 0x80000000):
        assert L.ramcrc_batch_device(ctx._h, p(data), p(off), p(ln), None, p(out), 2, fl, None) == -1
        assert L.ramcrc_entries_device(ctx._h, p(data), p(off), p(ln), None, p(out), 2, fl, None) == -1
        assert L.ramcrc_segments_device(ctx._h, p(data), 512, 2, None, p(out), fl, None) == -1
    assert L.ramcrc_batch_device(ctx._h, p(data), p(off), p(ln), None, p(out), 2, 1, None) == 0
    torch.cuda.synchronize()
