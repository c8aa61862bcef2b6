"""Ordered batches (RAMCRC_ORDERED: entries in log order, checksummed as one
byte stream by k_stream_prep / k_stream / k_stream_fix) against the oracle,
bit for bit, on both APIs.

Cases: the BASELINE config-3 mix at full size and 1M x 100 B; random lengths
0 .. 5000 with and without gaps (up to 4095 bytes) at every start alignment;
empty entries (alone, in runs, at step and span boundaries); entries that
start or end exactly on 128-byte steps; spans of more than 64 entries (the
entry window refill); entries crossing one or many spans (k_stream_fix);
raw (unfinalized) output; and batches that break the order (overlap, out of
order, a 4 KiB gap), which are refused with RAMCRC_EORDER and write nothing,
followed by a valid batch on the same context."""
import numpy as np
import pytest

from ramcloud_amd import workloads

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(ramcrc):
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    c = ramcrc.Context(0)
    yield c
    c.close()


def _dev64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def _run(ctx, api, base_t, off, lens, finalize=True, sentinel=0x5A5A5A5A):
    n = len(off)
    out = torch.full((n,), np.int32(np.uint32(sentinel).view(np.int32)), dtype=torch.int32,
                     device="cuda")
    getattr(ctx, api)(base_t, _dev64(off), _dev64(lens), out, finalize=finalize, ordered=True)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def _table(rng, n, lo=0, hi=5000, gap=0, start=0):
    lens = rng.integers(lo, hi + 1, n).astype(np.uint64)
    gaps = rng.integers(0, gap + 1, n).astype(np.uint64) if gap else np.zeros(n, np.uint64)
    off = np.empty(n, np.uint64)
    pos = np.uint64(start)
    for i in range(n):
        pos += gaps[i]
        off[i] = pos
        pos += lens[i]
    return off, lens, int(pos)


def _check(ctx, oracle_mod, base, off, lens, apis=("entries", "batch"), finalize=True):
    base_t = torch.from_numpy(base).cuda()
    want = oracle_mod.entries(base, off, lens, finalize=finalize)
    for api in apis:
        got = _run(ctx, api, base_t, off, lens, finalize=finalize)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (api, bad[:10], got[bad[:5]], want[bad[:5]], off[bad[:5]], lens[bad[:5]])
    ctx.check()


@pytest.mark.parametrize("start", [0, 1, 3, 4, 13, 64, 127, 128])
def test_random_packed(ctx, oracle_mod, start):
    rng = np.random.default_rng(100 + start)
    off, lens, end = _table(rng, 3000, start=start)
    base = oracle_mod.splitmix_bytes(7 + start, end + 256)
    _check(ctx, oracle_mod, base, off, lens)


@pytest.mark.parametrize("gap", [1, 64, 4095])
def test_random_gapped(ctx, oracle_mod, gap):
    rng = np.random.default_rng(gap)
    off, lens, end = _table(rng, 4000, hi=3000, gap=gap, start=5)
    base = oracle_mod.splitmix_bytes(gap, end + 256)
    _check(ctx, oracle_mod, base, off, lens)


def test_small_and_empty_entries(ctx, oracle_mod):
    """Lengths 0 .. 12 (runs of empty entries, several boundaries per dword)."""
    rng = np.random.default_rng(5)
    off, lens, end = _table(rng, 20000, hi=12, start=2)
    base = oracle_mod.splitmix_bytes(5, end + 256)
    _check(ctx, oracle_mod, base, off, lens)


def test_step_aligned_boundaries(ctx, oracle_mod):
    """Entries of multiples of 128 bytes from a 128-byte aligned start: every
    boundary falls on a step (and often a span) boundary; empty ones too."""
    rng = np.random.default_rng(9)
    lens = (rng.integers(0, 40, 5000) * 128).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    end = int(off[-1] + lens[-1])
    base = oracle_mod.splitmix_bytes(9, end + 256)
    _check(ctx, oracle_mod, base, off, lens)
    # and each boundary 1, 2, 3, 4 bytes after a step start
    for shift in (1, 2, 3, 4):
        _check(ctx, oracle_mod, base, off + np.uint64(shift), lens, apis=("entries",))


@pytest.mark.parametrize("n,size", [(1, 1), (1, 0), (1, 300000), (2, 70000), (3, 9),
                                    (5, 1 << 20), (40, 200000)])
def test_few_and_large_entries(ctx, oracle_mod, n, size):
    """Entries much larger than a span (chains through k_stream_fix)."""
    lens = np.full(n, size, np.uint64)
    off = (np.arange(n, dtype=np.uint64) * np.uint64(size)) + np.uint64(3)
    base = oracle_mod.splitmix_bytes(n + size, int(off[-1] + lens[-1]) + 256)
    _check(ctx, oracle_mod, base, off, lens)


def test_window_refill(ctx, oracle_mod):
    """4M entries of 0 .. 24 bytes: about 200 entries per span, so every
    group refills its 64-entry window several times."""
    rng = np.random.default_rng(11)
    lens = rng.integers(0, 25, 4_000_000).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) + np.uint64(7)
    end = int(off[-1] + lens[-1])
    base = oracle_mod.splitmix_bytes(11, end + 256)
    _check(ctx, oracle_mod, base, off, lens, apis=("entries",))


def test_raw_output(ctx, oracle_mod):
    rng = np.random.default_rng(12)
    off, lens, end = _table(rng, 2000, start=9)
    base = oracle_mod.splitmix_bytes(12, end + 256)
    _check(ctx, oracle_mod, base, off, lens, finalize=False)


def test_config3_full(ctx, oracle_mod):
    """BASELINE config 3: 1M entries of the Zipf mix packed back to back."""
    lens = workloads.entry_lengths(1_000_000)
    off = workloads.packed_offsets(lens)
    total = int(lens.sum())
    base = workloads.splitmix_bytes_np(workloads.ENTRY_SEED, total)
    _check(ctx, oracle_mod, base, off, lens, apis=("entries",))


def test_1m_x_100(ctx, oracle_mod):
    lens = np.full(1_000_000, 100, np.uint64)
    off = workloads.packed_offsets(lens)
    base = workloads.splitmix_bytes_np(workloads.ENTRY_SEED, 100_000_000)
    _check(ctx, oracle_mod, base, off, lens, apis=("entries",))


@pytest.mark.parametrize("kind", ["overlap", "order", "gap"])
def test_refused_batches(ctx, ramcrc, oracle_mod, kind):
    rng = np.random.default_rng(13)
    off, lens, end = _table(rng, 1000, lo=10, hi=500)
    i = 500
    if kind == "overlap":
        off[i] = off[i - 1] + lens[i - 1] - np.uint64(1)
    elif kind == "order":
        off[i], off[i + 1] = off[i + 1], off[i]
    else:
        off[i:] += np.uint64(4096)
    base = oracle_mod.splitmix_bytes(13, int((off + lens).max()) + 256)
    base_t = torch.from_numpy(base).cuda()
    got = _run(ctx, "entries", base_t, off, lens, sentinel=0x5A5A5A5A)
    assert (got == 0x5A5A5A5A).all()   # nothing written
    with pytest.raises(ramcrc.RamcrcError) as e:
        ctx.check()
    assert e.value.code == ramcrc.EORDER
    # the context is usable again at once
    off2, lens2, end2 = _table(rng, 500, start=1)
    base2 = oracle_mod.splitmix_bytes(14, end2 + 256)
    _check(ctx, oracle_mod, base2, off2, lens2, apis=("entries",))
