"""Batched write path: Object::assembleForLog's checksum
(src/Object.cc:213-238, value Object::computeChecksum src/Object.cc:770-819)
stamped by the GPU into every object header, device- and host-resident,
against the oracle's CRC of bytes [4, len) -- bit for bit, including objects
shorter than the header (left unchanged), unaligned packing, objects on both
sides of the 64 KiB small/large split, and the reference's own goldens
(src/ObjectTest.cc:171,321)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

LENS = [0, 3, 4, 23, 24, 25, 35, 36, 100, 127, 128, 129, 1024, 4096, 65535, 65536, 65537,
        262144 + 7, 1 << 20, 3 * (1 << 20) + 5]


@pytest.fixture(scope="module")
def ctx(ramcrc):
    c = ramcrc.Context(0)
    yield c
    c.close()


def _packed(oracle_mod, lens, seed, gap=3):
    lens = np.asarray(lens, dtype=np.uint64)
    offs = np.zeros(lens.size, dtype=np.uint64)
    pos = 5   # unaligned first object
    for i, L in enumerate(lens):
        offs[i] = pos
        pos += int(L) + gap
    host = oracle_mod.splitmix_bytes(seed, pos + 16)
    return host, offs, lens


def _expect(oracle_mod, host, offs, lens):
    """Header checksum each object must end up with (0 for short objects)."""
    live = lens >= 24
    want = np.zeros(lens.size, np.uint32)
    if live.any():
        want[live] = oracle_mod.entries(host, offs[live] + 4, lens[live] - 4)
    return want, live


def _headers(buf, offs):
    idx = (offs[:, None].astype(np.int64) + np.arange(4)).reshape(-1)
    return buf[idx].reshape(-1, 4).copy().view("<u4")[:, 0]


@pytest.mark.parametrize("with_out", [True, False])
def test_assemble_device_edge_lengths(ctx, oracle_mod, with_out):
    rng = np.random.default_rng(8)
    lens = LENS + [int(x) for x in rng.integers(0, 9000, 400)]
    host, offs, lens = _packed(oracle_mod, lens, 31)
    want, live = _expect(oracle_mod, host, offs, lens)
    d = torch.from_numpy(host.copy()).cuda()
    off_t = torch.from_numpy(offs.view(np.int64)).cuda()
    len_t = torch.from_numpy(lens.view(np.int64)).cuda()
    out = torch.full((lens.size,), -1, dtype=torch.int32, device="cuda") if with_out else None
    ctx.assemble_objects(d, off_t, len_t, out)
    torch.cuda.synchronize()
    ctx.check()
    got = d.cpu().numpy()
    assert np.array_equal(_headers(got, offs)[live], want[live])
    # nothing but the live headers changed
    expect_buf = host.copy()
    for i in np.nonzero(live)[0]:
        o = int(offs[i])
        expect_buf[o:o + 4] = np.frombuffer(np.uint32(want[i]).tobytes(), np.uint8)
    assert np.array_equal(got, expect_buf)
    if with_out:
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


def test_assemble_then_verify_roundtrip(ctx, oracle_mod):
    """Stamped objects pass Object::computeChecksum == header.checksum
    (src/ObjectManager.cc:659-663) on the oracle."""
    lens = [24, 35, 100, 1024, 4096, 70000]
    host, offs, lens = _packed(oracle_mod, lens, 5, gap=0)
    d = torch.from_numpy(host.copy()).cuda()
    ctx.assemble_objects(d, torch.from_numpy(offs.view(np.int64)).cuda(),
                         torch.from_numpy(lens.view(np.int64)).cuda())
    torch.cuda.synchronize()
    buf = d.cpu().numpy()
    for o, L in zip(offs, lens):
        o, L = int(o), int(L)
        stored = int(buf[o:o + 4].view("<u4")[0])
        assert oracle_mod.crc32c(buf[o + 4:o + L]) == stored


def test_assemble_reference_goldens(ctx, golden, oracle_mod):
    objs = golden["object_checksums"]
    blobs = [b"\0\0\0\0" + bytes.fromhex(g["bytes"]) for g in objs]
    host = np.frombuffer(b"".join(blobs), np.uint8).copy()
    offs = np.cumsum([0] + [len(b) for b in blobs[:-1]]).astype(np.uint64)
    lens = np.array([len(b) for b in blobs], np.uint64)
    d = torch.from_numpy(host).cuda()
    ctx.assemble_objects(d, torch.from_numpy(offs.view(np.int64)).cuda(),
                         torch.from_numpy(lens.view(np.int64)).cuda())
    torch.cuda.synchronize()
    assert list(_headers(d.cpu().numpy(), offs)) == [g["checksum"] for g in objs]


def test_assemble_host(ctx, oracle_mod):
    rng = np.random.default_rng(12)
    lens = LENS + [int(x) for x in rng.integers(0, 5000, 50)]
    objs = [oracle_mod.splitmix_bytes(100 + i, L) for i, L in enumerate(lens)]
    before = [o.copy() for o in objs]
    ctx.assemble_objects_host(objs)
    for o, b in zip(objs, before):
        if o.size < 24:
            assert np.array_equal(o, b)
            continue
        assert np.array_equal(o[4:], b[4:])
        assert int(o[:4].view("<u4")[0]) == oracle_mod.crc32c(b[4:])


def test_assemble_empty(ctx):
    base = torch.zeros(16, dtype=torch.uint8, device="cuda")
    e = torch.zeros(0, dtype=torch.int64, device="cuda")
    ctx.assemble_objects(base, e, e)
    ctx.assemble_objects_host([])
    torch.cuda.synchronize()
    assert int(base.sum()) == 0
