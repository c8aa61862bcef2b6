"""Certificates of rebuilt recovery segments on the device
(ramcrc_segments_certify_device): Segment::getAppendedLength
(src/Segment.cc:672-684) as a backup seals the segments
RecoverySegmentBuilder::build appended (src/BackupMasterRecovery.cc:367-368,
src/RecoverySegmentBuilder.cc:195).

  * the reference's own goldens: an empty segment, "hi" and "yo!" objects
    (src/SegmentTest.cc:159, 369, 373);
  * segments of mixed entries (objects of 24 B .. 200 KiB, tombstones) whose
    certificates the oracle's append restatement produced;
  * 8 MiB RecoverSegmentBenchmark object segments built on the device, whose
    certificates the fill computed;
  * heads that cut an entry or run past the last one: the certificate equals
    the oracle walk's checksum up to that head, and the flags say which."""
import numpy as np
import pytest

from ramcloud_amd import segments

import segment_cases

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _certify(ctx, buf, cap, nseg, heads, stride=None):
    d = torch.from_numpy(np.ascontiguousarray(buf)).cuda()
    h = torch.from_numpy(np.asarray(heads, dtype=np.uint32).view(np.int32)).cuda()
    certs = torch.zeros((nseg, 2), dtype=torch.int32, device="cuda")
    flags = torch.zeros(nseg, dtype=torch.int32, device="cuda")
    ctx.certify(d, stride or cap, cap, nseg, h, certs, flags)
    torch.cuda.synchronize()
    return certs.cpu().numpy().view(np.uint32), flags.cpu().numpy().view(np.uint32)


@pytest.fixture(scope="module")
def ctx(ramcrc):
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    c = ramcrc.Context(0)
    yield c
    c.close()


def test_certify_reference_goldens(ctx, golden):
    """The three SegmentTest certificates, each stream at the start of a
    64 KiB segment with a zero tail."""
    cap = 64 * 1024
    gold = golden["segment_certificates"]
    buf = np.zeros(len(gold) * cap, np.uint8)
    heads = []
    for i, c in enumerate(gold):
        stream = bytes.fromhex(c["stream"])
        head = c["segmentLength"]
        # the stream is the metadata bytes the checksum covers followed by the
        # 4 head bytes: rebuild the entry itself (header, length, payload)
        meta = stream[:len(stream) - 4]
        if meta:
            hdr, ln = meta[0], meta[1]
            entry = bytes([hdr, ln]) + {2: b"hi", 3: b"yo!"}[ln]   # SegmentTest's payloads
            buf[i * cap:i * cap + len(entry)] = np.frombuffer(entry, np.uint8)
            assert len(entry) == head
        heads.append(head)
    certs, flags = _certify(ctx, buf, cap, len(gold), heads)
    assert list(certs[:, 0]) == [c["segmentLength"] for c in gold]
    assert list(certs[:, 1]) == [c["checksum"] for c in gold]
    assert (flags == segments.SEG_OK).all()


def test_certify_mixed_segments(ctx, oracle_mod):
    cap, nseg = 1 * MiB, 12
    buf, certs, counts = segment_cases.mixed_segments(oracle_mod, nseg, cap)
    got, flags = _certify(ctx, buf, cap, nseg, certs[:, 0])
    assert np.array_equal(got, certs)
    assert (flags == segments.SEG_OK).all()
    assert counts.sum() > 1000


def test_certify_device_object_segments(ctx):
    """RecoverSegmentBenchmark's 8 MiB segments (1 KiB values), built in place
    on the device with their certificates; 64 B values too (dense walk)."""
    for value_len, nseg in ((1024, 64), (64, 16)):
        cap = 8 * MiB
        d = torch.empty(nseg * cap, dtype=torch.uint8, device="cuda")
        d.random_(0, 256)
        dc = torch.zeros((nseg, 2), dtype=torch.int32, device="cuda")
        per, seg_len, ck = ctx.fill_objects(d, cap, cap, nseg, value_len, certs=dc)
        heads = torch.full((nseg,), seg_len, dtype=torch.int32, device="cuda")
        certs = torch.zeros((nseg, 2), dtype=torch.int32, device="cuda")
        flags = torch.zeros(nseg, dtype=torch.int32, device="cuda")
        ctx.certify(d, cap, cap, nseg, heads, certs, flags)
        torch.cuda.synchronize()
        got = certs.cpu().numpy().view(np.uint32)
        assert (got[:, 0] == seg_len).all() and (got[:, 1] == ck).all(), value_len
        assert np.array_equal(got, dc.cpu().numpy().view(np.uint32))
        assert (flags.cpu().numpy() == segments.SEG_OK).all()


def test_certify_heads_off_the_entries(ctx, oracle_mod):
    """Heads inside an entry (the walk runs past the head), past the last
    entry (the zero tail walks as 2-byte INVALID entries) and at 0: the
    checksum is the oracle walk's up to that head; flags match its findings."""
    cap, nseg = 256 * 1024, 8
    buf, certs, _ = segment_cases.mixed_segments(oracle_mod, nseg, cap, seed=31)
    rng = np.random.default_rng(5)
    heads = []
    for i in range(nseg):
        pos = int(certs[i, 0])
        heads.append([pos - 1, pos + 6, int(rng.integers(1, pos)), 0, pos, cap, pos + 1,
                      int(rng.integers(pos, cap))][i])
    got, flags = _certify(ctx, buf, cap, nseg, heads)
    for i in range(nseg):
        s = buf[i * cap:(i + 1) * cap]
        f, ck, _, _ = oracle_mod.check_metadata(s, heads[i], 0, capacity=cap, table_cap=cap + 1)
        assert got[i, 0] == heads[i]
        assert got[i, 1] == ck, (i, heads[i])
        want = f & (2 | 4 | 32)
        assert flags[i] == (want if want else segments.SEG_OK), (i, heads[i], f, flags[i])
