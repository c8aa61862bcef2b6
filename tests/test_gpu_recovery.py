"""BASELINE config 4 at its stated size on one MI355X: 2048 x 8 MiB = 16 GiB of
RecoverSegmentBenchmark-shaped object segments
(nanobenchmarks/RecoverSegmentBenchmark.cc:123-146, 1 KiB values, keys
continuing across segments) built on the device, then

  * the full-segment CRC of every segment (ramcrc_segments_device, the
    recovery-scan shard of one GPU, and the C-ABI shard entry with one rank),
  * Segment::checkMetadataIntegrity of every segment and every object's
    Object::computeChecksum against its stored checksum (walk + verify),

all against the oracle on the host copy.  The device fill itself is checked
byte for byte against the host append path (ramcrc_segment_fill_objects)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

MiB = 1 << 20
SEG = 8 * MiB
NSEG = 2048
VLEN = 1024


@pytest.fixture(scope="module")
def batch(ramcrc):
    from ramcloud_amd import segments, workloads
    ctx = ramcrc.Context(0)
    d = torch.empty(NSEG * SEG, dtype=torch.uint8, device="cuda")
    certs = torch.zeros((NSEG, 2), dtype=torch.int32, device="cuda")
    workloads.splitmix_fill_segments(d, SEG, workloads.SEGMENT_SEED)
    per, length, ck = ctx.fill_objects(d, SEG, SEG, NSEG, VLEN, first_key=0, certs=certs)
    assert per == segments.objects_per_segment(SEG, VLEN) == 7898
    torch.cuda.synchronize()
    yield ctx, d, certs, per, (length, ck)
    ctx.close()


def test_device_fill_equals_host_fill(ramcrc, batch):
    from ramcloud_amd import workloads
    ctx, d, certs, per, (length, ck) = batch
    for i in (0, 1, 1023, NSEG - 1):
        host = workloads.splitmix_bytes_np(workloads.SEGMENT_SEED + i, SEG)
        n, hl, hck = ramcrc.segment_fill_objects(host, VLEN, first_key=i * per)
        assert (n, hl, hck) == (per, length, ck)
        assert np.array_equal(d[i * SEG:(i + 1) * SEG].cpu().numpy(), host), i
    c = certs.cpu().numpy().view(np.uint32)
    assert (c[:, 0] == length).all() and (c[:, 1] == ck).all()


def test_recovery_batch_full_size(ramcrc, oracle_mod, batch):
    from ramcloud_amd import segments
    ctx, d, certs, per, (length, ck) = batch
    out = torch.zeros(NSEG, dtype=torch.int32, device="cuda")
    ctx.segments(d, SEG, NSEG, out)
    sh = ramcrc.Shard(devices=[0])
    try:
        out2 = torch.zeros(NSEG, dtype=torch.int32, device="cuda")
        sh.segments([d], SEG, NSEG, outs=[out2])
        sh.sync()
    finally:
        sh.close()
    rv = segments.RecoveryVerify(ctx, NSEG, SEG, entries_cap=NSEG * per + NSEG)
    st = rv.verify(d, certs, check=True)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(out2.cpu().numpy().view(np.uint32), got)
    status = st.cpu().numpy().view(np.uint32)
    n = int(rv.n_entries.item())
    table = rv.entries[:n].cpu().numpy().view(np.uint32)
    obj_crc = rv.obj_crc[:n].cpu().numpy().view(np.uint32)
    host = d.cpu().numpy()
    want = oracle_mod.segments(host, SEG, NSEG, threads=16)
    assert np.array_equal(got, want)
    # metadata walk of every segment and every object's checksum
    assert (status[:, 0] == segments.SEG_OK).all()
    assert (status[:, 2] == per).all() and (status[:, 3] == 0).all()
    assert (status[:, 1] == ck).all()
    assert n == NSEG * per
    for i in (0, 777, NSEG - 1):
        f, k, cnt, _ = oracle_mod.check_metadata(host[i * SEG:(i + 1) * SEG], length, ck, segment=i)
        assert (f, k, cnt) == (segments.SEG_OK, ck, per)
    bad, crc_exp, _ = oracle_mod.verify_objects(host, SEG, table, NSEG)
    assert bad == 0
    assert np.array_equal(obj_crc, crc_exp)
