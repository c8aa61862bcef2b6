"""The reference's own walk scenarios on the device: every case of
tests/golden/segment_walk_ref.json (src/SegmentTest.cc:598-648 at 8 MiB and
66,560-byte segments, src/SegmentIteratorTest.cc:44-186) through both
ramcrc_segment_walk_device walkers (the parallel walk at two part sizes and
the serial one) and, where the case has an appended head,
ramcrc_segments_certify_device.  The flag each case ends with is the outcome
the reference test expects (OK / bad checksum / past expected length / past
allocated size); records are the entries the reference test finds; every
other status field equals the oracle's restatement."""
import numpy as np
import pytest

from ramcloud_amd import segments

import segment_ref

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def groups(oracle_mod):
    return segment_ref.batches(oracle_mod)


@pytest.mark.parametrize("walker", ["parallel", "parallel_8k_parts", "serial"])
def test_walkers_match_reference_expectations(ramcrc, oracle_mod, groups, walker):
    for cap, (cases, buf, certs) in sorted(groups.items()):
        nseg = len(cases)
        ctx = ramcrc.Context(0)
        if walker == "serial":
            ctx.set_serial_walk(True)
        elif walker == "parallel_8k_parts":
            ctx.set_walk_part_shift(13)
        d = torch.from_numpy(buf).cuda()
        dc = torch.from_numpy(np.ascontiguousarray(certs).view(np.int32)).cuda()
        rv = segments.RecoveryVerify(ctx, nseg, cap, entries_cap=64)
        st = rv.verify(d, dc, check=True).cpu().numpy().view(np.uint32)
        n = int(rv.n_entries.item())
        table = rv.entries[:n].cpu().numpy().view(np.uint32)
        for i, c in enumerate(cases):
            seg = buf[i * cap:(i + 1) * cap]
            f, ck, ne, _ = oracle_mod.check_metadata(seg, c["cert"][0], c["cert"][1],
                                                     capacity=cap, table_cap=cap + 1)
            assert st[i, 0] == segment_ref.flag_value(c["expect"]), (c["name"], st[i], walker)
            assert (st[i, 0], st[i, 1], st[i, 2]) == (f, ck, ne), (c["name"], st[i], walker)
            if "records" in c:
                mine = table[table[:, 0] == i]
                mine = mine[np.argsort(mine[:, 1], kind="stable")]
                assert segment_ref.records_of(mine) == c["records"], (c["name"], walker)
        ctx.close()


def test_certify_matches_reference_certificates(ramcrc, oracle_mod, groups):
    ctx = ramcrc.Context(0)
    checked = 0
    for cap, (cases, buf, _) in sorted(groups.items()):
        nseg = len(cases)
        heads = np.array([c.get("head", 0) for c in cases], np.uint32)
        d = torch.from_numpy(buf).cuda()
        h = torch.from_numpy(heads.view(np.int32)).cuda()
        certs = torch.zeros((nseg, 2), dtype=torch.int32, device="cuda")
        flags = torch.zeros(nseg, dtype=torch.int32, device="cuda")
        ctx.certify(d, cap, cap, nseg, h, certs, flags)
        torch.cuda.synchronize()
        got = certs.cpu().numpy().view(np.uint32)
        fl = flags.cpu().numpy().view(np.uint32)
        for i, c in enumerate(cases):
            if "head" not in c:
                continue
            want = c["certify"]
            assert fl[i] == segment_ref.flag_value(want["flags"]), (c["name"], fl[i])
            assert got[i, 0] == c["head"]
            if want["cert"] is not None:
                # getAppendedLength of the appended entries (reference value)
                assert list(got[i]) == want["cert"], (c["name"], got[i])
            else:
                # the walk's checksum of what it read up to the head (oracle)
                seg = buf[i * cap:(i + 1) * cap]
                _, ck, _, _ = oracle_mod.check_metadata(seg, c["head"], 0, capacity=cap,
                                                        table_cap=cap + 1)
                assert got[i, 1] == ck, c["name"]
            checked += 1
    ctx.close()
    assert checked >= 12
