"""Round 6 debug: the 2 KiB-value replay line's records against the oracle's
walk, per forced part shift and per call (fused replay verify / walk only)."""
import sys
import numpy as np
import torch
from ramcloud_amd import ramcrc, segments
from oracle import oracle

SEG = 8 << 20
nseg = int(sys.argv[1]) if len(sys.argv) > 1 else 16
vlen = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
ctx = ramcrc.Context(0)
d = torch.empty(nseg * SEG, dtype=torch.uint8, device="cuda")
certs = torch.zeros((nseg, 2), dtype=torch.int32, device="cuda")
from ramcloud_amd import workloads
workloads.splitmix_fill_segments(d, SEG, 0x5A17)
per, _, _ = ctx.fill_objects(d, SEG, SEG, nseg, vlen, first_key=0, certs=certs)
torch.cuda.synchronize()
host = d.cpu().numpy()
cn = certs.cpu().numpy().view(np.uint32)
want = []
for s in range(nseg):
    _, _, _, t = oracle.check_metadata(host[s * SEG:(s + 1) * SEG], int(cn[s, 0]), int(cn[s, 1]),
                                       segment=s, capacity=SEG)
    want.append(t)
want = np.concatenate(want)
print("per", per, "oracle records", want.shape[0], flush=True)
for shift in (0, 16, 17, 18):
    for fused in (True, False):
        c2 = ramcrc.Context(0)
        if shift:
            c2.set_walk_part_shift(shift)
        rv = segments.RecoveryVerify(c2, nseg, SEG, entries_cap=nseg * per + nseg)
        if fused:
            st = rv.verify(d, certs, check=True)
        else:
            rv.walk(d, certs)
            st = rv.verify_objects(d)
            rv.check()
        torch.cuda.synchronize()
        n = int(rv.n_entries.item())
        t = rv.entries[:n].cpu().numpy().view(np.uint32).reshape(-1, 4)
        o = np.lexsort((t[:, 1], t[:, 0]))
        t = t[o]
        ok = t.shape == want.shape and np.array_equal(t, want)
        msg = ""
        if not ok and t.shape == want.shape:
            bad = np.nonzero((t != want).any(axis=1))[0]
            i = bad[0]
            msg = f"{len(bad)} rows differ; first {i}: got {t[i].tolist()} want {want[i].tolist()}"
            # duplicates / missing
            gk = set(map(tuple, t[:, :2].tolist())); wk = set(map(tuple, want[:, :2].tolist()))
            msg += f"; missing {len(wk - gk)} extra {len(gk - wk)}"
            if wk - gk:
                msg += f" e.g. missing {sorted(wk - gk)[:3]}"
        elif not ok:
            msg = f"shape {t.shape} vs {want.shape}"
        print(f"shift {shift} fused {fused}: n {n} match {ok} {msg}", flush=True)
        c2.close()
ctx.close()
