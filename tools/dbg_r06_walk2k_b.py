"""Round 6 debug: bench-shaped 2 KiB replay (nseg segments, fused call
repeated like the bench's steps), records of the first ns segments against
the oracle after every call."""
import sys
import numpy as np
import torch
from ramcloud_amd import ramcrc, segments, workloads
from oracle import oracle
import bench

SEG = 8 << 20
nseg, vlen, reps, ns, shift = (int(a) for a in sys.argv[1:6])
ctx = ramcrc.Context(0)
if shift:
    ctx.set_walk_part_shift(shift)
d = torch.empty(nseg * SEG, dtype=torch.uint8, device="cuda")
certs_t = torch.zeros((nseg, 2), dtype=torch.int32, device="cuda")
per, _, _ = bench._fill_recovery_shard(ctx, d, SEG, 0, nseg, vlen, certs=certs_t)
certs = certs_t.cpu().numpy().view(np.uint32)
cap = per * nseg + nseg
rv = segments.RecoveryVerify(ctx, nseg, SEG, entries_cap=cap)
host = d[:ns * SEG].cpu().numpy()
want = []
for s in range(ns):
    _, _, _, t = oracle.check_metadata(host[s * SEG:(s + 1) * SEG], int(certs[s, 0]), int(certs[s, 1]),
                                       segment=s, capacity=SEG)
    want.append(t)
want = np.concatenate(want)
print("per", per, "want", want.shape, flush=True)
for r in range(reps):
    st = rv.verify(d, certs_t)
    torch.cuda.synchronize()
    n = int(rv.n_entries.item())
    t = rv.entries[:n].cpu().numpy().view(np.uint32).reshape(-1, 4)
    t = t[t[:, 0] < ns]
    t = t[np.lexsort((t[:, 1], t[:, 0]))]
    ok = t.shape == want.shape and np.array_equal(t, want)
    msg = ""
    if not ok:
        if t.shape == want.shape:
            bad = np.nonzero((t != want).any(axis=1))[0]
            i = bad[0]
            msg = f"{len(bad)} rows differ, segs {np.unique(want[bad, 0]).tolist()[:8]}; first {i}: got {t[i].tolist()} want {want[i].tolist()}"
        else:
            msg = f"shape {t.shape} vs {want.shape}"
    s = st.cpu().numpy().view(np.uint32)
    print(f"rep {r}: n {n} match {ok} seg_ok {(s[:, 0] == segments.SEG_OK).all()} {msg}", flush=True)
ctx.close()
