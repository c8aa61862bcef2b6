"""k_entries phase timing from a RAMCRC_STAMPS=1 build (probe, not product).

    RAMCRC_LIB=ramcloud_amd/lib/variants/libramcrc_stamps.so \\
        python tools/stamps.py [--entry-size S] [--replay]

Runs the config-3 entries batch (or 1M entries of one size) a few times, then
prints, over all waves of the last launch, when each phase ended relative to
the kernel's first stamp (100 MHz clock: 10 ns units): start, tiny phase,
LDS refill, short bins, long bins.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--entry-size", type=int, default=0)
    ap.add_argument("--entries", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--save", default="", help="write the raw stamps (.npy)")
    a = ap.parse_args()
    import torch
    from ramcloud_amd import ramcrc, workloads
    ctx = ramcrc.Context(0)
    lens = workloads.entry_lengths(a.entries)
    if a.entry_size:
        lens = lens * 0 + np.uint64(a.entry_size)
    offs = workloads.packed_offsets(lens)
    total = int(lens.sum())
    data = torch.empty(((total + 7) // 8) * 8, dtype=torch.uint8, device="cuda")
    data[:total].copy_(torch.from_numpy(workloads.splitmix_bytes_np(workloads.ENTRY_SEED, total)))
    off_t = torch.from_numpy(offs.view(np.int64)).cuda()
    len_t = torch.from_numpy(lens.view(np.int64)).cuda()
    out = torch.zeros(lens.size, dtype=torch.int32, device="cuda")
    for _ in range(a.reps):
        ctx.entries(data, off_t, len_t, out)
    torch.cuda.synchronize()
    ctx.check()
    L = ramcrc.lib()
    L.ramcrc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    st = np.zeros(8192 * 8, dtype=np.uint64)
    rc = L.ramcrc_debug_stamps(st.ctypes.data, st.nbytes)
    if rc != 0:
        sys.exit(f"ramcrc_debug_stamps: {rc} (not a RAMCRC_STAMPS build?)")
    raw = st.reshape(-1, 8).astype(np.int64)
    st = raw[:, :5]
    st = st[:4096] if (st[:4096, 0] > 0).all() else st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    rel = (st - t0) * 10 / 1000.0   # us
    names = ["start", "tiny done", "refill done", "short done", "long done"]
    mix = f"{a.entry_size} B" if a.entry_size else "config-3 mix"
    print(f"k_entries phase ends, us after the first wave's start ({len(st)} waves, 1M x {mix}):")
    for k, n in enumerate(names):
        c = rel[:, k]
        print(f"  {n:12s} min {c.min():8.2f}  p10 {np.percentile(c, 10):8.2f}  median {np.median(c):8.2f}"
              f"  p90 {np.percentile(c, 90):8.2f}  max {c.max():8.2f}")
    if (raw[: len(st), 5] > 0).any():   # tiny phase: table filled, first round done
        t5 = (raw[: len(st), 5] - t0) * 10 / 1000.0
        t6 = (raw[: len(st), 6] - t0) * 10 / 1000.0
        ok = raw[: len(st), 6] > raw[: len(st), 5]
        print(f"  tiny: table filled median {np.median(t5):.2f} max {t5.max():.2f}; first round done "
              f"median {np.median(t6[ok]):.2f} max {t6[ok].max():.2f} ({ok.sum()} waves)")
    d = np.diff(rel, axis=1)
    for k in range(4):
        c = d[:, k]
        print(f"  dur {names[k+1]:12s} median {np.median(c):8.2f}  p90 {np.percentile(c, 90):8.2f}  max {c.max():8.2f}")
    print(f"  kernel span {rel[:, 4].max():.2f} us; mean wave busy {np.mean(rel[:, 4] - rel[:, 0]):.2f} us")
    # where the slow waves are: by workgroup % 8 (XCD under round-robin
    # dispatch) and by wave slot in the workgroup (slot % 4 = SIMD)
    idx = np.nonzero(st[:, 0] > 0)[0] if False else np.arange(len(st))
    wg, slot = idx // 16, idx % 16
    end = rel[:, 4]
    print("  long-done median by workgroup % 8:",
          " ".join(f"{np.median(end[wg % 8 == x]):.1f}" for x in range(8)))
    print("  long-done median by wave slot:", " ".join(f"{np.median(end[slot == x]):.1f}" for x in range(16)))
    e16 = end[: len(end) // 16 * 16].reshape(-1, 16)
    print(f"  long-done spread inside a workgroup (max - min): median {np.median(e16.max(1) - e16.min(1)):.1f}"
          f"; workgroup means: min {e16.mean(1).min():.1f} median {np.median(e16.mean(1)):.1f}"
          f" max {e16.mean(1).max():.1f}")
    r16 = rel[: len(end) // 16 * 16, 2].reshape(-1, 16).max(1)   # workgroup's refill (tiny phase end)
    late = r16 > np.median(r16) + 2.0
    if late.any():
        print(f"  workgroups whose tiny phase ended > 2 us after the median: {late.sum()}; their long-done mean "
              f"{e16.mean(1)[late].mean():.1f} vs {e16.mean(1)[~late].mean():.1f} for the others")
    # long-phase duration per workgroup against its index: workgroups own
    # contiguous ranges of the bins (small bins first), so a trend here is
    # the work estimate (kcost) disagreeing with the time an octet takes
    lg = (rel[:, 4] - rel[:, 2])[: len(end) // 16 * 16].reshape(-1, 16).mean(1)
    dec = np.array_split(np.arange(lg.size), 8)
    print("  long-phase mean by workgroup-index eighth:", " ".join(f"{lg[x].mean():.1f}" for x in dec))
    if a.save:
        np.save(a.save, raw)
    order = np.argsort(np.argsort(rel[:, 0].reshape(-1, 16), axis=1), axis=1).reshape(-1)
    print("  long-done median by start rank in workgroup:",
          " ".join(f"{np.median(end[order == x]):.1f}" for x in range(16)))


if __name__ == "__main__":
    main()
