"""Diagnostic for the small-entry binning (it found the round-2 histogram bug,
DESIGN.md section 9) and the batch path with and without large buffers (the
plan skip): repeats test_plan_skip_alternating's sequence with several seeds and
prints every mismatching entry (index, offset, length, init, got, want) and
whether an immediate re-run of the same call reproduces it."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import oracle  # noqa: E402
from ramcloud_amd import ramcrc  # noqa: E402


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


MODE = "plain"


def call(ctx, base, offs, lens, init):
    out = torch.zeros(len(offs), dtype=torch.int32, device="cuda")
    off_t = dev(np.asarray(offs, dtype=np.uint64).view(np.int64))
    len_t = dev(np.asarray(lens, dtype=np.uint64).view(np.int64))
    init_t = None if init is None else dev(np.asarray(init, dtype=np.uint32).view(np.int32))
    if MODE == "sync":
        torch.cuda.synchronize()
    elif MODE == "touch":
        (off_t ^ len_t).sum().item()
    elif MODE == "clone":
        off_t, len_t = off_t.clone(), len_t.clone()
    ctx.batch(base, off_t, len_t, out, init=init_t)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def main():
    global MODE
    if len(sys.argv) > 2:
        MODE = sys.argv[2]
    oracle.lib()
    total = 8 << 20
    host = oracle.splitmix_bytes(11, total)
    base = dev(host)
    nbad_calls = 0
    for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
        ctx = ramcrc.Context(0)
        rng = np.random.default_rng(99 + seed)
        for k in range(6):
            big = k % 2 == 1
            lens = [int(x) for x in rng.integers(0, 5000, 2000)]
            if big:
                lens += [65536, 65537, 300000, 1 << 20]
            offs = [int(rng.integers(0, total - L + 1)) for L in lens]
            init = None if k % 3 == 0 else rng.integers(0, 2 ** 32, len(lens),
                                                       dtype=np.uint64).astype(np.uint32)
            got = call(ctx, base, offs, lens, init)
            want = oracle.entries(host, offs, lens, init=init)
            bad = np.nonzero(got != want)[0]
            if bad.size:
                nbad_calls += 1
                count, cursor, hist, par_next = ctx.debug_bins()
                par = par_next ^ 1
                mism = np.nonzero(count != cursor[par])[0]
                print(f"  par {par}: bins with count != cursor: "
                      f"{[(int(b), int(count[b]), int(cursor[par][b]), int(hist[par][b])) for b in mism[:10]]}",
                      flush=True)
                again = call(ctx, base, offs, lens, init)
                print(f"seed {seed} k {k}: {bad.size} bad; rerun bad "
                      f"{int(np.count_nonzero(again != want))}", flush=True)
                for i in bad[:12]:
                    print(f"   i={i} off={offs[i]} len={lens[i]} init="
                          f"{None if init is None else hex(int(init[i]))} got={got[i]:#010x} "
                          f"want={want[i]:#010x} rerun={again[i]:#010x}", flush=True)
        try:
            ctx.check()
        except ramcrc.RamcrcError as e:
            print("check:", e, flush=True)
        ctx.close()
    print(f"bad calls: {nbad_calls}", flush=True)


if __name__ == "__main__":
    main()
