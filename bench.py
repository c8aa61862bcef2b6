"""Benchmark: device-resident CRC32C over a batch of 8 MiB segments (BASELINE config 2).

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--config segments|recovery|entries|stream|replay|append|host]

One step = one pass of the hot path over one batch: ramcrc_segments_device on
1024 x 8 MiB = 8 GiB of segments already resident in this GPU's HBM (the
recovery-scan batch, src/BackupMasterRecovery.cc:743-809), plus -- with N > 1
-- the RCCL all-gather of the per-segment CRCs (the only exchange step).
Weak scaling: every rank owns its own 1024 segments.

Rank 0 prints one JSON line.  `roofline` prices the dominant kernel (k_chunks)
from its own HIP-event duration on the launch stream; `cpu_baseline` times the
reference's compiled intelCrc32C (oracle/_ref) -- or the oracle restatement if
_ref was not shipped -- on a bounded sample of the same segments on this
host's cores, and checks the GPU CRCs of that sample bit for bit.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from ramcloud_amd import ramcrc, workloads  # noqa: E402
from ramcloud_amd.recovery_scan import RecoveryScan, shard_range  # noqa: E402

MiB = 1 << 20
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "device-resident CRC32C GB/s over 8MiB-segment batch; % of HBM roofline"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_traffic(kernel):
    """Corrected HBM bytes per launch from the committed PMC summary, if any."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d[kernel]["hbm_read_bytes_per_launch_corrected"]
    except Exception:
        return None


def cpu_baseline(host_sample, seg_bytes, nseg_sample, gpu_crcs):
    from oracle import oracle
    kind = "reference" if oracle.ref_available() else "port"
    use_ref = kind == "reference"
    try:
        cpus = len(os.sched_getaffinity(0))
    except AttributeError:
        cpus = os.cpu_count() or 1
    threads = max(1, min(16, cpus))
    res = {}
    for t in sorted({1, threads}):
        best = None
        crcs = None
        for _ in range(3):
            t0 = time.perf_counter()
            crcs = oracle.segments(host_sample, seg_bytes, nseg_sample, threads=t, use_ref=use_ref)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        res[t] = (nseg_sample * seg_bytes / best / 1e9, crcs)
    ok = all(np.array_equal(c, gpu_crcs) for _, c in res.values())
    value, _ = res[threads]
    return {
        "value": round(value, 3), "unit": "GB/s", "cores": threads, "kind": kind,
        "sample": f"{nseg_sample} x {seg_bytes // MiB} MiB of the same segments "
                  f"(first {nseg_sample} of the batch), best of 3, "
                  f"{'RAMCloud intelCrc32C (src/Crc32C.h:39-93) built -O3 -msse4.2' if use_ref else 'oracle restatement'}, "
                  f"whole segments round-robin over pinned threads",
        "single_thread_GBs": round(res[1][0], 3),
        "host_cpus_visible": cpus,
        "bit_exact_vs_gpu": bool(ok),
    }


def run_segments(args, rank, world, local_rank, ctx):
    seg_bytes = args.seg_mib * MiB
    if args.config == "recovery":
        nseg_total = args.nseg_total
        lo, hi = shard_range(nseg_total, rank, world)
        nseg = hi - lo
        first_seed = workloads.SEGMENT_SEED + lo
        scaling = "strong"
    else:
        nseg = args.nseg
        nseg_total = nseg * world
        first_seed = workloads.SEGMENT_SEED + rank * nseg
        scaling = "weak"
    data = torch.empty(nseg * seg_bytes, dtype=torch.uint8, device="cuda")
    workloads.splitmix_fill_segments(data, seg_bytes, first_seed)
    out = torch.zeros(nseg, dtype=torch.int32, device="cuda")
    if args.config == "recovery":
        scan = RecoveryScan(nseg_total, seg_bytes, rank, world, ctx=ctx)
    else:
        scan = RecoveryScan(nseg_total, seg_bytes, rank, world,
                            scan_fn=lambda d, sb, c, o: ctx.segments(d, sb, c, o))
        scan.lo, scan.hi = rank * nseg, (rank + 1) * nseg
    torch.cuda.synchronize()

    def step():
        return scan.step(data, out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ctx.set_timing(True)
    ctx.scan_time()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        full = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    scan_ms, launches = ctx.scan_time()
    ctx.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    gpu_crcs = full.cpu().numpy().view(np.uint32) if world > 1 else out.cpu().numpy().view(np.uint32)
    local_crcs = out.cpu().numpy().view(np.uint32)
    return dict(seg_bytes=seg_bytes, nseg=nseg, nseg_total=nseg_total, elapsed=elapsed,
                scan_ms=scan_ms, launches=launches, data=data, local_crcs=local_crcs,
                all_crcs=gpu_crcs, first_seed=first_seed, scaling=scaling)


def max_over_ranks(elapsed, world):
    """Whole-job time: the slowest rank's timed region."""
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def run_entries(args, ctx, world=1):
    """Config 3. The small-entry batch does not shard: at N>1
    every rank runs an independent replica of the same 1M-entry batch, and the
    job value is N x bytes / the slowest rank's time (weak scaling)."""
    lens = workloads.entry_lengths(args.entries)
    if args.entry_size:
        lens = lens * 0 + np.uint64(args.entry_size)
    offs = workloads.packed_offsets(lens)
    total = int(lens.sum())
    data = torch.empty(((total + 7) // 8) * 8, dtype=torch.uint8, device="cuda")
    host = workloads.splitmix_bytes_np(workloads.ENTRY_SEED, total)
    data[:total].copy_(torch.from_numpy(host))
    off_t = torch.from_numpy(offs.view(np.int64)).cuda()
    len_t = torch.from_numpy(lens.view(np.int64)).cuda()
    out = torch.zeros(lens.size, dtype=torch.int32, device="cuda")
    fn = ctx.entries if args.path == "entries" else ctx.batch
    for _ in range(args.warmup):
        fn(data, off_t, len_t, out)
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.scan_time()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fn(data, off_t, len_t, out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    scan_ms, launches = ctx.scan_time()
    ctx.set_timing(False)
    return dict(total=total, n=lens.size, elapsed=elapsed, scan_ms=scan_ms, launches=launches,
                host=host, offs=offs, lens=lens, crcs=out.cpu().numpy().view(np.uint32))


def run_replay(args, ctx):
    """Recovery replay verify (RecoverSegmentBenchmark-shaped,
    nanobenchmarks/RecoverSegmentBenchmark.cc:123-146): nseg 8 MiB segments
    full of objects with 8-byte counter keys and value_len-byte values, built
    by the host append path; one step = Segment::checkMetadataIntegrity of
    every segment (src/Segment.cc:758-800) + Object::computeChecksum of every
    object compared with its stored checksum (src/ObjectManager.cc:659-669)."""
    from ramcloud_amd import segments
    seg_bytes = args.seg_mib * MiB
    nseg = args.replay_nseg
    # value bytes: splitmix64 streams generated on the device, objects
    # appended on the host (C append path, threads), copied back
    d = torch.empty(nseg * seg_bytes, dtype=torch.uint8, device="cuda")
    workloads.splitmix_fill_segments(d, seg_bytes, segments.REPLAY_SEED)
    host = d.cpu().numpy()
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    certs, counts = segments.fill_segments_host(host, nseg, seg_bytes, args.value_len,
                                                threads=threads)
    d.copy_(torch.from_numpy(host))
    dc = torch.from_numpy(np.ascontiguousarray(certs).view(np.int32)).cuda()
    cap = int(counts.sum()) + nseg
    if args.walk_cus:
        elapsed, scan_ms, launches, sts = _replay_pipelined(args, ctx, d, dc, nseg, seg_bytes, cap)
    else:
        rv = segments.RecoveryVerify(ctx, nseg, seg_bytes, entries_cap=cap)
        for _ in range(args.warmup):
            rv.verify(d, dc)
        torch.cuda.synchronize()
        ctx.set_timing(True)
        ctx.scan_time()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            st = rv.verify(d, dc)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        scan_ms, launches = ctx.scan_time()
        ctx.set_timing(False)
        sts = [st]
    ok = True
    for st in sts:
        status = st.cpu().numpy().view(np.uint32)
        ok = ok and bool((status[:, 0] == segments.SEG_OK).all() and (status[:, 3] == 0).all()
                         and np.array_equal(status[:, 2], counts)
                         and np.array_equal(status[:, 1], certs[:, 1]))
    return dict(seg_bytes=seg_bytes, nseg=nseg, counts=counts, certs=certs, host=host,
                elapsed=elapsed, scan_ms=scan_ms, launches=launches, ok=ok)


def _walk_cu_list(ncu, walk_cus):
    """CUs for the walk stream: runs of 8 consecutive CU ids spread evenly
    over the device, so every XCD gets an equal share whether CU ids map to
    XCDs round-robin (id % 8) or in contiguous blocks (id // 32)."""
    runs = walk_cus // 8
    stride = ncu // 8 // runs
    return [r * stride * 8 + j for r in range(runs) for j in range(8)]


def _replay_pipelined(args, ctx, d, dc, nseg, seg_bytes, cap):
    """Replay of a stream of segment batches (a recovery master replaying
    batch after batch, src/ObjectManager.cc:580-1100) with the walk of batch k
    on walk_cus CUs overlapped with the object scan of batch k-1 on the
    others (ramcrc_stream_create_cu_mask).  Two batches alternate: the second
    is a copy of the first at another HBM address.  Every timed step walks and
    verifies exactly one whole batch: the first walk and the last scan are
    inside the timed region."""
    from ramcloud_amd import ramcrc, segments
    dev = torch.cuda.current_device()
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    walk = _walk_cu_list(ncu, args.walk_cus)
    rest = [c for c in range(ncu) if c not in set(walk)]
    s_walk = ramcrc.CuMaskStream(dev, walk)
    s_scan = ramcrc.CuMaskStream(dev, rest)
    t_walk = torch.cuda.ExternalStream(s_walk.handle)
    t_scan = torch.cuda.ExternalStream(s_scan.handle)
    ctx_walk = ramcrc.Context(dev)
    ctx.set_cus(len(rest))
    bufs = [d, d.clone()]
    rvs = [segments.RecoveryVerify(ctx, nseg, seg_bytes, entries_cap=cap) for _ in range(2)]
    ev_walk = [torch.cuda.Event() for _ in range(2)]
    ev_scan = [torch.cuda.Event() for _ in range(2)]
    torch.cuda.synchronize()

    def do_walk(k):
        b = k % 2
        if k >= 2:
            t_walk.wait_event(ev_scan[b])   # batch k-2's scan has read table b
        rv = rvs[b]
        ctx_walk.segment_walk(bufs[b], rv.stride, rv.capacity, nseg, dc, rv.status, rv.entries,
                              rv.n_entries, stream=s_walk)
        ev_walk[b].record(t_walk)

    def do_scan(k):
        b = k % 2
        t_scan.wait_event(ev_walk[b])
        rvs[b].verify_objects(bufs[b], stream=s_scan)
        ev_scan[b].record(t_scan)

    def run(steps):
        for k in range(steps):
            do_walk(k)
            if k:
                do_scan(k - 1)
        do_scan(steps - 1)

    run(max(args.warmup, 2))
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.scan_time()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    scan_ms, launches = ctx.scan_time()
    ctx.set_timing(False)
    sts = [rv.status.clone() for rv in rvs]
    ctx.set_cus(0)
    ctx_walk.close()
    s_walk.destroy()
    s_scan.destroy()
    return elapsed, scan_ms, launches, sts


def run_append(args, ctx):
    """Batched write-path checksum: Object::assembleForLog
    (src/Object.cc:213-238) over a batch of 1M serialized objects of the
    config-3 sizes (100 B / 1 KiB / 4 KiB, Zipf), packed back to back in HBM;
    one step = every header.checksum computed and stamped."""
    from oracle import oracle
    lens = workloads.entry_lengths(args.entries)
    offs = workloads.packed_offsets(lens)
    total = int(lens.sum())
    host = workloads.splitmix_bytes_np(workloads.ENTRY_SEED, total)
    data = torch.from_numpy(host).cuda()
    off_t = torch.from_numpy(offs.view(np.int64)).cuda()
    len_t = torch.from_numpy(lens.view(np.int64)).cuda()
    out = torch.zeros(lens.size, dtype=torch.int32, device="cuda")
    for _ in range(args.warmup):
        ctx.assemble_objects(data, off_t, len_t, out)
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.scan_time()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.assemble_objects(data, off_t, len_t, out)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    scan_ms, _ = ctx.scan_time()
    ctx.set_timing(False)
    credited = total - 4 * lens.size   # bytes [4, len) of every object
    want = oracle.entries(host, offs + 4, lens - 4)
    got = out.cpu().numpy().view(np.uint32)
    stamped = data.cpu().numpy()
    hdr = stamped[(offs.astype(np.int64)[:, None] + np.arange(4)).reshape(-1)].reshape(-1, 4).copy().view("<u4")[:, 0]
    ok = bool(np.array_equal(got, want) and np.array_equal(hdr, want))
    value = credited * args.steps / elapsed / 1e9
    scan_s = scan_ms / args.steps / 1e3
    achieved = credited / scan_s / 1e9 if scan_s > 0 else None
    return {
        "metric": "device-resident Object::assembleForLog checksum GB/s over 1M objects "
                  "(100B/1KiB/4KiB Zipf)",
        "value": round(value, 2), "unit": "GB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic", "config": {"workload": f"{lens.size} objects, {total} bytes",
                                        "credited_bytes": credited},
        "roofline": {"bound": "hbm", "kernel": "k_entries",
                     "achieved": round(achieved, 1) if achieved else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": None, "scan_ms_per_step": round(scan_s * 1e3, 4)},
        "bit_exact_vs_oracle": ok,
    }


def run_host():
    """The synchronous host path Crc32C::update now calls (no GPU), timed
    beside the reference's own intelCrc32C (oracle/_ref, the CPU baseline) by
    tools/bin/host_bench in the shape of src/misc/crc32c.cc:57-104."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "bin", "host_bench")
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_crc32c.so")
    if not os.path.exists(exe):
        raise RuntimeError("tools/bin/host_bench not built (make -C tools)")
    out = subprocess.run([exe, ref], capture_output=True, text=True, check=True).stdout
    rows = [json.loads(x) for x in out.splitlines() if x.strip()]
    summary = rows[-1]
    table = {r["bytes"]: r for r in rows[:-1]}
    pick = [1, 8, 64, 100, 128, 1024, 4096, 65536, 1 << 20, 8 << 20, 16 << 20]
    big = table[8 << 20]
    return {
        "metric": "host Crc32C::update MB/s (drop-in SSE4.2 path vs reference intelCrc32C)",
        "value": big["ramcrc_hw_MBps"], "unit": "MB/s (2^20 B/s)", "n_gpus": 0,
        "higher_is_better": True, "dtype": "u8", "data": "synthetic (xorshift bytes)",
        "config": {"workload": "one update per run, sizes as src/misc/crc32c.cc:97-104; value at 8 MiB"},
        "cpu_baseline": {"value": big["reference_intelCrc32C_MBps"], "unit": "MB/s", "cores": 1,
                         "kind": "reference" if summary["reference_loaded"] else "none",
                         "sample": "same buffer, same sizes, RAMCloud intelCrc32C (src/Crc32C.h:39-93)"},
        "by_size": {str(n): [table[n]["ramcrc_hw_MBps"], table[n]["ramcrc_sw_MBps"],
                             table[n]["reference_intelCrc32C_MBps"]] for n in pick},
        "by_size_columns": ["ramcrc_hw", "ramcrc_sw", "reference_intelCrc32C"],
        "bit_exact_vs_reference": summary["mismatches"] == 0,
    }


def replay_cpu_baseline(host, seg_bytes, certs, nsample):
    """The restated reference walk + per-object verify (oracle, SSE4.2 CRC) on
    nsample segments, one thread -- the checksum work of one
    RecoverSegmentBenchmark replay thread."""
    from oracle import oracle
    t0 = time.perf_counter()
    bad = 0
    for i in range(nsample):
        seg = host[i * seg_bytes:(i + 1) * seg_bytes]
        f, ck, n, table = oracle.check_metadata(seg, int(certs[i, 0]), int(certs[i, 1]),
                                                segment=0, table_cap=seg_bytes // 36 + 1)
        b, _, _ = oracle.verify_objects(seg, seg_bytes, table, 1)
        bad += b + (0 if f == 1 else 1)
    dt = time.perf_counter() - t0
    return {"value": round(nsample * seg_bytes / dt / 1e9, 3), "unit": "GB/s", "cores": 1,
            "kind": "port",
            "sample": f"{nsample} x {seg_bytes // MiB} MiB object segments, oracle restatement of "
                      "Segment::checkMetadataIntegrity + Object::computeChecksum, 1 thread",
            "all_verified": bad == 0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="segments",
                    choices=["segments", "recovery", "entries", "stream", "replay", "append",
                             "host"])
    ap.add_argument("--nseg", type=int, default=1024, help="segments per GPU (weak scaling)")
    ap.add_argument("--nseg-total", type=int, default=2048, help="recovery config: total segments")
    ap.add_argument("--seg-mib", type=int, default=8)
    ap.add_argument("--entries", type=int, default=1_000_000)
    ap.add_argument("--path", default="entries", choices=["entries", "batch"])
    ap.add_argument("--entry-size", type=int, default=0, help="fixed entry length (default: Zipf mix)")
    ap.add_argument("--replay-nseg", type=int, default=512,
                    help="replay config: segments (RecoverSegmentBenchmark: 4096/8)")
    ap.add_argument("--value-len", type=int, default=1024, help="replay config: object value bytes")
    ap.add_argument("--cpu-sample", type=int, default=128, help="segments timed on the CPU")
    ap.add_argument("--replay-cpu-sample", type=int, default=16,
                    help="replay config: segments verified by the CPU baseline")
    ap.add_argument("--walk-cus", type=int, default=0,
                    help="replay config: pipeline batches, walking on this many CUs "
                         "(a multiple of 8) beside the object scan on the rest; 0 = serial")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ramcrc.lib()  # fail loudly if the HIP library is missing
    if args.config == "host":
        print(json.dumps(run_host()), flush=True)
        return
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    ctx = ramcrc.Context(local_rank)

    if args.config in ("segments", "recovery"):
        r = run_segments(args, rank, world, local_rank, ctx)
        total_bytes = r["nseg_total"] * r["seg_bytes"] * args.steps
        value = total_bytes / r["elapsed"] / 1e9
        avg_scan_s = r["scan_ms"] / max(r["launches"], 1) / 1e3
        bytes_per_launch = r["nseg"] * r["seg_bytes"]
        achieved = bytes_per_launch / avg_scan_s / 1e9 if avg_scan_s > 0 else None
        # correctness of this run: known answers for the first segments
        kat_ok = None
        if rank == 0 and r["first_seed"] == workloads.SEGMENT_SEED:
            with open(os.path.join(ROOT, "tests", "golden", "crc32c_golden.json")) as f:
                kats = {k["name"]: k["crc"] for k in json.load(f)["kat"] if "crc" in k}
            kat_ok = all(int(r["local_crcs"][i]) == kats[f"bench_segment_{i}"]
                         for i in range(min(4, r["nseg"])))
        line = None
        if rank == 0:
            cpu = None
            if world == 1 and not args.no_cpu_baseline:
                ns = min(args.cpu_sample, r["nseg"])
                sample = r["data"][: ns * r["seg_bytes"]].cpu().numpy()
                cpu = cpu_baseline(sample, r["seg_bytes"], ns, r["local_crcs"][:ns])
            line = {
                "metric": METRIC,
                "value": round(value, 2),
                "unit": "GB/s",
                "n_gpus": world,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": round(r["elapsed"] / args.steps * 1e3, 4),
                "higher_is_better": True,
                "scaling": r["scaling"],
                "vs_baseline": None,
                "dtype": "u8",
                "data": "synthetic (splitmix64 bytes, seed 0x52414D43+i per segment)",
                "config": {
                    "workload": ("recovery scan: %d x %d MiB segments sharded over %d GPUs"
                                 % (r["nseg_total"], args.seg_mib, world))
                    if args.config == "recovery" else
                    ("%d x %d MiB device-resident segments per GPU (BASELINE config 2)"
                     % (r["nseg"], args.seg_mib)),
                    "segments_per_gpu": r["nseg"],
                    "segment_bytes": r["seg_bytes"],
                    "batch_bytes_per_gpu": r["nseg"] * r["seg_bytes"],
                    "parallelism": f"shard{world}" if world > 1 else "single",
                    "exchange": "rccl all_gather of uint32 CRCs" if world > 1 else "none",
                },
                "roofline": {
                    "bound": "hbm",
                    "kernel": "k_chunks",
                    "achieved": round(achieved, 1) if achieved else None,
                    "peak": HBM_PEAK_GBS,
                    "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                    "traffic": load_traffic("k_chunks"),
                    "avg_kernel_ms": round(avg_scan_s * 1e3, 4),
                    "algorithmic_bytes_per_launch": bytes_per_launch,
                },
                "cpu_baseline": cpu,
                "bit_exact_kat": kat_ok,
            }
    elif args.config == "entries":
        r = run_entries(args, ctx, world)
        value = world * r["total"] * args.steps / r["elapsed"] / 1e9
        # scan kernels bracketed per call (k_entries; k_chunks + k_entries on the batch path)
        scan_s_per_step = r["scan_ms"] / args.steps / 1e3
        achieved = r["total"] / scan_s_per_step / 1e9 if scan_s_per_step > 0 else None
        from oracle import oracle
        ok = (bool(np.array_equal(r["crcs"], oracle.entries(r["host"], r["offs"], r["lens"])))
              if rank == 0 else None)
        line = {
            "metric": "device-resident CRC32C GB/s over 1M mixed log entries (100B/1KiB/4KiB Zipf)",
            "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(r["elapsed"] / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic", "config": {"workload": f"{r['n']} entries, {r['total']} bytes per GPU",
                                            "path": args.path,
                                            "parallelism": f"replicas{world}" if world > 1 else "single",
                                            "exchange": "none"},
            "roofline": {"bound": "hbm", "kernel": "k_entries" if args.path == "entries" else "k_chunks+k_entries",
                         "achieved": round(achieved, 1) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                         "traffic": load_traffic("entries_scan") if args.path == "entries" else None,
                         "scan_ms_per_step": round(scan_s_per_step * 1e3, 4)},
            "bit_exact_vs_oracle": ok,
        }
    elif args.config == "replay":
        from ramcloud_amd import segments
        r = run_replay(args, ctx)
        seg_total = r["nseg"] * r["seg_bytes"]
        value = seg_total * args.steps / r["elapsed"] / 1e9
        obj_bytes = int(r["counts"].sum()) * (segments.OBJECT_OVERHEAD + args.value_len - 4)
        scan_s_per_step = r["scan_ms"] / args.steps / 1e3
        achieved = obj_bytes / scan_s_per_step / 1e9 if scan_s_per_step > 0 else None
        cpu = None if args.no_cpu_baseline else replay_cpu_baseline(
            r["host"], r["seg_bytes"], r["certs"], min(args.replay_cpu_sample, r["nseg"]))
        line = {
            "metric": "device-resident recovery replay verify GB/s of 8 MiB object segments "
                      "(segment walk + per-object checksum compare)",
            "value": round(value, 2), "unit": "GB/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(r["elapsed"] / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (RecoverSegmentBenchmark-shaped objects, splitmix64 values)",
            "config": {"workload": f"{r['nseg']} x {args.seg_mib} MiB segments of "
                                   f"{args.value_len} B-value objects",
                       "pipeline": (f"walk on {args.walk_cus} CUs beside the scan of the previous batch"
                                    if args.walk_cus else "none"),
                       "objects": int(r["counts"].sum()), "object_bytes_checksummed": obj_bytes},
            "roofline": {"bound": "hbm", "kernel": "k_entries (object verify)",
                         "achieved": round(achieved, 1) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                         "traffic": None, "scan_ms_per_step": round(scan_s_per_step * 1e3, 4)},
            "cpu_baseline": cpu,
            "all_segments_verified": r["ok"],
        }
    elif args.config == "append":
        line = run_append(args, ctx)
    else:  # stream (config 5): host-to-host
        seg_bytes = args.seg_mib * MiB
        nseg = args.nseg
        host = torch.empty(nseg * seg_bytes, dtype=torch.uint8).pin_memory()
        dev = torch.empty(nseg * seg_bytes, dtype=torch.uint8, device="cuda")
        workloads.splitmix_fill_segments(dev, seg_bytes, workloads.SEGMENT_SEED)
        host.copy_(dev)
        del dev
        torch.cuda.synchronize()
        out = ctx.stream_host(host, seg_bytes, nseg)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = ctx.stream_host(host, seg_bytes, nseg, batch=8, depth=3)
        elapsed = time.perf_counter() - t0
        value = nseg * seg_bytes * args.steps / elapsed / 1e9
        line = {"metric": "host-to-host streamed CRC32C GB/s (pinned H2D overlapped)",
                "value": round(value, 2), "unit": "GB/s", "n_gpus": 1, "steps": args.steps,
                "warmup": 1, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
                "data": "synthetic", "config": {"workload": f"{nseg} x {args.seg_mib} MiB pinned host segments"},
                "first_crc": int(out[0])}

    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
