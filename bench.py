"""Benchmark of RAMCloud's CRC32C integrity-checksum path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--config segments|recovery|entries|stream|replay|append|host]

Default (--config segments):
  N = 1  BASELINE config 2: 1024 x 8 MiB segments resident in HBM, one step =
         ramcrc_segments_device over the whole 8 GiB batch (the recovery-scan
         batch, src/BackupMasterRecovery.cc:743-809).
  N > 1  BASELINE config 4, strong scaling: 2048 x 8 MiB
         RecoverSegmentBenchmark-shaped object segments
         (nanobenchmarks/RecoverSegmentBenchmark.cc:123-146) sharded over N
         GPUs, one step = every rank scans its contiguous range + one RCCL
         all-gather of the uint32 CRCs (the C-ABI shard entry, ramcrc_shard_*).
         Rank 0 also times the whole 2048-segment batch alone on its GPU
         (t1) and reports t1 / tN.
  `python bench.py --gpus N` with no launcher around it starts N ranks
  itself (torch.distributed.run, 127.0.0.1) from a process that has made no
  GPU call; under a launcher WORLD_SIZE must equal N.

Rank 0 prints one JSON line.  `roofline` prices the dominant kernel from its
HIP-event duration on its launch stream; `traffic` is the corrected PMC
FETCH_SIZE of that kernel measured on this exact workload (profiles/pmc/),
or null when no such profile exists.  `cpu_baseline` (N = 1) times the
reference's compiled intelCrc32C (oracle/_ref) -- or the oracle restatement
when _ref was not shipped -- over the same 8 GiB batch on this host's cores
(1 thread and T = min(physical cores, cgroup CPU quota) threads, best and
median of 5) and checks every GPU CRC against it.

--host-dry-run runs the N-rank launcher, sharding, host segment fill and the
result all-gather on the CPU (gloo, libramcrc's host CRC path, no GPU): the
CPU test of the multi-GPU plumbing.  Its numbers are not GPU measurements.
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MiB = 1 << 20
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "device-resident CRC32C GB/s over 8MiB-segment batch; % of HBM roofline"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------ launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """Start n ranks of this script (one process per GPU) and return the
    launcher's exit code.  Runs before anything touches the GPU; the ranks are
    child processes (no exec), each reading RANK/LOCAL_RANK/WORLD_SIZE."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------- host facts
def host_cpu_info():
    """Logical CPUs, physical cores, sockets, model and the cgroup CPU quota
    (cpu.max) of this host."""
    info = {"logical": os.cpu_count() or 1}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = info["logical"]
    cores, sockets, model = set(), set(), None
    try:
        phys = core = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "physical id":
                    phys = v
                elif k == "core id":
                    core = v
                elif k == "model name" and model is None:
                    model = v
                elif not k and phys is not None:
                    cores.add((phys, core))
                    sockets.add(phys)
                    phys = core = None
        if phys is not None:
            cores.add((phys, core))
            sockets.add(phys)
    except OSError:
        pass
    info["physical_cores"] = len(cores) or info["logical"]
    info["sockets"] = len(sockets) or 1
    info["model"] = model
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    info["cgroup_cpu_quota"] = quota
    return info


def baseline_threads(info):
    t = min(info["physical_cores"], info["affinity"])
    if info["cgroup_cpu_quota"]:
        t = min(t, max(1, int(info["cgroup_cpu_quota"])))
    return max(1, t)


# --------------------------------------------------------------- PMC traffic
def traffic_for(key):
    """Corrected HBM read bytes per launch of the dominant kernel, measured by
    rocprofv3 --pmc FETCH_SIZE on exactly this workload (profiles/pmc/<key>.json,
    written by tools/pmc_traffic.py), or (None, None)."""
    p = os.path.join(ROOT, "profiles", "pmc", key + ".json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d["hbm_read_bytes_per_launch"], os.path.relpath(p, ROOT)
    except (OSError, KeyError, ValueError):
        return None, None


def roofline(kernel, algo_bytes, kernel_ms, traffic_key):
    achieved = algo_bytes / (kernel_ms / 1e3) / 1e9 if kernel_ms > 0 else None
    traffic, src = traffic_for(traffic_key)
    return {"bound": "hbm", "kernel": kernel,
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "traffic": traffic, "traffic_source": src,
            "avg_kernel_ms": round(kernel_ms, 4),
            "algorithmic_bytes_per_launch": algo_bytes, "traffic_key": traffic_key}


# ------------------------------------------------------------ distributed
class Ranks:
    """RANK/LOCAL_RANK/WORLD_SIZE of this process and the torch.distributed
    group for barriers, max-over-ranks timing and small host objects."""

    def __init__(self, backend):
        import torch.distributed as dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = dist
        self.backend = backend
        if self.world > 1:
            if backend == "nccl":
                import torch
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            else:
                dist.init_process_group("gloo")

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, x):
        if self.world == 1:
            return x
        import torch
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather_objects(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def broadcast_object(self, obj):
        if self.world == 1:
            return obj
        box = [obj]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def timed(steps, warmup, step, sync, ranks, on_start=None):
    """W untimed steps, then exactly K steps bracketed by sync + barrier on
    both sides; returns the slowest rank's seconds.  on_start() runs between
    the warmup and the timed steps (to reset kernel timers)."""
    for _ in range(warmup):
        step()
    sync()
    if on_start:
        on_start()
    ranks.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    ranks.barrier()
    return ranks.max(time.perf_counter() - t0)


# -------------------------------------------------------------- CPU baselines
def cpu_baseline_segments(host, seg_bytes, nseg, gpu_crcs, reps=5):
    """The reference's intelCrc32C (src/Crc32C.h:39-93; oracle/_ref, compiled
    from /root/reference) over the whole batch, 1 thread and T threads taking
    whole segments round-robin (RecoverSegmentBenchmark's pool,
    nanobenchmarks/RecoverSegmentBenchmark.cc:90-118), pinned; best and median
    of `reps`.  Also the bit-exact check of every GPU CRC."""
    from oracle import oracle
    use_ref = oracle.ref_available()
    info = host_cpu_info()
    threads = baseline_threads(info)
    res = {}
    crcs = None
    for t in sorted({1, threads}):
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            crcs = oracle.segments(host, seg_bytes, nseg, threads=t, use_ref=use_ref)
            times.append(time.perf_counter() - t0)
        res[t] = (nseg * seg_bytes / min(times) / 1e9, nseg * seg_bytes / statistics.median(times) / 1e9)
    ok = bool(np.array_equal(crcs, gpu_crcs))
    best, median = res[threads]
    return {
        "value": round(best, 3), "unit": "GB/s", "cores": threads,
        "kind": "reference" if use_ref else "port",
        "sample": (f"the whole batch: {nseg} x {seg_bytes // MiB} MiB, best of {reps} "
                   f"(median {median:.3f} GB/s); "
                   + ("RAMCloud intelCrc32C (src/Crc32C.h:39-93) compiled -O3 -msse4.2 from the reference"
                      if use_ref else "oracle restatement of intelCrc32C")
                   + "; whole segments round-robin over pinned threads"),
        "median": round(median, 3),
        "single_thread_GBs": round(res[1][0], 3),
        "single_thread_median_GBs": round(res[1][1], 3),
        "threads_rule": "min(physical cores, affinity, cgroup cpu.max quota)",
        "host": info,
        "bit_exact_vs_gpu": ok,
    }


def cpu_baseline_entries(host, offs, lens, gpu_crcs, reps=5):
    """The reference's own intelCrc32C (src/Crc32C.h:39-93; oracle/_ref) once
    per entry -- the reference's loop of one Crc32C per log entry / object
    (src/ObjectManager.cc:659-669, src/Object.cc:805-819) -- 1 thread and T
    threads (blocks of 4096 entries round-robin over pinned threads), best and
    median of `reps`; the oracle restatement on 1 thread when oracle/_ref was
    not built.  Also the bit-exact check of every GPU CRC."""
    from oracle import oracle
    use_ref = oracle.ref_available()
    info = host_cpu_info()
    threads = baseline_threads(info) if use_ref else 1
    total = int(lens.sum())
    res, want = {}, None
    for t in sorted({1, threads}):
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            want = (oracle.ref_entries(host, offs, lens, threads=t) if use_ref
                    else oracle.entries(host, offs, lens))
            times.append(time.perf_counter() - t0)
        res[t] = (total / min(times) / 1e9, total / statistics.median(times) / 1e9)
    best, median = res[threads]
    return {"value": round(best, 3), "unit": "GB/s", "cores": threads,
            "kind": "reference" if use_ref else "port",
            "sample": (f"all {lens.size} entries ({total} B), one Crc32C per entry, best of {reps} "
                       f"(median {median:.3f} GB/s); "
                       + ("RAMCloud intelCrc32C (src/Crc32C.h:39-93) compiled -O3 -msse4.2 from the "
                          "reference, blocks of 4096 entries round-robin over pinned threads"
                          if use_ref else "oracle SSE4.2 restatement of intelCrc32C, 1 thread")),
            "median": round(median, 3),
            "single_thread_GBs": round(res[1][0], 3),
            "threads_rule": "min(physical cores, affinity, cgroup cpu.max quota)",
            "host": info,
            "bit_exact_vs_gpu": bool(np.array_equal(want, gpu_crcs))}


# ------------------------------------------------------------------ configs
def run_c2(args, ranks):
    """BASELINE config 2 on each rank's GPU (replicas when run by itself at N > 1
    with --config c2)."""
    import torch
    from ramcloud_amd import ramcrc, workloads
    ctx = ramcrc.Context(ranks.local)
    seg = args.seg_mib * MiB
    nseg = args.nseg
    data = torch.empty(nseg * seg, dtype=torch.uint8, device="cuda")
    workloads.splitmix_fill_segments(data, seg, workloads.SEGMENT_SEED)
    out = torch.zeros(nseg, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.set_timing(True)
    elapsed = timed(args.steps, args.warmup, lambda: ctx.segments(data, seg, nseg, out),
                    torch.cuda.synchronize, ranks, on_start=ctx.scan_time)
    kernel_ms, launches = ctx.scan_time()
    ctx.set_timing(False)
    avg_ms = kernel_ms / max(launches, 1)
    gpu = out.cpu().numpy().view(np.uint32)
    kat_ok = None
    if ranks.rank == 0:
        with open(os.path.join(ROOT, "tests", "golden", "crc32c_golden.json")) as f:
            kats = {k["name"]: k["crc"] for k in json.load(f)["kat"] if "crc" in k}
        kat_ok = all(int(gpu[i]) == kats[f"bench_segment_{i}"] for i in range(min(4, nseg)))
    line = None
    if ranks.rank == 0:
        cpu = None
        if ranks.world == 1 and not args.no_cpu_baseline:
            host = data.cpu().numpy()
            cpu = cpu_baseline_segments(host, seg, nseg, gpu, reps=args.cpu_reps)
        key = f"c2_{nseg}x{args.seg_mib}MiB_k_chunks"
        line = {
            "metric": METRIC,
            "value": round(ranks.world * nseg * seg * args.steps / elapsed / 1e9, 2),
            "unit": "GB/s", "n_gpus": ranks.world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if ranks.world == 1 else "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (splitmix64 bytes, seed 0x52414D43+i per segment)",
            "config": {"workload": f"{nseg} x {args.seg_mib} MiB device-resident segments "
                                   "(BASELINE config 2)" + (" per GPU" if ranks.world > 1 else ""),
                       "segments_per_gpu": nseg, "segment_bytes": seg,
                       "batch_bytes_per_gpu": nseg * seg,
                       "parallelism": "single" if ranks.world == 1 else f"replicas{ranks.world}",
                       "exchange": "none"},
            "roofline": roofline("k_chunks", nseg * seg, avg_ms, key),
            "cpu_baseline": cpu,
            "bit_exact_kat": kat_ok,
        }
        if ranks.world == 1:
            line["scaling_note"] = ("N=1 runs BASELINE config 2 (1024 segments); N>1 runs config 4 "
                                    "(2048 segments sharded, strong scaling); value is GB/s in both")
    ctx.close()
    return line


def _fill_recovery_shard(ctx, data, seg, lo, count, value_len, certs=None):
    """Segments lo .. lo+count-1 of the C4 batch: splitmix64 value bytes (seed
    0x52414D43 + i), then RecoverSegmentBenchmark's objects with keys
    continuing across segments (first key of segment i = i * per), built on
    the device (ramcrc_segment_fill_objects_device).  Returns (objects per
    segment, certificate length, certificate checksum)."""
    from ramcloud_amd import segments, workloads
    per = segments.objects_per_segment(seg, value_len)
    if count:
        workloads.splitmix_fill_segments(data, seg, workloads.SEGMENT_SEED + lo)
    got, length, ck = ctx.fill_objects(data, seg, seg, count, value_len, first_key=lo * per,
                                       certs=certs)
    assert got == per, (got, per)
    return per, length, ck


def run_recovery(args, ranks):
    """BASELINE config 4: the recovery-scan shard, strong scaling."""
    import torch
    from ramcloud_amd import ramcrc
    seg = args.seg_mib * MiB
    total = args.nseg_total
    lo, hi = ramcrc.shard_range(total, ranks.world, ranks.rank)
    count = hi - lo
    setup = ramcrc.Context(ranks.local)
    data = torch.empty(max(count, 1) * seg, dtype=torch.uint8, device="cuda")
    per, _, _ = _fill_recovery_shard(setup, data, seg, lo, count, args.value_len)
    uid = ranks.broadcast_object(ramcrc.shard_unique_id() if ranks.rank == 0 else None)
    shard = ramcrc.Shard(uid=uid, nranks=ranks.world, rank=ranks.rank, device=ranks.local)
    out = torch.zeros(total, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    shard.set_timing(True)

    def sync():
        shard.sync()
        torch.cuda.synchronize()

    elapsed = timed(args.steps, args.warmup, lambda: shard.segments([data], seg, total, outs=[out]),
                    sync, ranks, on_start=shard.scan_time)
    kernel_ms, launches = shard.scan_time()
    shard.set_timing(False)
    avg_ms = kernel_ms / max(launches, 1)
    gathered = out.cpu().numpy().view(np.uint32)
    # Full check of the gathered batch on every rank: each rank CRCs its own
    # segments on the host (libramcrc's SSE4.2 path, independent of the
    # kernels), the per-rank lists are exchanged, and every rank compares all
    # `total` gathered CRCs with them.
    mine = _host_segment_crcs(data, seg, count)
    expect = np.zeros(total, np.uint32)
    for q_lo, q_crcs in ranks.gather_objects((lo, mine.tobytes())):
        q = np.frombuffer(q_crcs, np.uint32)
        expect[q_lo:q_lo + q.size] = q
    bad = int((gathered != expect).sum())
    bad_per_rank = ranks.gather_objects(bad)
    shard.close()
    # The reference's CPU path beside the GPU line, at every N (rank 0, outside
    # the timed region): intelCrc32C over the whole batch on this host's cores.
    cpu = None
    if ranks.rank == 0 and ranks.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_segments(data.cpu().numpy(), seg, total, gathered, reps=args.cpu_reps)
    del data
    torch.cuda.empty_cache()
    ranks.barrier()
    t1 = None
    if ranks.rank == 0 and ranks.world > 1 and not (args.no_t1 and args.no_cpu_baseline):
        t1, cpu = _recovery_t1(args, ranks, setup, gathered)
    ranks.barrier()
    setup.close()
    if ranks.rank != 0:
        return None
    tn_ms = elapsed / args.steps * 1e3
    key = f"c4_{total}x{args.seg_mib}MiB_v{args.value_len}_n{ranks.world}_k_chunks"
    line = {
        "metric": METRIC,
        "value": round(total * seg * args.steps / elapsed / 1e9, 2),
        "unit": "GB/s", "n_gpus": ranks.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(tn_ms, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u8",
        "data": ("synthetic RecoverSegmentBenchmark-shaped object segments "
                 f"({per} objects of {args.value_len} B values per segment, splitmix64 value "
                 "bytes seed 0x52414D43+i, keys continuing across segments)"),
        "config": {"workload": f"recovery scan (BASELINE config 4): {total} x {args.seg_mib} MiB "
                               f"segments sharded over {ranks.world} GPUs",
                   "segments_total": total, "segments_per_gpu_max": (total + ranks.world - 1) // ranks.world,
                   "segment_bytes": seg, "parallelism": f"shard{ranks.world}",
                   "exchange": "RCCL ncclAllGather of uint32 CRCs (libramcrc ramcrc_shard_segments)"},
        "roofline": roofline("k_chunks", count * seg, avg_ms, key),
        "cpu_baseline": cpu,
        "bit_exact": all(b == 0 for b in bad_per_rank),
        "bit_exact_check": (f"all {total} gathered CRCs on each of the {ranks.world} ranks vs "
                            "each owner's host CRCs of its segments (libramcrc SSE4.2 path); "
                            f"mismatches per rank {bad_per_rank}"),
    }
    if t1 is not None:
        line["t1_ms"] = round(t1, 4)
        line["speedup_t1_over_tN"] = round(t1 / tn_ms, 3)
    return line


def _host_segment_crcs(data, seg, count, batch=32, threads=8):
    """Finalized CRCs of the `count` segments of a device tensor, through the
    host hardware CRC path, copied out `batch` segments at a time."""
    from concurrent.futures import ThreadPoolExecutor
    from ramcloud_amd import ramcrc
    out = np.zeros(count, np.uint32)
    with ThreadPoolExecutor(max_workers=threads) as ex:
        for j in range(0, count, batch):
            n = min(batch, count - j)
            host = data[j * seg:(j + n) * seg].cpu().numpy()
            out[j:j + n] = list(ex.map(lambda i: ramcrc.crc32c(host[i * seg:(i + 1) * seg]),
                                       range(n)))
    return out


def _recovery_t1(args, ranks, ctx, gathered):
    """The whole C4 batch built on rank 0's GPU: timed there alone (a 1-rank
    shard, same steps; unless --no-t1) and, unless --no-cpu-baseline, copied to
    the host for the reference CPU baseline, whose CRCs are compared with the
    N-rank step's gathered ones.  Returns (t1 ms or None, cpu_baseline or None)."""
    import torch
    from ramcloud_amd import ramcrc
    seg = args.seg_mib * MiB
    total = args.nseg_total
    data = torch.empty(total * seg, dtype=torch.uint8, device="cuda")
    _fill_recovery_shard(ctx, data, seg, 0, total, args.value_len)
    t1 = None
    if not args.no_t1:
        solo = ramcrc.Shard(uid=ramcrc.shard_unique_id(), nranks=1, rank=0, device=ranks.local)
        out = torch.zeros(total, dtype=torch.int32, device="cuda")
        step = lambda: solo.segments([data], seg, total, outs=[out])  # noqa: E731
        for _ in range(args.warmup):
            step()
        solo.sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        solo.sync()
        t1 = (time.perf_counter() - t0) / args.steps * 1e3
        solo.close()
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_baseline_segments(data.cpu().numpy(), seg, total, gathered, reps=args.cpu_reps)
    del data
    torch.cuda.empty_cache()
    return t1, cpu


def run_recovery_host_dry(args, ranks):
    """The N-rank plumbing of config 4 on the CPU: the same launcher, shard
    ranges, object fill (host append path) and result all-gather (gloo), with
    libramcrc's host CRC path as the per-segment scan.  No GPU numbers."""
    import torch
    from ramcloud_amd import ramcrc, segments, workloads
    from ramcloud_amd.recovery_scan import RecoveryScan
    seg = args.seg_kib * 1024 if args.seg_kib else args.seg_mib * MiB
    total = args.nseg_total
    per = segments.objects_per_segment(seg, args.value_len)

    def scan_fn(shard, seg_bytes, count, out):
        a = shard.numpy()
        for j in range(count):
            out[j] = int(np.uint32(ramcrc.crc32c(a[j * seg_bytes:(j + 1) * seg_bytes])).view(np.int32))

    scan = RecoveryScan(total, seg, ranks.rank, ranks.world, scan_fn=scan_fn)
    shard = torch.empty(max(scan.count, 1) * seg, dtype=torch.uint8)
    a = shard.numpy()
    for i in range(scan.lo, scan.hi):
        s = a[(i - scan.lo) * seg:(i - scan.lo + 1) * seg]
        s[:] = workloads.splitmix_bytes_np(workloads.SEGMENT_SEED + i, seg)
        ramcrc.segment_fill_objects(s, args.value_len, first_key=i * per)
    out = torch.zeros(max(scan.count, 1), dtype=torch.int32)
    box = {}

    def step():
        box["full"] = scan.step(shard, out)

    elapsed = timed(args.steps, args.warmup, step, lambda: None, ranks)
    if ranks.rank != 0:
        return None
    crcs = box["full"].numpy().view(np.uint32)
    cpu = None
    if not args.no_cpu_baseline:
        # as the GPU line: the reference's CPU path over the whole batch, rank 0
        full = np.empty(total * seg, np.uint8)
        for i in range(total):
            s = full[i * seg:(i + 1) * seg]
            s[:] = workloads.splitmix_bytes_np(workloads.SEGMENT_SEED + i, seg)
            ramcrc.segment_fill_objects(s, args.value_len, first_key=i * per)
        cpu = cpu_baseline_segments(full, seg, total, crcs, reps=args.cpu_reps)
    return {
        "metric": METRIC + " [host dry run: CPU plumbing test, not a GPU measurement]",
        "value": round(total * seg * args.steps / elapsed / 1e9, 4), "unit": "GB/s",
        "n_gpus": ranks.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic RecoverSegmentBenchmark-shaped object segments (host dry run)",
        "config": {"workload": f"recovery scan: {total} x {seg} B segments sharded over "
                               f"{ranks.world} ranks", "segments_total": total,
                   "segment_bytes": seg, "value_len": args.value_len,
                   "parallelism": f"shard{ranks.world}", "exchange": "gloo all_gather (dry run)"},
        "dry_run": True,
        "cpu_baseline": cpu,
        "crcs": [int(c) for c in crcs] if total <= 256 else None,
        "crc_of_crcs": ramcrc.crc32c(np.ascontiguousarray(crcs)),
    }


def run_entries(args, ranks):
    """Config 3: 1 M mixed log entries; replicas at N > 1."""
    import torch
    from ramcloud_amd import ramcrc, workloads
    ctx = ramcrc.Context(ranks.local)
    lens = workloads.entry_lengths(args.entries)
    if args.entry_size:
        lens = lens * 0 + np.uint64(args.entry_size)
    if args.exclude_size:   # A/B: the mix without one of its sizes
        lens = lens[lens != np.uint64(args.exclude_size)]
    offs = workloads.packed_offsets(lens)
    total = int(lens.sum())
    data = torch.empty(((total + 7) // 8) * 8, dtype=torch.uint8, device="cuda")
    host = workloads.splitmix_bytes_np(workloads.ENTRY_SEED, total)
    data[:total].copy_(torch.from_numpy(host))
    off_t = torch.from_numpy(offs.view(np.int64)).cuda()
    len_t = torch.from_numpy(lens.view(np.int64)).cuda()
    out = torch.zeros(lens.size, dtype=torch.int32, device="cuda")
    fn = ctx.entries if args.path == "entries" else ctx.batch
    torch.cuda.synchronize()
    ctx.set_timing(True)
    elapsed = timed(args.steps, args.warmup, lambda: fn(data, off_t, len_t, out),
                    torch.cuda.synchronize, ranks, on_start=ctx.scan_time)
    kernel_ms, _ = ctx.scan_time()
    ctx.set_timing(False)
    ctx.check()
    if ranks.rank != 0:
        ctx.close()
        return None
    gpu = out.cpu().numpy().view(np.uint32)
    cpu = None if args.no_cpu_baseline else cpu_baseline_entries(host, offs, lens, gpu)
    scan_ms = kernel_ms / args.steps
    mix = "fixed %d B" % args.entry_size if args.entry_size else "100B/1KiB/4KiB Zipf"
    key = f"c3_{lens.size}_{'mix' if not args.entry_size else args.entry_size}_{args.path}"
    kernel = "k_entries (tiny + long phases)" if args.path == "entries" else "k_chunks+k_entries"
    ctx.close()
    return {
        "metric": f"device-resident CRC32C GB/s over {lens.size} log entries ({mix})",
        "value": round(ranks.world * total * args.steps / elapsed / 1e9, 2), "unit": "GB/s",
        "n_gpus": ranks.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"{lens.size} entries, {total} bytes per GPU (BASELINE config 3)",
                   "path": args.path,
                   "parallelism": f"replicas{ranks.world}" if ranks.world > 1 else "single",
                   "exchange": "none", "table_bytes_not_credited": 16 * lens.size},
        "roofline": dict(roofline(kernel, total, scan_ms, key),
                         scan_ms_per_step=round(scan_ms, 4)),
        "cpu_baseline": cpu,
    }


def replay_cpu_baseline(host, seg_bytes, certs, nsample, reps=3):
    """The checksum work of RecoverSegmentBenchmark's replay threads
    (nanobenchmarks/RecoverSegmentBenchmark.cc:90-118) on nsample segments:
    Segment::checkMetadataIntegrity (the oracle's restated walk) and the
    replaySegment checks of every record, every CRC byte through the
    reference's own intelCrc32C (oracle/_ref; the SSE4.2 restatement when it
    was not built), whole segments round-robin over 1 and T pinned threads,
    best and median of `reps`."""
    from oracle import oracle
    use_ref = oracle.ref_available()
    info = host_cpu_info()
    threads = baseline_threads(info)
    certs = np.ascontiguousarray(certs, dtype=np.uint32).reshape(-1, 2)
    res, failed = {}, None
    for t in sorted({1, threads}):
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            failed = oracle.replay_mt(host, seg_bytes, nsample, certs, threads=t, use_ref=use_ref)
            times.append(time.perf_counter() - t0)
        res[t] = (nsample * seg_bytes / min(times) / 1e9,
                  nsample * seg_bytes / statistics.median(times) / 1e9)
    best, median = res[threads]
    return {"value": round(best, 3), "unit": "GB/s", "cores": threads,
            "kind": "reference" if use_ref else "port",
            "sample": (f"{nsample} x {seg_bytes // MiB} MiB object segments, best of {reps} "
                       f"(median {median:.3f} GB/s): the oracle's restated walk "
                       "(Segment::checkMetadataIntegrity) + replaySegment checks, every CRC byte "
                       + ("through RAMCloud intelCrc32C (src/Crc32C.h:39-93) compiled from the reference"
                          if use_ref else "through the oracle's SSE4.2 restatement")
                       + ", whole segments round-robin over pinned threads"),
            "median": round(median, 3),
            "single_thread_GBs": round(res[1][0], 3),
            "threads_rule": "min(physical cores, affinity, cgroup cpu.max quota)",
            "host": info,
            "all_verified": failed == 0}


def replay_bit_exact(host, seg_bytes, certs, ns, table, obj_crc):
    """The GPU's walk records and object CRCs of the first ns segments against
    the oracle: records = the restated Segment::checkMetadataIntegrity walk
    (src/Segment.cc:758-800) of each segment, CRCs = the restated
    Object::computeChecksum (src/Object.cc:805-819) of those records."""
    from oracle import oracle
    certs = np.ascontiguousarray(certs, dtype=np.uint32).reshape(-1, 2)
    table = np.ascontiguousarray(table, dtype=np.uint32).reshape(-1, 4)
    mine = table[:, 0] < ns
    g_tab, g_crc = table[mine], obj_crc[mine]
    order = np.lexsort((g_tab[:, 1], g_tab[:, 0]))
    g_tab, g_crc = g_tab[order], g_crc[order]
    want = []
    for s in range(ns):
        _, _, _, t = oracle.check_metadata(host[s * seg_bytes:(s + 1) * seg_bytes], int(certs[s, 0]),
                                           int(certs[s, 1]), segment=s, capacity=seg_bytes)
        want.append(t)
    want = np.concatenate(want) if want else np.zeros((0, 4), np.uint32)
    records_ok = bool(np.array_equal(g_tab, want))
    _, crc, _ = oracle.verify_objects(host[:ns * seg_bytes], seg_bytes, want, ns)
    crcs_ok = records_ok and bool(np.array_equal(g_crc, crc))
    return {"segments": ns, "records": int(want.shape[0]), "records_match": records_ok,
            "object_crcs_match": crcs_ok}


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
    import torch
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
    if args.serial_walk:
        ctx_walk.set_serial_walk(True)
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
    for rv in rvs:
        rv.check()
    sts = [rv.status.clone() for rv in rvs]
    ctx.set_cus(0)
    ctx_walk.close()
    s_walk.destroy()
    s_scan.destroy()
    return elapsed, scan_ms, launches, sts


def run_replay(args, ranks):
    """Recovery replay verify (RecoverSegmentBenchmark-shaped,
    nanobenchmarks/RecoverSegmentBenchmark.cc:123-146): nseg 8 MiB segments
    full of objects with 8-byte counter keys and value_len-byte values; one
    step = Segment::checkMetadataIntegrity of every segment
    (src/Segment.cc:758-800) + Object::computeChecksum of every object
    compared with its stored checksum (src/ObjectManager.cc:659-669)."""
    import torch
    from ramcloud_amd import ramcrc, segments
    ctx = ramcrc.Context(ranks.local)
    ctx.set_option(ramcrc.OPT_VERIFY_IN_WALK, args.verify_in_walk)
    if args.serial_walk:
        ctx.set_serial_walk(True)
    if args.walk_part_shift:
        ctx.set_walk_part_shift(args.walk_part_shift)
    seg = args.seg_mib * MiB
    nseg = args.replay_nseg
    d = torch.empty(nseg * seg, dtype=torch.uint8, device="cuda")
    certs_t = torch.zeros((nseg, 2), dtype=torch.int32, device="cuda")
    per, _, _ = _fill_recovery_shard(ctx, d, seg, 0, nseg, args.value_len, certs=certs_t)
    certs = certs_t.cpu().numpy().view(np.uint32)
    counts = np.full(nseg, per, np.uint32)
    cap = int(counts.sum()) + nseg
    if args.walk_cus:
        elapsed, scan_ms, launches, sts = _replay_pipelined(args, ctx, d, certs_t, nseg, seg, cap)
    else:
        rv = segments.RecoveryVerify(ctx, nseg, seg, entries_cap=cap)
        torch.cuda.synchronize()
        ctx.set_timing(True)
        box = {}

        def step():
            box["st"] = rv.verify(d, certs_t)

        elapsed = timed(args.steps, args.warmup, step, torch.cuda.synchronize, ranks,
                        on_start=ctx.scan_time)
        scan_ms, launches = ctx.scan_time()
        ctx.set_timing(False)
        rv.check()
        sts = [box["st"]]
    ok = True
    for st in sts:
        status = st.cpu().numpy().view(np.uint32)
        ok = ok and bool((status[:, 0] == segments.SEG_OK).all() and (status[:, 3] == 0).all()
                         and np.array_equal(status[:, 2], counts)
                         and np.array_equal(status[:, 1], certs[:, 1]))
    obj_bytes = int(counts.sum()) * (segments.OBJECT_OVERHEAD + args.value_len - 4)
    cpu, exact = None, None
    if not args.no_cpu_baseline:
        ns = min(args.replay_cpu_sample, nseg)
        sample = d[:ns * seg].cpu().numpy()
        cpu = replay_cpu_baseline(sample, seg, certs, ns)
        if not args.walk_cus:
            n = int(rv.n_entries.item())
            exact = replay_bit_exact(sample, seg, certs, ns, rv.entries[:n].cpu().numpy().view(np.uint32),
                                     rv.obj_crc[:n].cpu().numpy().view(np.uint32))
            cpu["bit_exact_vs_gpu"] = exact["object_crcs_match"]
    ctx.close()
    scan_s = scan_ms / args.steps / 1e3
    achieved = obj_bytes / scan_s / 1e9 if scan_s > 0 else None
    # the object checks: k_entries, or k_walk_copyv in verify-in-walk mode
    # (the timer brackets both, the idle one exits at once: 5-10 us)
    tkey = f"replay_{nseg}x{args.seg_mib}MiB_v{args.value_len}_verify"
    return {
        "metric": "device-resident recovery replay verify GB/s of 8 MiB object segments "
                  "(segment walk + per-object checksum compare)",
        "value": round(nseg * seg * args.steps / elapsed / 1e9, 2), "unit": "GB/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (RecoverSegmentBenchmark-shaped objects, splitmix64 values)",
        "config": {"workload": f"{nseg} x {args.seg_mib} MiB segments of "
                               f"{args.value_len} B-value objects",
                   "pipeline": (f"walk on {args.walk_cus} CUs beside the scan of the previous batch"
                                if args.walk_cus else "none"),
                   "verify_in_walk": args.verify_in_walk,
                   "walk": ("serial (one wave per segment)" if args.serial_walk else
                            f"parallel ({1 << (args.walk_part_shift - 10)} KiB parts, forced)"
                            if args.walk_part_shift else
                            "parallel (part size from the entry density, k_walk_probe)"),
                   "objects": int(counts.sum()), "object_bytes_checksummed": obj_bytes},
        "roofline": {"bound": "hbm",
                     "kernel": "object verify (k_entries, or k_walk_copyv in verify-in-walk mode; "
                               "the launches of both summed)",
                     "achieved": round(achieved, 1) if achieved else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic_for(tkey)[0], "traffic_source": traffic_for(tkey)[1],
                     "scan_ms_per_step": round(scan_s * 1e3, 4),
                     "algorithmic_bytes_per_launch": obj_bytes, "traffic_key": tkey},
        "cpu_baseline": cpu,
        "all_segments_verified": ok,
        "bit_exact": None if exact is None else exact["object_crcs_match"],
        "bit_exact_check": exact,
    }


def run_contexts(args, ranks):
    """The reference's concurrency shape on one GPU: K replay (or log-entry)
    threads, as RecoverSegmentBenchmark sweeps replay threads {1, 2, 4, 8, 16}
    (nanobenchmarks/RecoverSegmentBenchmark.cc:181-183,273).  Each host thread
    owns one context and one stream (include/ramcrc.h: one context per
    launching thread) and its own copy of the batch, and submits a step per
    iteration back to back while the others run.  value = K x batch bytes x
    steps / wall time.  Every output of every context is checked: entries
    against the reference's intelCrc32C per entry, replay statuses and object
    CRCs against context 0's and context 0's first segments against the
    oracle's walk and checksums.  bin_rescues: k_bin_one launches of each
    context that aborted (grid not all resident in time) and were binned by
    the guarded scatter."""
    import threading
    import torch
    from ramcloud_amd import ramcrc, segments, workloads
    K = args.contexts
    dev = ranks.local
    ctxs = [ramcrc.Context(dev) for _ in range(K)]
    for c in ctxs:
        c.set_option(ramcrc.OPT_VERIFY_IN_WALK, args.verify_in_walk)
    streams = [torch.cuda.Stream() for _ in range(K)]
    if args.config == "entries":
        lens = workloads.entry_lengths(args.entries)
        if args.entry_size:
            lens = lens * 0 + np.uint64(args.entry_size)
        offs = workloads.packed_offsets(lens)
        total = int(lens.sum())
        host = workloads.splitmix_bytes_np(workloads.ENTRY_SEED, total)
        data0 = torch.from_numpy(host).cuda()
        off_t = torch.from_numpy(offs.view(np.int64)).cuda()
        len_t = torch.from_numpy(lens.view(np.int64)).cuda()
        datas = [data0] + [data0.clone() for _ in range(K - 1)]
        outs = [torch.zeros(lens.size, dtype=torch.int32, device="cuda") for _ in range(K)]
        step_bytes = total

        def step(i):
            ctxs[i].entries(datas[i], off_t, len_t, outs[i], stream=streams[i])
        what = f"{lens.size} log entries ({'fixed %d B' % args.entry_size if args.entry_size else '100B/1KiB/4KiB Zipf'})"
    else:
        seg = args.seg_mib * MiB
        nseg = args.replay_nseg
        d0 = torch.empty(nseg * seg, dtype=torch.uint8, device="cuda")
        certs_t = torch.zeros((nseg, 2), dtype=torch.int32, device="cuda")
        per, _, _ = _fill_recovery_shard(ctxs[0], d0, seg, 0, nseg, args.value_len, certs=certs_t)
        certs = certs_t.cpu().numpy().view(np.uint32)
        cap = per * nseg + nseg
        datas = [d0] + [d0.clone() for _ in range(K - 1)]
        rvs = [segments.RecoveryVerify(ctxs[i], nseg, seg, entries_cap=cap) for i in range(K)]
        step_bytes = nseg * seg
        sts = [None] * K

        def step(i):
            sts[i] = rvs[i].verify(datas[i], certs_t, stream=streams[i])
        what = f"{nseg} x {args.seg_mib} MiB segments of {args.value_len} B-value objects (replay verify)"
    torch.cuda.synchronize()
    go = threading.Barrier(K + 1)
    done = threading.Barrier(K + 1)
    errors = []

    def worker(i):
        try:
            torch.cuda.set_device(dev)
            for _ in range(args.warmup):
                step(i)
            streams[i].synchronize()
        except Exception as e:   # reported below; the barriers still release
            errors.append(repr(e))
        go.wait()
        try:
            for _ in range(args.steps):
                step(i)
            streams[i].synchronize()
        except Exception as e:
            errors.append(repr(e))
        done.wait()

    th = [threading.Thread(target=worker, args=(i,)) for i in range(K)]
    for t in th:
        t.start()
    go.wait()
    t0 = time.perf_counter()
    done.wait()
    elapsed = time.perf_counter() - t0
    for t in th:
        t.join()
    torch.cuda.synchronize()
    if errors:
        raise RuntimeError(f"context threads failed: {errors[:3]}")
    for c in ctxs:
        c.check()
    rescues = [c.bin_rescues() for c in ctxs]
    check = {}
    if args.config == "entries":
        from oracle import oracle
        want = (oracle.ref_entries(host, offs, lens, threads=baseline_threads(host_cpu_info()))
                if oracle.ref_available() else oracle.entries(host, offs, lens))
        check["all_crcs_match"] = all(
            bool(np.array_equal(o.cpu().numpy().view(np.uint32), want)) for o in outs)
        check["crcs_checked"] = int(lens.size) * K
    else:
        # segments take their record slots in the order their walks finish,
        # so tables are compared in (segment, offset) order
        def canon(rv):
            n = int(rv.n_entries.item())
            tab = rv.entries[:n].cpu().numpy().view(np.uint32)
            crc = rv.obj_crc[:n].cpu().numpy().view(np.uint32)
            o = np.lexsort((tab[:, 1], tab[:, 0]))
            return tab[o], crc[o]
        ok = True
        tab0, crc0 = canon(rvs[0])
        n0 = tab0.shape[0]
        for i in range(K):
            st = sts[i].cpu().numpy().view(np.uint32)
            ok = ok and bool((st[:, 0] == segments.SEG_OK).all() and (st[:, 3] == 0).all()
                             and (st[:, 2] == per).all() and np.array_equal(st[:, 1], certs[:, 1]))
            if i:
                tab, crc = canon(rvs[i])
                ok = ok and np.array_equal(tab, tab0) and np.array_equal(crc, crc0)
        ns = min(8, nseg)
        ex = replay_bit_exact(datas[0][:ns * seg].cpu().numpy(), seg, certs, ns, tab0, crc0)
        check = {"all_contexts_equal_and_verified": ok, "oracle_sample": ex,
                 "all_crcs_match": ok and ex["object_crcs_match"], "crcs_checked": n0 * K}
    for c in ctxs:
        c.close()
    return {
        "metric": f"aggregate device-resident CRC32C GB/s, {K} concurrent contexts on one GPU: {what}",
        "value": round(K * step_bytes * args.steps / elapsed / 1e9, 2), "unit": "GB/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": what, "contexts": K, "threads": K,
                   "per_context": "own context, stream and copy of the batch; steps back to back"},
        "bin_rescues": rescues, "check": check, "bit_exact": check["all_crcs_match"],
    }


def run_append(args, ranks):
    """Batched write-path checksum: Object::assembleForLog
    (src/Object.cc:213-238) over a batch of 1M serialized objects of the
    config-3 sizes (100 B / 1 KiB / 4 KiB, Zipf), packed back to back in HBM;
    one step = every header.checksum computed and stamped."""
    import torch
    from ramcloud_amd import ramcrc, workloads
    ctx = ramcrc.Context(ranks.local)
    lens = workloads.entry_lengths(args.entries)
    offs = workloads.packed_offsets(lens)
    total = int(lens.sum())
    host = workloads.splitmix_bytes_np(workloads.ENTRY_SEED, total)
    data = torch.from_numpy(host).cuda()
    off_t = torch.from_numpy(offs.view(np.int64)).cuda()
    len_t = torch.from_numpy(lens.view(np.int64)).cuda()
    out = torch.zeros(lens.size, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.set_timing(True)
    elapsed = timed(args.steps, args.warmup,
                    lambda: ctx.assemble_objects(data, off_t, len_t, out),
                    torch.cuda.synchronize, ranks, on_start=ctx.scan_time)
    scan_ms, _ = ctx.scan_time()
    ctx.set_timing(False)
    ctx.check()
    credited = total - 4 * lens.size   # bytes [4, len) of every object
    got = out.cpu().numpy().view(np.uint32)
    stamped = data.cpu().numpy()
    hdr = stamped[(offs.astype(np.int64)[:, None] + np.arange(4)).reshape(-1)].reshape(-1, 4).copy().view("<u4")[:, 0]
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_baseline_entries(host, offs + 4, lens - 4, got, reps=1)
        cpu["stamped_headers_match"] = bool(np.array_equal(hdr, got))
        cpu["sample"] += " (object bytes [4, len))"
    ctx.close()
    scan_s = scan_ms / args.steps / 1e3
    return {
        "metric": "device-resident Object::assembleForLog checksum GB/s over 1M objects "
                  "(100B/1KiB/4KiB Zipf)",
        "value": round(credited * args.steps / elapsed / 1e9, 2), "unit": "GB/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"{lens.size} objects, {total} bytes", "credited_bytes": credited},
        "roofline": dict(roofline("k_entries", credited, scan_s * 1e3, f"append_{lens.size}_mix"),
                         scan_ms_per_step=round(scan_s * 1e3, 4)),
        "cpu_baseline": cpu,
    }


def run_stream(args, ranks):
    """Config 5: pinned host segments streamed through the GPU (H2D on a copy
    stream overlapped with the kernels), CRCs back to host: host-to-host."""
    import torch
    from ramcloud_amd import ramcrc, workloads
    ctx = ramcrc.Context(ranks.local)
    seg = args.seg_mib * MiB
    nseg = args.nseg
    host = torch.empty(nseg * seg, dtype=torch.uint8).pin_memory()
    dev = torch.empty(nseg * seg, dtype=torch.uint8, device="cuda")
    workloads.splitmix_fill_segments(dev, seg, workloads.SEGMENT_SEED)
    host.copy_(dev)
    del dev
    torch.cuda.synchronize()
    box = {}

    def step():
        box["out"] = ctx.stream_host(host, seg, nseg, batch=8, depth=3)

    elapsed = timed(args.steps, 1, step, lambda: None, ranks)
    out = box["out"]
    a = host.numpy()
    spot = all(int(out[i]) == ramcrc.crc32c(a[i * seg:(i + 1) * seg]) for i in range(min(4, nseg)))
    ctx.close()
    return {"metric": "host-to-host streamed CRC32C GB/s (pinned H2D overlapped)",
            "value": round(nseg * seg * args.steps / elapsed / 1e9, 2), "unit": "GB/s",
            "n_gpus": 1, "steps": args.steps, "warmup": 1,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"{nseg} x {args.seg_mib} MiB pinned host segments"},
            "bit_exact_spot_check_host_path": bool(spot)}


def run_host():
    """The synchronous host path Crc32C::update now calls (no GPU), timed
    beside the reference's own intelCrc32C (oracle/_ref, the CPU baseline) by
    tools/bin/host_bench in the shape of src/misc/crc32c.cc:57-104."""
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


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks); default WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="segments",
                    choices=["segments", "c2", "recovery", "entries", "stream", "replay", "append",
                             "host"],
                    help="segments: config 2 at N=1, config 4 (recovery) at N>1")
    ap.add_argument("--nseg", type=int, default=1024, help="config 2/5: segments per GPU")
    ap.add_argument("--nseg-total", type=int, default=2048, help="config 4: segments in the batch")
    ap.add_argument("--seg-mib", type=int, default=8)
    ap.add_argument("--seg-kib", type=int, default=0, help="--host-dry-run: segment KiB")
    ap.add_argument("--value-len", type=int, default=1024,
                    help="config 4 / replay: object value bytes (RecoverSegmentBenchmark default)")
    ap.add_argument("--walk-part-shift", type=int, default=0,
                    help="replay: force log2 of the parallel walk's part bytes (0: chosen per batch)")
    ap.add_argument("--entries", type=int, default=1_000_000)
    ap.add_argument("--path", default="entries", choices=["entries", "batch"])
    ap.add_argument("--entry-size", type=int, default=0, help="fixed entry length (default: Zipf mix)")
    ap.add_argument("--exclude-size", type=int, default=0,
                    help="entries config: drop the entries of this size from the mix (A/B only)")
    ap.add_argument("--replay-nseg", type=int, default=512,
                    help="replay config: segments (RecoverSegmentBenchmark: 4096/8)")
    ap.add_argument("--replay-cpu-sample", type=int, default=64,
                    help="replay config: segments verified by the CPU baseline")
    ap.add_argument("--walk-cus", type=int, default=0,
                    help="replay config: pipeline batches, walking on this many CUs "
                         "(a multiple of 8) beside the object scan on the rest; 0 = serial")
    ap.add_argument("--verify-in-walk", type=int, default=1, choices=[0, 1, 2],
                    help="replay: check small objects while the walk copies their records "
                         "(RAMCRC_OPT_VERIFY_IN_WALK; 1 = for small entries, the default)")
    ap.add_argument("--serial-walk", action="store_true",
                    help="replay config: one wavefront per segment walk (RAMCRC_OPT_SERIAL_WALK)")
    ap.add_argument("--contexts", type=int, default=0,
                    help="entries / replay config: K host threads, one context and stream each, "
                         "submitting concurrently (RecoverSegmentBenchmark's replay threads)")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-t1", action="store_true", help="config 4 at N>1: skip the 1-GPU t1 run")
    ap.add_argument("--host-dry-run", action="store_true",
                    help="config 4 plumbing on the CPU (gloo, host CRC path, no GPU)")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    n = args.gpus if args.gpus is not None else int(env_world or 1)
    if n < 1:
        log("bench: --gpus must be >= 1")
        return 2
    if env_world is None and n > 1:
        return launch_ranks(n, sys.argv[1:])   # before any GPU call
    if int(env_world or 1) != n:
        log(f"bench: --gpus {n} but the launcher started WORLD_SIZE={env_world} ranks")
        return 2

    # stdout carries exactly one JSON line: everything else the ranks' libraries
    # print there (RCCL's version banner at communicator creation) goes to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    from ramcloud_amd import build as rbuild, ramcrc
    ramcrc.lib()  # fail loudly if the HIP library is missing
    info = ramcrc.lib().ramcrc_build_info().decode()

    def emit(line):
        # provenance: the source hash compiled into the library that ran, and
        # whether it matches the sources of this tree
        line["build_info"] = info
        line["build_matches_tree"] = rbuild.built_sha(ramcrc.lib_path()) == rbuild.source_sha()
        os.write(json_fd, (json.dumps(line) + "\n").encode())

    if args.config == "host":
        emit(run_host())
        return 0
    if args.host_dry_run:
        ranks = Ranks("gloo")
        line = run_recovery_host_dry(args, ranks)
    else:
        import torch
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        ranks = Ranks("nccl")
        config = args.config
        if config == "segments":
            config = "c2" if ranks.world == 1 else "recovery"
        run = {"c2": run_c2, "recovery": run_recovery, "entries": run_entries,
               "replay": run_replay, "append": run_append, "stream": run_stream}[config]
        if args.contexts and config in ("entries", "replay"):
            run = run_contexts
        line = run(args, ranks)
    if ranks.rank == 0:
        emit(line)
    ranks.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
