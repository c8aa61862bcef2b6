"""Multi-rank recovery scan on CPU with the gloo backend (world_size 2 and 3).

The sharding and the result all-gather are the same code the GPU ranks run
over RCCL (ramcloud_amd/recovery_scan.py); here the per-shard scan is the
oracle on host memory, standing in for the kernel launch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ramcloud_amd.recovery_scan import RecoveryScan, gather_results, shard_range

SEG = 4096


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, nseg, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        from ramcloud_amd import workloads

        def scan_fn(data, seg_bytes, count, out):
            host = data.numpy()
            res = oracle.segments(host, seg_bytes, count, threads=1)
            out[:count] = torch.from_numpy(res.view(np.int32))

        scan = RecoveryScan(nseg, SEG, rank, world, scan_fn=scan_fn)
        lo, hi = scan.lo, scan.hi
        shard = torch.empty(max(hi - lo, 1) * SEG, dtype=torch.uint8)
        for i in range(lo, hi):  # each rank holds only its own segments
            shard[(i - lo) * SEG:(i - lo + 1) * SEG] = torch.from_numpy(
                workloads.splitmix_bytes_np(workloads.SEGMENT_SEED + i, SEG))
        out = torch.zeros(max(hi - lo, 1), dtype=torch.int32)
        full = scan.step(shard, out)
        q.put((rank, full.numpy().view(np.uint32).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nseg", [(2, 10), (2, 1), (3, 11)])
def test_recovery_scan_gloo(world, nseg):
    from oracle import oracle
    from ramcloud_amd import workloads
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nseg, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [oracle.crc32c(workloads.splitmix_bytes_np(workloads.SEGMENT_SEED + i, SEG))
            for i in range(nseg)]
    for r in range(world):
        assert results[r] == want, r


def test_shard_range_partitions():
    for n in range(0, 40):
        for w in range(1, 9):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_gather_single_rank_identity():
    t = torch.arange(5, dtype=torch.int32)
    assert gather_results(t, 5, 1, 0) is t
