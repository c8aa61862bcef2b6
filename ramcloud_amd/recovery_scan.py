"""Multi-GPU recovery scan: the backup segment batch sharded across GPUs.

RAMCloud verifies each loaded 8 MiB replica independently
(BackupMasterRecovery::CyclicReplicaBuffer::buildNext,
src/BackupMasterRecovery.cc:743-809 -> SegmentIterator / RecoverySegmentBuilder),
so the batch partitions with no data exchange: rank r of N scans a contiguous
range of segments that already sits in its own HBM (one process per GPU), and
the only collective is one RCCL all-gather of the 4-byte per-segment results,
after which every rank (in particular the coordinating one) holds all CRCs for
host-side verification.  Segment bytes never cross xGMI in the timed path.

Works with any torch.distributed backend: "nccl" (= RCCL on ROCm) on the GPU
box, "gloo" in the CPU tests (with a host compute function standing in for
the kernel launch).
"""
import torch
import torch.distributed as dist


def shard_range(nseg, rank, world):
    """Contiguous [lo, hi) of segment indices owned by `rank` (sizes differ by <= 1)."""
    base, rem = divmod(nseg, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def gather_results(local, nseg, world, rank, group=None):
    """All-gather each rank's per-segment CRCs (int32 tensor) into one tensor of
    nseg CRCs ordered by segment index, on every rank."""
    if world == 1:
        return local
    width = (nseg + world - 1) // world
    padded = torch.zeros(width, dtype=local.dtype, device=local.device)
    padded[: local.numel()] = local
    backend = dist.get_backend(group)
    if backend == "nccl":
        full = torch.empty(width * world, dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(full, padded, group=group)
        parts = list(full.view(world, width))
    else:
        parts = [torch.empty_like(padded) for _ in range(world)]
        dist.all_gather(parts, padded, group=group)
    pieces = []
    for r in range(world):
        lo, hi = shard_range(nseg, r, world)
        pieces.append(parts[r][: hi - lo])
    return torch.cat(pieces)


class RecoveryScan:
    """One rank's share of a recovery scan of `nseg` segments of `seg_bytes`.

    `scan_fn(shard_data, seg_bytes, count, out)` computes the CRCs of `count`
    contiguous segments into `out`; by default it is the MI355X kernel
    (libramcrc ramcrc_segments_device) on this rank's GPU.
    """

    def __init__(self, nseg, seg_bytes, rank=0, world=1, ctx=None, scan_fn=None, group=None):
        self.nseg, self.seg_bytes = nseg, seg_bytes
        self.rank, self.world, self.group = rank, world, group
        self.lo, self.hi = shard_range(nseg, rank, world)
        if scan_fn is None:
            if ctx is None:
                raise ValueError("need a ramcrc Context or a scan_fn")

            def scan_fn(data, seg_bytes_, count, out):
                ctx.segments(data, seg_bytes_, count, out)
        self.scan_fn = scan_fn

    @property
    def count(self):
        return self.hi - self.lo

    def step(self, shard_data, out_local):
        """Scan this rank's shard and all-gather every rank's results."""
        if self.count:
            self.scan_fn(shard_data, self.seg_bytes, self.count, out_local)
        return gather_results(out_local[: self.count], self.nseg, self.world, self.rank,
                              self.group)
