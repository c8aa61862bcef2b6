// The recovery-scan shard's layout arithmetic and step orchestration, shared
// by the C-ABI shard (ramcrc_shard.hip, with HIP streams and RCCL) and the
// host unit test (tests/cpp/shard_plan_test.cc, with host stand-ins for the
// scan kernels and the collective), so that the index math and the order of
// operations a rank > 0 executes are tested on the CPU before any multi-GPU
// run.
//
// Reference behaviour: BackupMasterRecovery::CyclicReplicaBuffer::buildNext
// (src/BackupMasterRecovery.cc:743-809) verifies every replica on its own, so
// the batch splits into contiguous segment ranges, one per rank; the only
// exchange is the 4-byte result per segment.
//
// One step on rank r of N (nseg segments, width = ceil(nseg / N)):
//   gather[r * width + j] = CRC of segment lo_r + j        (scan)
//   all-gather in place: gather[q * width + j] on every rank (collective)
//   all[s] = gather[gather_index(s)]                        (unpad; skipped
//                                                           when N divides nseg
//                                                           and all == gather)
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define RAMCRC_SHARD_HD __host__ __device__ __forceinline__
#else
#define RAMCRC_SHARD_HD inline
#endif

namespace ramcrc_shard_plan {

// Contiguous [lo, hi) of rank `rank`: sizes differ by at most one, lower
// ranks get the extra segments.
RAMCRC_SHARD_HD void range(uint64_t nseg, uint64_t nranks, uint64_t rank, uint64_t* lo,
                           uint64_t* hi)
{
    const uint64_t base = nseg / nranks, rem = nseg % nranks;
    *lo = rank * base + (rank < rem ? rank : rem);
    *hi = *lo + base + (rank < rem ? 1 : 0);
}

// Slots per rank in the gather buffer.
RAMCRC_SHARD_HD uint64_t width(uint64_t nseg, uint64_t nranks) { return (nseg + nranks - 1) / nranks; }

// Owner rank of segment s (s < nseg).
RAMCRC_SHARD_HD uint64_t owner(uint64_t s, uint64_t nseg, uint64_t nranks)
{
    const uint64_t base = nseg / nranks, rem = nseg % nranks;
    const uint64_t big = rem * (base + 1);   // segments of the ranks holding base + 1
    return s < big ? s / (base + 1) : rem + (s - big) / base;
}

// Where segment s's CRC lands in the gathered buffer.
RAMCRC_SHARD_HD uint64_t gather_index(uint64_t s, uint64_t nseg, uint64_t nranks)
{
    const uint64_t q = owner(s, nseg, nranks);
    uint64_t lo, hi;
    range(nseg, nranks, q, &lo, &hi);
    return q * width(nseg, nranks) + (s - lo);
}

// The operations one step needs from its environment, for local rank k
// (global rank ranks[k]).  Every enqueue is ordered on that rank's stream.
//   int  check(k, lo, hi)                  argument check, nothing enqueued
//   int  reserve(k, gather_elems, all_elems)   size buffers, nothing enqueued
//   int  scan(k, lo, hi, dst_is_caller, offset)  CRCs of [lo, hi) -> recv + offset
//   int  poison(k, dst_is_caller, offset, count) fill a failed rank's slots
//   int  group_start() / group_end()
//   int  all_gather(k, dst_is_caller, offset, count)  recv[offset, +count) -> all ranks
//   int  unpad(k, nseg, nranks)             all[s] = gather[gather_index(s)]
//   void set_failed(k, rc)                  remember a failure for the next sync
// A failure after the checks does not skip the collective: the rank's slots
// are poisoned and it still takes part, so that peers in other processes do
// not block in the all-gather forever; the failure is returned (and kept for
// the rank's next sync).
template <class Ops>
int run_step(Ops& ops, int nlocal, const int* ranks, int nranks, uint64_t nseg, bool have_all)
{
    const uint64_t N = uint64_t(nranks);
    const uint64_t w = width(nseg, N);
    if (w == 0)
        return 0;
    const bool direct = (nseg % N) == 0 && have_all;
    // 1. every argument and buffer of every local rank before any work
    for (int k = 0; k < nlocal; k++) {
        uint64_t lo, hi;
        range(nseg, N, uint64_t(ranks[k]), &lo, &hi);
        int rc = ops.check(k, lo, hi);
        if (rc)
            return rc;
        rc = ops.reserve(k, direct ? 0 : w * N, have_all ? 0 : nseg);
        if (rc)
            return rc;
    }
    // 2. the scans; a failed rank's slots are poisoned instead
    int first_err = 0;
    for (int k = 0; k < nlocal; k++) {
        uint64_t lo, hi;
        range(nseg, N, uint64_t(ranks[k]), &lo, &hi);
        const uint64_t off = uint64_t(ranks[k]) * w;
        int rc = ops.scan(k, lo, hi, direct, off);
        if (rc) {
            ops.set_failed(k, rc);
            (void)ops.poison(k, direct, off, w);
            if (!first_err)
                first_err = rc;
        }
    }
    // 3. one group: a process driving several ranks issues their collectives
    // together (a lone rank's call would block on the others)
    int rc = ops.group_start();
    if (rc)
        return rc;
    for (int k = 0; k < nlocal; k++) {
        rc = ops.all_gather(k, direct, uint64_t(ranks[k]) * w, w);
        if (rc) {
            (void)ops.group_end();
            return rc;
        }
    }
    rc = ops.group_end();
    if (rc)
        return rc;
    // 4. compaction into segment order
    if (!direct) {
        for (int k = 0; k < nlocal; k++) {
            rc = ops.unpad(k, nseg, N);
            if (rc) {
                ops.set_failed(k, rc);
                if (!first_err)
                    first_err = rc;
            }
        }
    }
    return first_err;
}

}  // namespace ramcrc_shard_plan
