// The recovery-scan shard's layout arithmetic and step orchestration, shared
// by the C-ABI shard (ramcrc_shard.hip, with HIP streams and RCCL) and the
// host unit test (tests/cpp/shard_plan_test.cc, with host stand-ins for the
// scan kernels and the collectives), so that the index math and the order of
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
//   status[q] = step status of rank q on every rank         (same RCCL group)
//   all[s] = gather[gather_index(s)]                        (unpad; skipped
//                                                           when N divides nseg
//                                                           and all == gather)
//
// Liveness rule: once a rank has entered a step it never leaves before the
// collective its peers are waiting in.  Two kinds of failure are possible:
//   - a buffer that has to grow cannot be allocated.  Whether a step grows is
//     a function of nseg alone (the capacity watermark below moves the same
//     way on every rank), so on exactly those steps every rank first grows,
//     then all ranks exchange one status word (agree); if any rank failed,
//     every rank returns before the data collective (the failing rank its own
//     error, the others kPeerFailed).  Steps that do not grow allocate
//     nothing and cannot fail this way.
//   - an argument check or a scan launch fails: the rank still joins the
//     all-gather, from its internal gather buffer (always as large as the
//     watermark), with its slots set to 0xFFFFFFFF, and its status word says
//     why; every peer learns of it from the gathered status words at its next
//     sync (peer_status) instead of taking the poisoned slots as CRCs.
// Every rank must call a step with the same nseg (the collectives' counts
// depend on it), as with any collective.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define RAMCRC_SHARD_HD __host__ __device__ __forceinline__
#else
#define RAMCRC_SHARD_HD inline
#endif

namespace ramcrc_shard_plan {

// Returned by a rank whose own part of a step succeeded while another rank's
// failed (RAMCRC_EPEER in include/ramcrc.h).
constexpr int kPeerFailed = -8;

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

// Capacity watermark after a step that needs `need` elements: the internal
// gather and result buffers of every rank hold at least this many.  A pure
// function of the history of nseg, hence equal on every rank.
inline uint64_t grow_target(uint64_t need)
{
    uint64_t c = 256;
    while (c < need)
        c <<= 1;
    return c;
}

// What a rank reports at sync: its own failure first, else kPeerFailed when
// any rank's gathered status word of the last step is nonzero.
inline int peer_status(int own_failed, const uint32_t* status, int nranks)
{
    if (own_failed)
        return own_failed;
    for (int q = 0; q < nranks; q++)
        if (status[q])
            return kPeerFailed;
    return 0;
}

// The operations one step needs from its environment, for local rank k
// (global rank ranks[k]).  Every enqueue is ordered on that rank's stream.
//   uint64_t capacity()                     watermark of the internal buffers
//   void set_capacity(c)
//   int  reserve(k, elems)                  grow rank k's gather + result buffers
//   int  agree(const int* st)               synchronous exchange of one status word
//                                           per rank (st[k] for local rank k): 0 when
//                                           every rank reported 0, else the first
//                                           nonzero st[k], else kPeerFailed
//   int  check(k, lo, hi)                   argument check, nothing enqueued
//   int  scan(k, lo, hi, dst_is_caller, offset)  CRCs of [lo, hi) -> recv + offset
//   int  poison(k, dst_is_caller, offset, count) fill a failed rank's slots
//   int  put_status(k, rc)                  this step's status word of rank k
//   int  group_start() / group_end()
//   int  all_gather(k, dst_is_caller, offset, count)  recv[offset, +count) -> all ranks
//   int  all_gather_status(k)               status[rank] -> every rank's status[]
//   int  unpad(k, nseg, nranks)             all[s] = gather[gather_index(s)]
//   void set_failed(k, rc)                  remember a failure for the next sync
template <class Ops>
int run_step(Ops& ops, int nlocal, const int* ranks, int nranks, uint64_t nseg, bool have_all)
{
    const uint64_t N = uint64_t(nranks);
    const uint64_t w = width(nseg, N);
    if (w == 0)
        return 0;
    if (nlocal < 1 || nlocal > 64)
        return -1;   // RAMCRC_EINVAL: more local ranks than GPUs a node has
    // 1. growth, agreed by every rank before any collective that needs it
    const uint64_t need = w * N;
    if (need > ops.capacity()) {
        const uint64_t cap = grow_target(need);
        int st[64];
        for (int k = 0; k < nlocal; k++)
            st[k] = ops.reserve(k, cap);
        const int rc = ops.agree(st);
        if (rc) {
            for (int k = 0; k < nlocal; k++)
                ops.set_failed(k, st[k] ? st[k] : kPeerFailed);
            return rc;
        }
        ops.set_capacity(cap);
    }
    // 2. checks and scans; a failed rank's slots are poisoned instead, in its
    // internal gather buffer when it cannot use the caller's
    const bool divisible = (nseg % N) == 0;
    bool direct[64];
    int first_err = 0;
    for (int k = 0; k < nlocal; k++) {
        uint64_t lo, hi;
        range(nseg, N, uint64_t(ranks[k]), &lo, &hi);
        const uint64_t off = uint64_t(ranks[k]) * w;
        int rc = ops.check(k, lo, hi);
        direct[k] = divisible && have_all && rc == 0;
        if (!rc)
            rc = ops.scan(k, lo, hi, direct[k], off);
        if (rc) {
            ops.set_failed(k, rc);
            (void)ops.poison(k, direct[k], off, w);
            if (!first_err)
                first_err = rc;
        }
        const int prc = ops.put_status(k, rc);
        if (prc && !first_err)
            first_err = prc;
    }
    // 3. one group: a process driving several ranks issues their collectives
    // together (a lone rank's call would block on the others)
    int rc = ops.group_start();
    if (rc)
        return rc;
    for (int k = 0; k < nlocal; k++) {
        rc = ops.all_gather(k, direct[k], uint64_t(ranks[k]) * w, w);
        if (!rc)
            rc = ops.all_gather_status(k);
        if (rc) {
            (void)ops.group_end();
            return rc;
        }
    }
    rc = ops.group_end();
    if (rc)
        return rc;
    // 4. compaction into segment order (not for a rank whose arguments failed)
    for (int k = 0; k < nlocal; k++) {
        if (direct[k])
            continue;
        uint64_t lo, hi;
        range(nseg, N, uint64_t(ranks[k]), &lo, &hi);
        if (ops.check(k, lo, hi))
            continue;
        rc = ops.unpad(k, nseg, N);
        if (rc) {
            ops.set_failed(k, rc);
            if (!first_err)
                first_err = rc;
        }
    }
    return first_err;
}

}  // namespace ramcrc_shard_plan
