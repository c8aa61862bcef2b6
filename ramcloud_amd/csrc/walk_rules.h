// The parallel segment walk's per-hop rules, shared by the device kernels
// (ramcrc_device.hip) and the host unit test of the synchronisation filter
// (tests/cpp/walk_rules_test.cc): how one hop of Segment::checkMetadataIntegrity
// (src/Segment.cc:758-800) advances, which hops a candidate chain may take, and
// the byte-parallel first-hop filter that must pass every plausible candidate.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define RAMCRC_WALK_HD __host__ __device__ __forceinline__
#else
#define RAMCRC_WALK_HD inline
#endif

namespace ramcrc_walk {

constexpr uint32_t kNumTypes = 12;                  // TOTAL_LOG_ENTRY_TYPES, src/LogEntryTypes.h:68

// One hop of the reference walk from a header read as q: the entry's metadata
// byte count (1 + lengthBytes), payload length and the next offset (64-bit,
// so that a uint32_t wrap is visible).
struct Hop {
    uint32_t mbytes, len;
    uint64_t next;
};

RAMCRC_WALK_HD Hop hop_of(uint64_t q, uint32_t pos)
{
    const uint32_t t = (uint32_t(q) >> 6) & 3;   // getLengthBytes() - 1
    const uint64_t mask = t == 3 ? 0xFFFFFFFFull : ((1ull << (8 * (t + 1))) - 1);
    Hop h;
    h.len = uint32_t((q >> 8) & mask);
    h.mbytes = t + 2;
    h.next = uint64_t(pos) + h.mbytes + h.len;
    return h;
}

// A hop a candidate chain may take: a header of a type the log writes
// (src/LogEntryTypes.h:29-68: 1 .. TOTAL-1; INVALID = 0 only fills the
// zeroed tail), length bytes in the canonical (shortest) form EntryHeader
// writes (src/Segment.h:135-148), and an entry that ends inside the segment.
RAMCRC_WALK_HD bool plausible(uint64_t q, const Hop& h, uint32_t capacity)
{
    const uint32_t type = uint32_t(q) & 0x3f;
    const uint32_t t = h.mbytes - 2;   // lengthBytes - 1
    const bool canon = t == 0 || ((h.len >> (8 * t)) != 0);
    return type != 0 && type < kNumTypes && canon && h.next <= capacity;
}

// First-hop filter of four candidates at once (bytes of h, one candidate
// per byte; top3 = for each, the byte three further on, the top length byte
// of a 3-byte length): a superset of plausible() -- the type is 1..11, and,
// where the capacity rules them out, no 4-byte length (>= 2^24 when
// canonical) and no 3-byte length with its top bit set (>= 2^23).  Returns
// one bit per candidate.
RAMCRC_WALK_HD uint32_t first_hop4(uint32_t h, uint32_t top3, bool kill4, bool kill3)
{
    const uint32_t t = h & 0x3f3f3f3fu;
    constexpr uint32_t kLo = 0x3f3f3f3fu;                      // t + 63 >= 64 iff t >= 1
    constexpr uint32_t kHi = 0x01010101u * (64 - kNumTypes);    // t + 52 >= 64 iff t >= 12
    uint32_t ok = ((t + kLo) & ~(t + kHi) & 0x40404040u) << 1;   // bit 7 of each byte
    const uint32_t lb4 = h & (h << 1) & 0x80808080u;
    const uint32_t lb3 = h & ~(h << 1) & 0x80808080u;
    ok &= ~((kill4 ? lb4 : 0u) | (kill3 ? (lb3 & top3) : 0u));
    const uint32_t x = ok >> 7;
    return (x | (x >> 7) | (x >> 14) | (x >> 21)) & 0xFu;
}

}  // namespace ramcrc_walk
