// Host-side CRC32C for the synchronous Crc32C::update() path.
//
// RAMCloud keeps update() synchronous and on the caller's thread
// (src/Crc32C.h:200-206); the 1-5 byte metadata updates of Segment::append
// (src/Segment.cc:211,218) and the per-object checksums on the write path must
// never wait on a GPU.  This file provides that host path behind the C ABI:
//
//   ramcrc_update_hw  SSE4.2 crc32 instruction.  The reference runs one
//                     dependency chain (src/Crc32C.h:52-84), bound by the
//                     3-cycle crc32q latency; here three independent chains
//                     run over three adjacent 8 KiB blocks and are merged with
//                     X^n operator tables (raw(0,A||B) = X^|B|(raw(0,A)) ^
//                     raw(0,B)), so the core issues one crc32q per cycle.
//   ramcrc_update_sw  slicing-by-8 like softwareCrc32C (src/Crc32C.h:96-153),
//                     tables generated from the polynomial at compile time.
#include "ramcrc.h"

#include <string.h>

#include "gf2.h"

namespace {

using ramcrc::ByteTable;
using ramcrc::OpTable;

struct Slice8 {
    uint32_t t[8][256];
};

constexpr Slice8 make_slice8()
{
    Slice8 s{};
    const ByteTable b = ramcrc::make_byte_table();
    for (int i = 0; i < 256; i++)
        s.t[0][i] = b.t[i];
    for (int i = 0; i < 256; i++) {
        uint32_t c = s.t[0][i];
        for (int k = 1; k < 8; k++) {
            c = s.t[0][c & 0xFF] ^ (c >> 8);
            s.t[k][i] = c;
        }
    }
    return s;
}

constexpr uint64_t kStreamBlock = 8192;  // bytes per interleaved chain
constexpr Slice8 kSlice = make_slice8();
constexpr OpTable kShift1 = ramcrc::make_op(kStreamBlock);
constexpr OpTable kShift2 = ramcrc::make_op(2 * kStreamBlock);

inline uint64_t ld64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
inline uint32_t ld32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint16_t ld16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }

#if defined(__x86_64__) || defined(__i386__)
__attribute__((target("sse4.2"))) uint32_t hw_chain(uint32_t s, const uint8_t* p, uint64_t n)
{
    uint64_t c = s;
    for (; n >= 8; n -= 8, p += 8)
        c = __builtin_ia32_crc32di(c, ld64(p));
    s = static_cast<uint32_t>(c);
    if (n & 4) {
        s = __builtin_ia32_crc32si(s, ld32(p));
        p += 4;
    }
    if (n & 2) {
        s = __builtin_ia32_crc32hi(s, ld16(p));
        p += 2;
    }
    if (n & 1)
        s = __builtin_ia32_crc32qi(s, *p);
    return s;
}

__attribute__((target("sse4.2"))) uint32_t hw_update(uint32_t s, const uint8_t* p, uint64_t n)
{
    while (n >= 3 * kStreamBlock) {
        uint64_t c0 = s, c1 = 0, c2 = 0;
        const uint8_t* p1 = p + kStreamBlock;
        const uint8_t* p2 = p + 2 * kStreamBlock;
        for (uint64_t i = 0; i < kStreamBlock; i += 8) {
            c0 = __builtin_ia32_crc32di(c0, ld64(p + i));
            c1 = __builtin_ia32_crc32di(c1, ld64(p1 + i));
            c2 = __builtin_ia32_crc32di(c2, ld64(p2 + i));
        }
        s = ramcrc::apply_op(kShift2, static_cast<uint32_t>(c0)) ^
            ramcrc::apply_op(kShift1, static_cast<uint32_t>(c1)) ^ static_cast<uint32_t>(c2);
        p += 3 * kStreamBlock;
        n -= 3 * kStreamBlock;
    }
    return hw_chain(s, p, n);
}
#endif

uint32_t sw_update(uint32_t crc, const uint8_t* p, uint64_t n)
{
    uint64_t lead = (4u - (reinterpret_cast<uintptr_t>(p) & 3u)) & 3u;
    if (lead > n)
        lead = n;
    for (uint64_t i = 0; i < lead; i++)
        crc = kSlice.t[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
    n -= lead;
    for (uint64_t k = n >> 3; k > 0; k--, p += 8) {
        const uint32_t lo = crc ^ ld32(p);
        const uint32_t hi = ld32(p + 4);
        crc = kSlice.t[7][lo & 0xFF] ^ kSlice.t[6][(lo >> 8) & 0xFF] ^
              kSlice.t[5][(lo >> 16) & 0xFF] ^ kSlice.t[4][lo >> 24] ^
              kSlice.t[3][hi & 0xFF] ^ kSlice.t[2][(hi >> 8) & 0xFF] ^
              kSlice.t[1][(hi >> 16) & 0xFF] ^ kSlice.t[0][hi >> 24];
    }
    for (uint64_t i = 0; i < (n & 7); i++)
        crc = kSlice.t[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
    return crc;
}

bool detect_hw()
{
#if defined(__x86_64__) || defined(__i386__)
    return __builtin_cpu_supports("sse4.2");
#else
    return false;
#endif
}

const bool g_have_hw = detect_hw();

}  // namespace

extern "C" {

uint32_t ramcrc_update_hw(uint32_t state, const void* data, uint64_t nbytes)
{
#if defined(__x86_64__) || defined(__i386__)
    if (g_have_hw)
        return hw_update(state, static_cast<const uint8_t*>(data), nbytes);
#endif
    return sw_update(state, static_cast<const uint8_t*>(data), nbytes);
}

uint32_t ramcrc_update_sw(uint32_t state, const void* data, uint64_t nbytes)
{
    return sw_update(state, static_cast<const uint8_t*>(data), nbytes);
}

uint32_t ramcrc_update(uint32_t state, const void* data, uint64_t nbytes)
{
    return ramcrc_update_hw(state, data, nbytes);
}

int ramcrc_cpu_has_hw(void) { return g_have_hw ? 1 : 0; }

uint32_t ramcrc_shift(uint32_t state, uint64_t nbytes)
{
    return ramcrc::mulmod(state, ramcrc::xpow8(nbytes));
}

uint32_t ramcrc_combine(uint32_t raw_a, uint32_t raw_b, uint64_t len_b)
{
    return ramcrc_shift(raw_a, len_b) ^ raw_b;
}

}  // extern "C"
