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

const uint32_t* ramcrc_slice8_tables(void) { return &kSlice.t[0][0]; }

uint32_t ramcrc_shift(uint32_t state, uint64_t nbytes)
{
    return ramcrc::mulmod(state, ramcrc::xpow8(nbytes));
}

uint32_t ramcrc_combine(uint32_t raw_a, uint32_t raw_b, uint64_t len_b)
{
    return ramcrc_shift(raw_a, len_b) ^ raw_b;
}

// The append path of RecoverSegmentBenchmark::run
// (nanobenchmarks/RecoverSegmentBenchmark.cc:131-146): Object(key, value,
// version 0, timestamp 0) serialised by Object::assembleForLog
// (src/Object.cc:213-218) -- Header{checksum, timestamp, version, tableId}
// (src/Object.h:137-182), KeyCount 1, CumulativeKeyLength 8, the 8-byte key
// (src/Object.cc:107-141), the value -- appended by Segment::append
// (src/Segment.cc:197-228) while hasSpaceFor (:136-154) holds.
int ramcrc_segment_fill_objects(uint8_t* seg, uint32_t capacity, uint32_t value_len,
                                uint64_t first_key, uint32_t* n_objects, ramcrc_seg_cert* cert)
{
    if (!seg || !cert)
        return RAMCRC_EINVAL;
    const uint64_t objlen64 = 24 + 1 + 2 + 8 + uint64_t(value_len);
    if (objlen64 > 0xFFFFFFFFull)
        return RAMCRC_EINVAL;
    const uint32_t objlen = uint32_t(objlen64);
    const uint32_t lb = objlen < 0x100u ? 1 : objlen < 0x10000u ? 2 : objlen < 0x1000000u ? 3 : 4;
    const uint8_t hdr = uint8_t(RAMCRC_LOG_ENTRY_TYPE_OBJ | ((lb - 1) << 6));
    const uint64_t entry = 1 + lb + uint64_t(objlen);
    uint32_t head = 0, n = 0, meta = 0xFFFFFFFFu;
    uint64_t key = first_key;
    while (entry <= uint64_t(capacity) - head) {
        uint8_t* e = seg + head;
        e[0] = hdr;
        for (uint32_t k = 0; k < lb; k++)
            e[1 + k] = uint8_t(objlen >> (8 * k));
        meta = ramcrc_update(meta, e, 1 + lb);   // Segment's running metadata checksum
        uint8_t* o = e + 1 + lb;
        memset(o + 4, 0, 20);                    // timestamp, version, tableId
        o[24] = 1;                               // KeyCount
        o[25] = 8;                               // CumulativeKeyLength (LE)
        o[26] = 0;
        for (int k = 0; k < 8; k++)
            o[27 + k] = uint8_t(key >> (8 * k));
        const uint32_t ck = ~ramcrc_update(0xFFFFFFFFu, o + 4, objlen - 4);   // Object::computeChecksum
        for (int k = 0; k < 4; k++)
            o[k] = uint8_t(ck >> (8 * k));
        head += uint32_t(entry);
        n++;
        key++;
    }
    memset(seg + head, 0, capacity - head);
    uint8_t lenle[4];
    for (int k = 0; k < 4; k++)
        lenle[k] = uint8_t(head >> (8 * k));
    cert->segment_length = head;
    cert->checksum = ~ramcrc_update(meta, lenle, 4);   // Segment::getAppendedLength
    if (n_objects)
        *n_objects = n;
    return RAMCRC_OK;
}

}  // extern "C"
