// MI355X (gfx950) kernels for batched CRC32C, plus the device half of the C ABI.
//
// What is computed: for every buffer i, the state RAMCloud's
// Crc32C::update(buf_i, len_i) (src/Crc32C.h:200-206) reaches from state
// init[i] (default 0xFFFFFFFF, src/Crc32C.h:177), optionally inverted as by
// getResult() (src/Crc32C.h:247-249).  Bit-identical to intelCrc32C /
// softwareCrc32C (src/Crc32C.h:39-153).
//
// How (see DESIGN.md for the derivation and the roofline):
//
//  * CRC is linear over GF(2) and every operator is a multiplication by a
//    constant power of x (gf2.h), so a buffer can be cut anywhere, the pieces
//    CRC'd from state 0, and the partials shifted into place and XORed.
//  * k_chunks -- the byte scan.  Buffers >= 64 KiB are cut into 256 KiB
//    chunks aligned to absolute 256 KiB boundaries; one wave scans one chunk
//    as 1 KiB blocks (lane l owns bytes [16l, 16l+16) of every block: one
//    coalesced global_load_dwordx4 per lane per block).  Each lane keeps four
//    accumulators (one per dword) updated by Horner's rule
//        u <- X^1024(u) ^ w
//    so the only per-byte work is one X^1024 table lookup per input byte.
//    The four X^1024 byte tables live in LDS replicated 32 times so that
//    lane l always hits bank l%32: ds_read_b32 without bank conflicts.  The
//    LDS address of a lookup is formed by ONE v_perm_b32 (byte k of u into
//    address byte 1, the lane's bank offset into byte 0, the table pair into
//    byte 2).  At the end of a chunk the 256 accumulators are folded with
//    X^4 in-lane and X^16..X^512 across lanes (wave shuffles), giving the raw
//    CRC of the chunk relative to its 1 KiB-aligned end.
//  * k_combine -- one wave per buffer merges its chunk partials with
//    x^(8d) constants (4 table lookups + GF(2) multiplies), removes the
//    zero-padding of the last block with x^(-8p), and writes the result.
//    The initial state is injected as an XOR into the first four message
//    bytes (raw(s,M) = raw(0, M ^ s||0...)) inside k_chunks.
//  * k_entries -- small buffers (log entries, objects): one lane per entry,
//    Horner with X^16 over 16-byte words (same replicated-LDS lookup),
//    masked head/tail words, then x^(-8p) to undo the tail padding.
//  * k_plan_* -- for the general offset/length table: per-entry chunk counts
//    and their exclusive prefix so waves can map a global chunk index to
//    (entry, chunk) with two binary searches.
//
// No MFMA: this is a byte scan, bound by HBM reads.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <mutex>
#include <new>
#include <utility>
#include <vector>
#include <stdio.h>
#include <string.h>

#include "gf2.h"
#include "walk_rules.h"
#include "ramcrc.h"

namespace {

using namespace ramcrc_walk;   // Hop, hop_of, plausible, first_hop4, kNumTypes

using ramcrc::OpTable;

constexpr int kWaveSize = 64;
constexpr int kWavesPerGroup = 16;                 // 1024-thread workgroups, 1 per CU
constexpr int kThreads = kWaveSize * kWavesPerGroup;
constexpr uint32_t kBlock = 1024;                  // bytes per wave step
#ifndef RAMCRC_CHUNK_SHIFT
#define RAMCRC_CHUNK_SHIFT 18
#endif
#ifndef RAMCRC_UNROLL
#define RAMCRC_UNROLL 4
#endif
#ifndef RAMCRC_ASM_XOR3
#define RAMCRC_ASM_XOR3 1
#endif
#ifndef RAMCRC_DYNAMIC
#define RAMCRC_DYNAMIC 0
#endif
constexpr int kChunkShift = RAMCRC_CHUNK_SHIFT;
constexpr uint64_t kChunk = 1ull << kChunkShift;   // 256 KiB per wave work item
constexpr uint64_t kLargeMin = 64 * 1024;          // batch API threshold
constexpr uint64_t kWideCombineMin = 16384;        // tables above: k_combine<kWide>
constexpr int kUnroll = RAMCRC_UNROLL;             // blocks per register group (x2 in flight)
constexpr bool kDynamic = RAMCRC_DYNAMIC;          // waves dequeue chunks from a counter

// ------------------------------------------------------------------ tables
struct alignas(16) DeviceTables {
    OpTable stride_large;   // X^1024: Horner step of k_chunks
    OpTable stride_small;   // X^128:  Horner step of k_entries (8 lanes x 16 B)
    OpTable comb[7];        // X^4, X^16, X^32, X^64, X^128, X^256, X^512
    ramcrc::ByteTable t0;   // X^1 byte step
    uint32_t xblk[4][256];  // x^(8 * 1024 * b * 256^j)
    uint32_t xinv[1024];    // x^(-8 p)
    uint32_t pos[132][256]; // k_entries, tiny phase: row r = X^(r-3)(byte), rows 0..3 (m <= 0) zero
    // The same rows laid out for conflict-free lookups (tiny phase, RAMCRC_TINY_CF):
    // word 128 (255 - b) + (128 - m) = X^m(b), m = 1 .. 128, then 128 zero words.
    uint32_t post[256 * 128 + 128];
    uint32_t xmeta[5 * 64 + 1];   // k_seg_walk: x^(8d), d = 0 .. 320 (one batch of metadata)
    uint32_t xbyte[4][256];       // x^(8 * b * 256^j): x^(8d) for any 32-bit d in 4 factors
    alignas(16) OpTable xinv128;  // tiny phase: X^-128 (a window sum moved back from the window end)
    // Bases the tiny phase builds its LDS tables from (tiny_fill_gen):
    // twb[q][k] = X^(128 - q)(1 << k), twib[j][k] = X^-128(1 << (8 j + k))
    alignas(16) uint32_t twb[128][8];
    alignas(16) uint32_t twib[4][8];
    // k_entries' long phase (group_fold, flush_batch, head and tail steps),
    // laid out as in LDS from kX4Off on, so one fill copies them all:
    struct alignas(16) LongTabs {
        OpTable x4, x16, x32, x64;        // group_fold
        OpTable x8;                       // X^8, the in-lane fold's second level
        uint32_t xinv4[256];              // x^(-8 (p - 4)): unpad by p, the fold's X^4 folded in
        uint32_t headtab[21][8];          // c = S - piece + 4 (0..20): 4 keep masks, 4 init selectors
        uint32_t tailtab[17][4];          // bytes d (0..16) of the piece below E: 4 keep masks
    } lt;
};

constexpr DeviceTables make_device_tables()
{
    DeviceTables t{};
    t.stride_large = ramcrc::make_op(kBlock);
    t.stride_small = ramcrc::make_op(128);
    const uint64_t comb_d[7] = {4, 16, 32, 64, 128, 256, 512};
    for (int i = 0; i < 7; i++)
        t.comb[i] = ramcrc::make_op(comb_d[i]);
    t.t0 = ramcrc::make_byte_table();
    for (int j = 0; j < 4; j++) {
        const uint32_t base = ramcrc::xpow8(uint64_t(kBlock) << (8 * j));
        uint32_t acc = ramcrc::kOne;
        for (int b = 0; b < 256; b++) {
            t.xblk[j][b] = acc;
            acc = ramcrc::mulmod(acc, base);
        }
    }
    const uint32_t inv8 = ramcrc::xinv8pow(1);
    uint32_t acc = ramcrc::kOne;
    for (int p = 0; p < 1024; p++) {
        t.xinv[p] = acc;
        acc = ramcrc::mulmod(acc, inv8);
    }
    for (int m = 1; m <= 128; m++) {
        const uint32_t c = ramcrc::xpow8(uint64_t(m));
        for (uint32_t b = 0; b < 256; b++) {
            t.pos[m + 3][b] = ramcrc::mulmod(b, c);
            t.post[128 * (255 - b) + (128 - m)] = t.pos[m + 3][b];
        }
    }
    for (int d = 0; d <= 5 * 64; d++)
        t.xmeta[d] = ramcrc::xpow8(uint64_t(d));
    for (int j = 0; j < 4; j++) {
        const uint32_t base = ramcrc::xpow8(uint64_t(1) << (8 * j));
        uint32_t acc = ramcrc::kOne;
        for (int b = 0; b < 256; b++) {
            t.xbyte[j][b] = acc;
            acc = ramcrc::mulmod(acc, base);
        }
    }
    {
        const uint32_t c = ramcrc::xinv8pow(128);
        for (int k = 0; k < 4; k++)
            for (uint32_t b = 0; b < 256; b++)
                t.xinv128.t[k][b] = ramcrc::mulmod(b << (8 * k), c);
        for (int k = 0; k < 4; k++)
            for (int j = 0; j < 8; j++)
                t.twib[k][j] = t.xinv128.t[k][1u << j];
    }
    for (int q = 0; q < 128; q++) {
        const uint32_t c = ramcrc::xpow8(uint64_t(128 - q));
        for (int j = 0; j < 8; j++)
            t.twb[q][j] = ramcrc::mulmod(1u << j, c);
    }
    t.lt.x4 = t.comb[0];
    t.lt.x16 = t.comb[1];
    t.lt.x32 = t.comb[2];
    t.lt.x64 = t.comb[3];
    t.lt.x8 = ramcrc::make_op(8);
    for (int p = 0; p < 256; p++)   // x^(-8 (p - 4)) = x^(-8 p) * x^32
        t.lt.xinv4[p] = ramcrc::mulmod(t.xinv[p], ramcrc::xpow8(4));
    for (int c = 0; c <= 20; c++) {   // c = clamp(S - piece, -4, 16) + 4
        const int off = c - 4;
        for (int j = 0; j < 4; j++) {
            uint32_t m = 0, sel = 0;
            for (int q = 0; q < 4; q++) {
                const int b = 4 * j + q, r = b - off;   // init byte r lands on piece byte b
                m |= uint32_t(b >= off ? 0xFF : 0) << (8 * q);
                // v_perm_b32(init, 0, sel): 4 + r picks init byte r, 0x0C yields 0
                sel |= uint32_t(r >= 0 && r < 4 ? 4 + r : 0x0C) << (8 * q);
            }
            t.lt.headtab[c][j] = m;
            t.lt.headtab[c][4 + j] = sel;
        }
    }
    for (int d = 0; d <= 16; d++)
        for (int j = 0; j < 4; j++) {
            const int k = d - 4 * j < 0 ? 0 : (d - 4 * j > 4 ? 4 : d - 4 * j);
            t.lt.tailtab[d][j] = k >= 4 ? 0xFFFFFFFFu : (1u << (8 * k)) - 1u;
        }
    return t;
}

__device__ const DeviceTables g_tab = make_device_tables();

// Compile-time self-checks of the algebra the kernels rely on.
static_assert(ramcrc::mulmod(ramcrc::kXInv, 0x40000000u) == ramcrc::kOne, "x * x^-1 != 1");
static_assert(ramcrc::mulmod(ramcrc::xpow8(3), ramcrc::xinv8pow(3)) == ramcrc::kOne,
              "x^24 * x^-24 != 1");

// --------------------------------------------------------- LDS layouts
// Replicated stride tables (both kernels): 128 KiB.
//   byte address = region*65536 + b*256 + (k&1)*128 + (lane&31)*4
//   region = k>>1, b = byte value, k = which byte of u (0..3)
// so ds_read_b32 of lane l always lands in bank l%32.
constexpr uint32_t kRepBytes = 131072;
constexpr uint32_t kCombOff = kRepBytes;                  // k_chunks: 7 x 4 KiB
constexpr uint32_t kLdsChunks = kCombOff + 7 * 4096;      // 159744 B
constexpr uint32_t kX4Off = kRepBytes;                    // k_entries: X^4,16,32,64 (16 KiB)
constexpr uint32_t kX8Off = kX4Off + 4 * 4096;            // k_entries: X^8 (4 KiB)
constexpr uint32_t kXinvOff = kX8Off + 4096;              // k_entries: x^(-8 (pad - 4)) (1 KiB)
constexpr uint32_t kHeadOff = kXinvOff + 1024;            // k_entries: head masks/selectors (672 B)
constexpr uint32_t kTailOff = kHeadOff + 21 * 32;         // k_entries: tail masks (272 B)
constexpr uint32_t kBinOff = kTailOff + 17 * 16;          // k_entries: bin table (4 KiB)
constexpr uint32_t kLdsEntries = kBinOff + 4096;          // 157616 B
static_assert(kBinOff % 16 == 0, "LDS table alignment");
static_assert(kBinOff - kX4Off == sizeof(DeviceTables::LongTabs), "long-phase tables: LDS = g_tab.lt");
static_assert(kLdsEntries <= 160 * 1024, "LDS budget");
static_assert(kLdsChunks <= 160 * 1024, "LDS budget");
#define RAMCRC_LDS_CHUNKS 159744    // reported by ramcrc_build_info
#define RAMCRC_LDS_ENTRIES 157616
static_assert(kLdsChunks == RAMCRC_LDS_CHUNKS && kLdsEntries == RAMCRC_LDS_ENTRIES,
              "build_info LDS sizes");

// LDS table fills.  Every thread issues all of its global loads before its
// first LDS store, so a fill costs about one L2 round trip instead of one per
// loop iteration (a 129 KiB fill would otherwise serialise ~33 round trips).
__device__ __forceinline__ void fill_replicated(uint8_t* lds, const OpTable& op)
{
    // 4 tables x 256 entries x 32 replicas; each item writes 4 replicas (16
    // contiguous bytes): 8192 items.
    constexpr uint32_t kItems = 4 * 256 * 8;
    constexpr int kU = 8;
    for (uint32_t base = threadIdx.x; base < kItems; base += kU * blockDim.x) {
        uint32_t v[kU];
#pragma unroll
        for (int j = 0; j < kU; j++) {
            const uint32_t idx = base + j * blockDim.x;
            const uint32_t ci = idx < kItems ? idx : 0;
            v[j] = op.t[ci >> 11][(ci >> 3) & 255];
        }
#pragma unroll
        for (int j = 0; j < kU; j++) {
            const uint32_t idx = base + j * blockDim.x;
            if (idx < kItems) {
                const uint32_t k = idx >> 11, bv = (idx >> 3) & 255, q = idx & 7;
                const uint32_t off = (k >> 1) * 65536 + bv * 256 + (k & 1) * 128 + q * 16;
                *reinterpret_cast<uint4*>(lds + off) = make_uint4(v[j], v[j], v[j], v[j]);
            }
        }
    }
}

// k_entries' long-phase LDS: the replicated X^128 table and g_tab.lt, every
// global load issued before the first LDS store (one L2 round trip for the
// whole refill instead of one per table: 5.5 -> ~2 us per launch).
__device__ __forceinline__ void fill_long(uint8_t* lds);

// words % 4 == 0; src and lds + off 16-byte aligned.
__device__ __forceinline__ void fill_plain(uint8_t* lds, uint32_t off, const uint32_t* src,
                                           uint32_t words)
{
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* dst = reinterpret_cast<uint4*>(lds + off);
    const uint32_t n = words / 4;
    constexpr int kU = 9;
    for (uint32_t base = threadIdx.x; base < n; base += kU * blockDim.x) {
        uint4 v[kU];
#pragma unroll
        for (int j = 0; j < kU; j++) {
            const uint32_t i = base + j * blockDim.x;
            v[j] = s[i < n ? i : 0];
        }
#pragma unroll
        for (int j = 0; j < kU; j++) {
            const uint32_t i = base + j * blockDim.x;
            if (i < n)
                dst[i] = v[j];
        }
    }
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
#if RAMCRC_ASM_XOR3
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return a ^ b ^ c;
#endif
}

// Per-lane constant for table k: [byte0 = bank offset (+128 for odd k),
// byte2 = region].
__device__ __forceinline__ uint32_t lane_reg(int k, int lane)
{
    return (uint32_t(k >> 1) << 16) | (uint32_t(k & 1) << 7) | (uint32_t(lane & 31) << 2);
}

// v_perm_b32 selector: dst.b0 = lanereg.b0, dst.b1 = u.byte(k), dst.b2 =
// lanereg.b2, dst.b3 = 0.  (sel 0-3 pick the 2nd operand's bytes, 4-7 the
// 1st operand's, 0x0C yields 0x00.)
template <int k>
__device__ __forceinline__ uint32_t rep_addr(uint32_t u, uint32_t lr)
{
    return __builtin_amdgcn_perm(u, lr, 0x0C020000u | ((4u + k) << 8));
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct RepOp {
    uint32_t lr0, lr1, lr2, lr3;
    __device__ explicit RepOp(int lane)
        : lr0(lane_reg(0, lane)), lr1(lane_reg(1, lane)), lr2(lane_reg(2, lane)),
          lr3(lane_reg(3, lane))
    {
    }
    // X^stride(u) ^ w through the replicated tables.  The four lookups are
    // consumed by two 3-input XORs, v_bitop3_b32 0x96 (inline asm so that hipcc waits once for all
    // four LDS reads instead of chaining 2-input XORs behind one wait each).
    __device__ __forceinline__ uint32_t apply(const uint8_t* lds, uint32_t u, uint32_t w) const
    {
        const uint32_t a = *reinterpret_cast<const uint32_t*>(lds + rep_addr<0>(u, lr0));
        const uint32_t b = *reinterpret_cast<const uint32_t*>(lds + rep_addr<1>(u, lr1));
        const uint32_t c = *reinterpret_cast<const uint32_t*>(lds + rep_addr<2>(u, lr2));
        const uint32_t d = *reinterpret_cast<const uint32_t*>(lds + rep_addr<3>(u, lr3));
        return xor3(xor3(a, b, w), c, d);
    }
    // One Horner step of the four word accumulators, issued as k_chunks' loop
    // runs it: the 16 table reads back to back, one wait, then the 8 XORs, so
    // a step costs one LDS round trip.  (Under k_entries' register pressure
    // hipcc otherwise interleaves the four lookup groups behind a wait each:
    // four round trips per step.)  The empty asm takes every read result at
    // once, so no XOR can be scheduled between the reads.
    __device__ __forceinline__ void apply4(const uint8_t* lds, uint32_t& u0, uint32_t& u1,
                                           uint32_t& u2, uint32_t& u3, const u32x4& w) const;
};

// X^d(v) through a plain (non-replicated) 4 KiB table at LDS byte offset off.
__device__ __forceinline__ uint32_t plain_apply(const uint8_t* lds, uint32_t off, uint32_t v)
{
    const uint32_t* t = reinterpret_cast<const uint32_t*>(lds + off);
    return t[v & 0xFF] ^ t[256 + ((v >> 8) & 0xFF)] ^ t[512 + ((v >> 16) & 0xFF)] ^
           t[768 + (v >> 24)];
}

__device__ __forceinline__ uint32_t mulmod_dev(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        p ^= (a & (0x80000000u >> i)) ? b : 0u;
        b = (b >> 1) ^ ((b & 1u) ? ramcrc::kPoly : 0u);
    }
    return p;
}

// Same product, Horner over the bits of a (highest power first): one running
// register, for call sites where register pressure matters more than latency.
__device__ __forceinline__ uint32_t mulmod_horner(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
#pragma unroll
    for (int j = 0; j < 32; j++) {
        const uint32_t ma = uint32_t(int32_t(a << (31 - j)) >> 31);   // coefficient of x^(31-j)
        const uint32_t mp = 0u - (p & 1u);
        p = (p >> 1) ^ (mp & ramcrc::kPoly) ^ (ma & b);
    }
    return p;
}

// x^(8 * 1024 * t) for t < 2^32 block units.
__device__ __forceinline__ uint32_t xpow_blocks(uint64_t t)
{
    uint32_t r = ramcrc::kOne;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t b = uint32_t(t >> (8 * j)) & 0xFF;
        if (b)
            r = (r == ramcrc::kOne) ? g_tab.xblk[j][b] : mulmod_dev(r, g_tab.xblk[j][b]);
    }
    return r;
}

// Mask a 4-byte word at absolute address a to the bytes inside [S, E) and XOR
// in the initial state at its byte position (bytes S..S+3).
__device__ __forceinline__ uint32_t fix_word(uint32_t w, uint64_t a, uint64_t S, uint64_t E,
                                             uint32_t init)
{
    // Branch-free.  ds/de: byte offsets of S and E from this word, clamped.
    const int64_t ds64 = int64_t(S - a), de64 = int64_t(E - a);
    const int ds = ds64 < -8 ? -8 : (ds64 > 8 ? 8 : int(ds64));
    const int de = de64 < -8 ? -8 : (de64 > 8 ? 8 : int(de64));
    const int lo = min(max(ds, 0), 4), hi = min(max(de, 0), 4);
    const uint32_t mhi = uint32_t((1ull << (8 * hi)) - 1);
    const uint32_t mlo = uint32_t((1ull << (8 * lo)) - 1);
    w &= mhi & ~mlo;
    // init occupies bytes S..S+3; word byte q holds init byte q - ds
    const int dd = -ds;   // a - S
    const uint32_t inj = uint32_t((uint64_t(init) << 24) >> (24 + 8 * (dd < -3 ? -3 : (dd > 3 ? 3 : dd))));
    return w ^ ((dd > -4 && dd < 4) ? inj : 0u);
}

// Wave-uniform 64-bit value into scalar registers.  (The builtin returns a
// signed int: each half goes through uint32_t, or the low half would
// sign-extend into the high one.)
__device__ __forceinline__ uint64_t rfl64(uint64_t v)
{
    const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(v)));
    const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(v >> 32)));
    return (uint64_t(hi) << 32) | lo;
}

// Explicit global address space: generic (flat_*) loads would also count in
// lgkmcnt and serialise against the LDS table lookups.
typedef const __attribute__((address_space(1))) u32x4 gu32x4;
typedef const __attribute__((address_space(1))) uint8_t gu8;

__device__ __forceinline__ const gu32x4* gptr16(uint64_t addr)
{
    return (const gu32x4*)addr;
}

__device__ __forceinline__ u32x4 load16(uint64_t addr) { return *gptr16(addr); }

// The 4 bytes at a (any alignment; a + 8 rounded down to 4 stays inside the
// buffer): two aligned dword loads and one byte funnel shift.
__device__ __forceinline__ uint32_t load_u32_any(uint64_t a)
{
    typedef const __attribute__((address_space(1))) uint32_t g32;
    const uint64_t b = a & ~uint64_t(3);
    const uint32_t w0 = *reinterpret_cast<g32*>(b), w1 = *reinterpret_cast<g32*>(b + 4);
    return __builtin_amdgcn_alignbyte(w1, w0, uint32_t(a) & 3);
}

#ifndef RAMCRC_STEP_BATCH
#define RAMCRC_STEP_BATCH 1
#endif
__device__ __forceinline__ void RepOp::apply4(const uint8_t* lds, uint32_t& u0, uint32_t& u1,
                                              uint32_t& u2, uint32_t& u3, const u32x4& w) const
{
#if RAMCRC_STEP_BATCH
    auto rd = [&](uint32_t a) { return *reinterpret_cast<const uint32_t*>(lds + a); };
    uint32_t a0 = rd(rep_addr<0>(u0, lr0)), a1 = rd(rep_addr<1>(u0, lr1));
    uint32_t a2 = rd(rep_addr<2>(u0, lr2)), a3 = rd(rep_addr<3>(u0, lr3));
    uint32_t b0 = rd(rep_addr<0>(u1, lr0)), b1 = rd(rep_addr<1>(u1, lr1));
    uint32_t b2 = rd(rep_addr<2>(u1, lr2)), b3 = rd(rep_addr<3>(u1, lr3));
    uint32_t c0 = rd(rep_addr<0>(u2, lr0)), c1 = rd(rep_addr<1>(u2, lr1));
    uint32_t c2 = rd(rep_addr<2>(u2, lr2)), c3 = rd(rep_addr<3>(u2, lr3));
    uint32_t d0 = rd(rep_addr<0>(u3, lr0)), d1 = rd(rep_addr<1>(u3, lr1));
    uint32_t d2 = rd(rep_addr<2>(u3, lr2)), d3 = rd(rep_addr<3>(u3, lr3));
    asm volatile(""
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3),
                   "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3));
    u0 = xor3(xor3(a0, a1, w.x), a2, a3);
    u1 = xor3(xor3(b0, b1, w.y), b2, b3);
    u2 = xor3(xor3(c0, c1, w.z), c2, c3);
    u3 = xor3(xor3(d0, d1, w.w), d2, d3);
#else
    u0 = apply(lds, u0, w.x);
    u1 = apply(lds, u1, w.y);
    u2 = apply(lds, u2, w.z);
    u3 = apply(lds, u3, w.w);
#endif
}

// ------------------------------------------------------------ descriptors
struct BatchDesc {
    const uint8_t* base;     // d_base
    const uint64_t* off;     // general mode
    const uint64_t* len;     // general mode
    uint64_t seg_bytes;      // uniform mode; segment stride in record mode
    uint64_t n;              // buffers (record mode: table capacity)
    const uint32_t* init;    // nullable
    uint32_t* out;
    uint32_t flags;
    uint32_t cshift;         // log2 chunk bytes of this launch (k_chunks/k_combine)
    const u32x4* rec;        // record mode: ramcrc_seg_entry table
    const uint64_t* n_dev;   // record mode: live entry count (device), <= n
    const u32x4* seg_status; // record mode: ramcrc_seg_status per segment (walk result)
    ramcrc_seg_status* vstat; // record mode, nullable: k_entries compares each object's CRC
                              // with its stored checksum (the 4 bytes before S, loaded beside
                              // its head) and counts mismatches in vstat[segment].bad_objects
};

// Buffer addressing modes.
//   kSegAligned: segment i = base + i*seg_bytes, base and seg_bytes multiples
//                of the chunk size -> chunk g maps to (g / per, g % per).
//   kSegUniform: same geometry, any alignment -> goes through the plan.
//   kTable:      buffer i = base + off[i], len[i] -> goes through the plan.
//   kRecords:    buffer i = the object of segment-walk record i: bytes
//                [4, length) of its payload (Object::computeChecksum,
//                src/Object.cc:805-819).  Inactive: records that are not
//                objects, objects shorter than their header or running past
//                the segment (kRecOverlong), and every record of a segment
//                whose metadata check failed (RecoverySegmentBuilder::build
//                stops there, src/RecoverySegmentBuilder.cc:61-203).
//   kObjects:    buffer i = bytes [4, len[i]) of the serialized object at
//                base + off[i] (Object::computeChecksum on the write path,
//                Object::assembleForLog, src/Object.cc:213-238); objects
//                shorter than their 24-byte header are inactive.
enum Mode { kSegAligned = 0, kSegUniform = 1, kTable = 2, kRecords = 3, kObjects = 4 };

constexpr uint32_t kObjHeaderBytes = 24;     // Object::Header, src/Object.h:137-182
constexpr uint32_t kTombHeaderBytes = 32;    // ObjectTombstone::Header, src/Object.h:285-338
constexpr uint32_t kSafeVersionBytes = 12;   // ObjectSafeVersion::Header, src/Object.h:402-427
constexpr uint32_t kPrepHeaderBytes = 32;    // PreparedOp::Header, src/PreparedOp.h:63-100
constexpr uint32_t kPrepTombBytes = 44;      // PreparedOpTombstone::Header, src/PreparedOp.h:142-185
constexpr uint32_t kTxDecisionHeaderBytes = 48;  // TxDecisionRecord::Header, src/TxDecisionRecord.h:62-128
constexpr uint32_t kTxPlistHeaderBytes = 24;     // ParticipantList::Header, src/ParticipantList.h:81-113
constexpr uint32_t kRecOverlong = 0x100;   // record header bit: payload past the capacity

template <int kMode>
__device__ __forceinline__ uint64_t entry_count(const BatchDesc& d)
{
    if (kMode == kRecords) {
        const uint64_t live = *d.n_dev;
        return live < d.n ? live : d.n;
    }
    return d.n;
}

// Header bytes a record of `type` must hold to be checked; 0 = not checked.
// (a nibble per type of bytes / 4 in one 64-bit constant: branch-free, and
// it can never become a lookup table in memory on a per-record path)
constexpr uint64_t replay_header_nibbles()
{
    const uint32_t t[][2] = {{RAMCRC_LOG_ENTRY_TYPE_OBJ, kObjHeaderBytes},
                             {RAMCRC_LOG_ENTRY_TYPE_OBJTOMB, kTombHeaderBytes},
                             {RAMCRC_LOG_ENTRY_TYPE_SAFEVERSION, kSafeVersionBytes},
                             {RAMCRC_LOG_ENTRY_TYPE_PREP, kPrepHeaderBytes + kObjHeaderBytes},
                             {RAMCRC_LOG_ENTRY_TYPE_PREPTOMB, kPrepTombBytes},
                             {RAMCRC_LOG_ENTRY_TYPE_TXDECISION, kTxDecisionHeaderBytes},
                             {RAMCRC_LOG_ENTRY_TYPE_TXPLIST, kTxPlistHeaderBytes}};
    uint64_t v = 0;
    for (const auto& e : t)
        v |= uint64_t(e[1] / 4) << (4 * e[0]);
    return v;
}
constexpr uint64_t kReplayHeaderNibbles = replay_header_nibbles();
static_assert(kObjHeaderBytes % 4 == 0 && kTombHeaderBytes % 4 == 0 && kSafeVersionBytes % 4 == 0 &&
                  kPrepTombBytes % 4 == 0 && kTxDecisionHeaderBytes % 4 == 0 && kTxPlistHeaderBytes % 4 == 0 &&
                  (kPrepHeaderBytes + kObjHeaderBytes) / 4 < 16 && kTxDecisionHeaderBytes / 4 < 16 &&
                  RAMCRC_LOG_ENTRY_TYPE_TXPLIST < 16,
              "replay header sizes: one nibble of bytes / 4 per type below 16");

__device__ __forceinline__ uint32_t replay_header_bytes(uint32_t type)
{
    return type < 16 ? 4 * uint32_t((kReplayHeaderNibbles >> (4 * type)) & 15) : 0u;
}

// The object bytes [S, E) of walk record r ({segment, offset, length,
// header}); false (S == E) unless it is an object of a segment that passed.
// (seg_st: the flags word of the record's segment status)
__device__ __forceinline__ bool record_range_st(const BatchDesc& d, const u32x4& r, uint32_t seg_st,
                                                uint64_t& S, uint64_t& E)
{
    const uint64_t payload = reinterpret_cast<uint64_t>(d.base) + uint64_t(r.x) * d.seg_bytes + r.y + 1 +
                             ((r.w >> 6) & 3) + 1;
    const bool obj = (r.w & (0x3f | kRecOverlong)) == RAMCRC_LOG_ENTRY_TYPE_OBJ && r.z >= kObjHeaderBytes &&
                     (seg_st & RAMCRC_SEG_OK);
    S = payload + 4;
    E = obj ? payload + r.z : S;
    return obj;
}

__device__ __forceinline__ bool record_range(const BatchDesc& d, const u32x4& r, uint64_t& S, uint64_t& E)
{
    return record_range_st(d, r, d.seg_status[r.x].x, S, E);
}

// [S, E) of buffer i; false for an inactive record (then S == E).
template <int kMode>
__device__ __forceinline__ bool buffer_range(const BatchDesc& d, uint64_t i, uint64_t& S,
                                             uint64_t& E)
{
    if (kMode == kRecords) {
        return record_range(d, d.rec[i], S, E);
    } else if (kMode == kObjects) {
        const uint64_t o = reinterpret_cast<uint64_t>(d.base) + d.off[i];
        const uint64_t L = d.len[i];
        S = o + 4;
        E = L >= kObjHeaderBytes ? o + L : S;
        return L >= kObjHeaderBytes;
    } else if (kMode != kTable) {
        S = reinterpret_cast<uint64_t>(d.base) + i * d.seg_bytes;
        E = S + d.seg_bytes;
    } else {
        S = reinterpret_cast<uint64_t>(d.base) + d.off[i];
        E = S + d.len[i];
    }
    return true;
}

__device__ __forceinline__ uint64_t chunk_count(uint64_t S, uint64_t E, uint32_t cshift)
{
    return ((E - 1) >> cshift) - (S >> cshift) + 1;
}

// Context status word (ramcrc_ctx_status / ramcrc_ctx_check).
constexpr uint32_t kStatusRefused = 1u;   // this launch's chunk plan overflowed (k_chunks)
constexpr uint32_t kStatusSticky = 2u;    // some launch wrote no outputs since the last check
constexpr uint32_t kStatusBins = 4u;      // a binned launch found its layout inconsistent

struct Plan {
    uint64_t* local;      // per entry: exclusive prefix of chunk counts within its group
    uint64_t* group_pref;  // per group of kThreads entries, exclusive prefix; [ngroups] = total
    uint64_t ngroups;
    uint32_t* partials;
    uint64_t partials_cap;
    uint32_t* status;      // bit 0: this launch's partials overflow; bit 1: sticky (ramcrc_ctx_check)
    unsigned long long* ticket;   // chunk dequeue counter; zero between launches
    const uint32_t* nlarge;       // nullable: large buffers counted by this sequence's
                                  // k_bin_count; 0 -> every plan kernel exits at once
};

__device__ __forceinline__ bool plan_empty(const Plan& pl) { return pl.nlarge && *pl.nlarge == 0; }

__device__ __forceinline__ bool is_large(uint64_t len) { return len >= kLargeMin; }

// ------------------------------------------------------------ k_chunks
// Scan one chunk [lo, hi) of buffer [S, E) as 1 KiB blocks; returns (in every
// lane) raw(0, zero-padded chunk) relative to the chunk's 1 KiB-aligned end.
__device__ __forceinline__ uint32_t scan_chunk(const uint8_t* lds, const RepOp& op, int lane,
                                               uint64_t S, uint64_t E, uint32_t init,
                                               uint64_t lo, uint64_t hi)
{
    uint32_t u0 = 0, u1 = 0, u2 = 0, u3 = 0;
    uint64_t first = lo & ~uint64_t(kBlock - 1);
    const uint64_t end = (hi + kBlock - 1) & ~uint64_t(kBlock - 1);

    auto step = [&](const u32x4& w) {
        u0 = op.apply(lds, u0, w.x);
        u1 = op.apply(lds, u1, w.y);
        u2 = op.apply(lds, u2, w.z);
        u3 = op.apply(lds, u3, w.w);
    };
    auto special = [&](uint64_t blk) {
        const uint64_t a = blk + uint64_t(lane) * 16;
        u32x4 w = {0u, 0u, 0u, 0u};
        if (a < E && a + 16 > S)
            w = load16(a);
        w.x = fix_word(w.x, a + 0, S, E, init);
        w.y = fix_word(w.y, a + 4, S, E, init);
        w.z = fix_word(w.z, a + 8, S, E, init);
        w.w = fix_word(w.w, a + 12, S, E, init);
        step(w);
    };

    // Head blocks that hold bytes before S or the injected init (S..S+3),
    // and any block cut by E.
    while (first < end && (first < S + 4 || first + kBlock > E)) {
        special(first);
        first += kBlock;
    }
    uint64_t fast_end = end;
    if (first < end && end > E)
        fast_end = end - kBlock;

    // Full blocks: two register groups of kUnroll blocks ping-pong so that one
    // group is always in flight while the other is hashed.  Loads past the
    // range are clamped to the last block (a harmless cached re-read).
    const uint64_t nf = (fast_end - first) / kBlock;
    if (nf > 0) {
        // Buffer loads: the chunk base lives in an SGPR descriptor and the
        // block offset in soffset, so each load costs no address VGPRs.
        const uint32_t lo_w = __builtin_amdgcn_readfirstlane(uint32_t(first));
        const uint32_t hi_w = __builtin_amdgcn_readfirstlane(uint32_t(first >> 32));
        const uint32_t nrec = __builtin_amdgcn_readfirstlane(uint32_t(nf * kBlock));
        void* basep = reinterpret_cast<void*>((uint64_t(hi_w) << 32) | lo_w);
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc(basep, (short)0, int(nrec), 0x00020000);
        const uint32_t voff = uint32_t(lane) * 16;
        auto ldb = [&](uint64_t b) -> u32x4 {
            b = b < nf ? b : nf - 1;
            return __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, uint32_t(b * kBlock),
                                                         2 /* nt */);
        };
        u32x4 A[kUnroll], B[kUnroll];
#pragma unroll
        for (int j = 0; j < kUnroll; j++)
            A[j] = ldb(j);
        uint64_t i = 0;
        for (; i + 2 * kUnroll <= nf; i += 2 * kUnroll) {
#pragma unroll
            for (int j = 0; j < kUnroll; j++)
                B[j] = ldb(i + kUnroll + j);
            // keep the whole group's loads issued ahead of the hashing (the
            // scheduler would otherwise sink them next to their uses)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < kUnroll; j++)
                step(A[j]);
#pragma unroll
            for (int j = 0; j < kUnroll; j++)
                A[j] = ldb(i + 2 * kUnroll + j);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < kUnroll; j++)
                step(B[j]);
        }
        // fewer than 2*kUnroll blocks left; A holds blocks i .. i+kUnroll-1
#pragma unroll
        for (int j = 0; j < kUnroll; j++)
            if (i + j < nf)
                step(A[j]);
        if (i + kUnroll < nf) {
#pragma unroll
            for (int j = 0; j < kUnroll; j++)
                B[j] = ldb(i + kUnroll + j);
#pragma unroll
            for (int j = 0; j < kUnroll; j++)
                if (i + kUnroll + j < nf)
                    step(B[j]);
        }
    }
    if (fast_end < end)
        special(fast_end);

    // Fold: in-lane with X^4, then across lanes with X^16 .. X^512.
    uint32_t y = plain_apply(lds, kCombOff, u0) ^ u1;
    y = plain_apply(lds, kCombOff, y) ^ u2;
    y = plain_apply(lds, kCombOff, y) ^ u3;
    uint32_t z = plain_apply(lds, kCombOff, y);
#pragma unroll
    for (int lvl = 0; lvl < 6; lvl++) {
        const uint32_t other = __shfl_xor(z, 1 << lvl, kWaveSize);
        const bool upper = (lane >> lvl) & 1;
        const uint32_t lower_v = upper ? other : z;
        const uint32_t upper_v = upper ? z : other;
        z = plain_apply(lds, kCombOff + (1 + lvl) * 4096, lower_v) ^ upper_v;
    }
    return z;
}

// A record k_obj_compare has work for: a checked type that is not a readable
// object below the large-buffer split (those are compared beside the scan).
__device__ __forceinline__ bool replay_other(const u32x4& r)
{
    const uint32_t type = r.w & 0x3f;
    const uint32_t hdr = replay_header_bytes(type);
    const bool readable = r.z >= hdr && !(r.w & kRecOverlong);
    return hdr != 0 && !(type == RAMCRC_LOG_ENTRY_TYPE_OBJ && readable && !is_large(uint64_t(r.z) - 4));
}



// Locate (entry, chunk) for global chunk index g in general mode.
__device__ __forceinline__ void plan_locate(const Plan& pl, uint64_t n, uint64_t g, uint64_t& entry,
                                            uint64_t& k)
{
    // group: last b with group_pref[b] <= g
    uint64_t lo = 0, hi = pl.ngroups;   // invariant: group_pref[lo] <= g < group_pref[hi]
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (pl.group_pref[mid] <= g) lo = mid; else hi = mid;
    }
    const uint64_t gbase = pl.group_pref[lo];
    uint64_t a = lo * kThreads, b = a + kThreads;
    if (b > n) b = n;
    // last entry j in [a, b) with gbase + local[j] <= g
    uint64_t l2 = a, h2 = b;
    while (h2 - l2 > 1) {
        const uint64_t mid = (l2 + h2) >> 1;
        if (gbase + pl.local[mid] <= g) l2 = mid; else h2 = mid;
    }
    entry = l2;
    k = g - gbase - pl.local[l2];
}

template <int kMode>
__global__ __launch_bounds__(kThreads, 1) void k_chunks(BatchDesc d, Plan pl, uint64_t per_seg)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsChunks];
    if (kMode != kSegAligned && plan_empty(pl))
        return;   // no buffer of this batch is large: skip the table fill too
    fill_replicated(lds, g_tab.stride_large);
    fill_plain(lds, kCombOff, &g_tab.comb[0].t[0][0], 7 * 1024);
    __syncthreads();

    const int lane = threadIdx.x & (kWaveSize - 1);
    const RepOp op(lane);
    const uint64_t wave = uint64_t(blockIdx.x) * kWavesPerGroup +
                          __builtin_amdgcn_readfirstlane(threadIdx.x / kWaveSize);
    const uint64_t nwaves = uint64_t(gridDim.x) * kWavesPerGroup;
    const uint64_t total = kMode == kSegAligned ? per_seg * d.n : pl.group_pref[pl.ngroups];
    if (total > pl.partials_cap) {
        if (wave == 0 && lane == 0)
            atomicOr(pl.status, 3u);   // refused: this launch, and sticky until checked
        return;
    }
    // Work: chunk g -> (buffer i, chunk k).  Dynamic: lane 0 takes tickets
    // from a device counter (one ahead, so the atomic's latency hides behind
    // a chunk); static: grid stride.
    auto take = [&]() -> uint64_t {
        uint64_t t = 0;
        if (lane == 0)
            t = atomicAdd(pl.ticket, 1ull);
        return rfl64(t);
    };
    uint64_t g = kDynamic ? take() : wave;
    while (g < total) {
        const uint64_t gnext = kDynamic ? take() : g + nwaves;
        uint64_t i, k;
        if (kMode == kSegAligned) {
            i = g / per_seg;
            k = g - i * per_seg;
        } else {
            plan_locate(pl, d.n, g, i, k);
        }
        uint64_t S, E;
        buffer_range<kMode>(d, i, S, E);
        const uint32_t init = d.init ? d.init[i] : 0xFFFFFFFFu;
        const uint64_t cs = S >> d.cshift;
        const uint64_t c_lo = (cs + k) << d.cshift;
        const uint64_t lo = c_lo > S ? c_lo : S;
        const uint64_t c_hi = c_lo + (1ull << d.cshift);
        const uint64_t hi = c_hi < E ? c_hi : E;
        const uint32_t r = scan_chunk(lds, op, lane, S, E, init, lo, hi);
        if (lane == 0)
            pl.partials[g] = r;
        g = gnext;
    }
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src)
{
    const uint32_t lo = __shfl(uint32_t(v), src, kWaveSize);
    const uint32_t hi = __shfl(uint32_t(v >> 32), src, kWaveSize);
    return (uint64_t(hi) << 32) | lo;
}

// ------------------------------------------------------------ k_combine
// Merge the chunk partials of large buffer i (one wave): lane k multiplies
// partial k by x^(8 * 1024 * t), t = its distance to the padded end in 1 KiB
// units; XOR across lanes; x^(-8 pad) removes the padding of the last block.
template <int kMode>
__device__ __forceinline__ void combine_one(const BatchDesc& d, const Plan& pl, uint64_t per_seg,
                                            uint64_t i, uint64_t S, uint64_t E, int lane)
{
    const uint64_t g0 = kMode == kSegAligned ? i * per_seg
                                             : pl.group_pref[i / kThreads] + pl.local[i];
    const uint64_t cnt = chunk_count(S, E, d.cshift);
    const uint64_t cs = S >> d.cshift;
    const uint64_t pend = (E + kBlock - 1) & ~uint64_t(kBlock - 1);
    uint32_t R = 0;
    for (uint64_t k = lane; k < cnt; k += kWaveSize) {
        const uint32_t r = pl.partials[g0 + k];
        const uint64_t ek = (k + 1 == cnt) ? pend : ((cs + k + 1) << d.cshift);
        const uint64_t t = (pend - ek) / kBlock;
        R ^= t ? mulmod_dev(r, xpow_blocks(t)) : r;
    }
#pragma unroll
    for (int lvl = 0; lvl < 6; lvl++)
        R ^= __shfl_xor(R, 1 << lvl, kWaveSize);
    const uint32_t pad = uint32_t(pend - E);
    if (pad)
        R = mulmod_dev(R, g_tab.xinv[pad]);
    if (lane == 0)
        d.out[i] = (d.flags & RAMCRC_FINALIZE) ? ~R : R;
}

// kWide = false: one wave per buffer (few buffers, most of them large).
// kWide = true:  one wave per 64 buffers -- each lane tests one, the wave
// merges the large ones it found -- for big tables of mostly small entries,
// where a wave per entry would cost more than the entries' own scan.
template <int kMode, bool kWide>
__global__ __launch_bounds__(256) void k_combine(BatchDesc d, Plan pl, uint64_t per_seg)
{
    const int lane = threadIdx.x & (kWaveSize - 1);
    const uint64_t wave = uint64_t(blockIdx.x) * (256 / kWaveSize) + threadIdx.x / kWaveSize;
    if (blockIdx.x == 0 && threadIdx.x == 0)
        *pl.ticket = 0;   // k_chunks of this launch is complete (same stream)
    if (kMode != kSegAligned && (plan_empty(pl) || ((*pl.status) & kStatusRefused)))
        return;   // nothing large, or k_chunks refused the launch (partials overflow)
    const uint64_t n = entry_count<kMode>(d);
    if (!kWide) {
        if (wave >= n)
            return;
        uint64_t S, E;
        buffer_range<kMode>(d, wave, S, E);
        if (is_large(E - S))   // (small ones: k_entries; inactive ones: none)
            combine_one<kMode>(d, pl, per_seg, wave, S, E, lane);
        return;
    }
    if (pl.group_pref[pl.ngroups] == 0)
        return;   // no large buffer in this launch
    // waves of 64 entries, grid-stride (capped grid, as k_plan_count)
    const uint64_t nwave = uint64_t(gridDim.x) * (256 / kWaveSize);
    for (uint64_t wv = wave; wv * kWaveSize < n; wv += nwave) {
        const uint64_t i = wv * kWaveSize + lane;
        uint64_t S = 0, E = 0;
        const bool big = i < n && buffer_range<kMode>(d, i, S, E) && is_large(E - S);
        uint64_t todo = __ballot(big);
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            combine_one<kMode>(d, pl, per_seg, wv * kWaveSize + j, shfl64(S, j), shfl64(E, j), lane);
        }
    }
}

// ------------------------------------------------------------ k_entries
// Small buffers (log entries, objects; src/ObjectManager.cc:659-669).  A
// group of 8 lanes owns one entry and reads it as 128-byte steps (lane l: 16
// bytes at A + 128 k + 16 l, A = S rounded down to 16): groups of 8 lanes
// reading 128 contiguous bytes stream at the full HBM rate on gfx950 (7.05
// TB/s measured, profiles/r01/membench_access_patterns.txt), while one lane
// per entry reaches only 2 TB/s.  Horner with X^128 per step through the
// replicated LDS tables; at the end the four slot accumulators fold with
// X^4, one GF(2) multiply by x^(8 (16 (7-l) - pad)) moves each lane's partial
// to the entry end (pad = zero bytes past E in the last step), and three
// shuffles XOR the group.  Entries are first binned by step count
// (k_bin_*) so the 8 groups of a wave finish together; bins of at most 8
// steps batch several entry octets per load round.
constexpr int kG = 8;                      // lanes per entry group
constexpr uint64_t kStep = kG * 16;        // bytes per group step
constexpr int kNB = 161;                   // step-count bins
#ifndef RAMCRC_SMALLK
#define RAMCRC_SMALLK 4
#endif
#ifndef RAMCRC_ENT_WAVES
#define RAMCRC_ENT_WAVES 16
#endif
constexpr int kEntWaves = RAMCRC_ENT_WAVES;   // k_entries: waves per workgroup (1 per CU)
constexpr int kSmallK = RAMCRC_SMALLK;     // bins 2..kSmallK: octets loaded one ahead
#ifndef RAMCRC_TINY_K
#define RAMCRC_TINY_K 4
#endif
// bins 2 .. kTinyK (entries of 2 .. kTinyK windows, e.g. objects of 129 ..
// ~500 B): the multi-window tiny phase (tiny_run_cf<true>); 1 = off (the short bins)
constexpr int kTinyK = RAMCRC_TINY_K;
static_assert(kTinyK >= 1 && kTinyK <= 7, "tiny windows: E - A (<= 128 kTinyK) fits 10 bits");

// What a walk record {segment, offset, length, header} rules out for the
// verify: bit 0, the direct one-window tiny path (a record k_obj_compare has
// work for, or an object whose bytes [4, length) span more than one 128-byte
// window -- the walk keeps segments 16-byte aligned, so the windows follow
// from the offset alone); bit 1, the direct multi-window path (anything but
// an object of 2 .. kTinyK windows); bit 2, an object of 3 or more windows.
// The fused replay call ORs this over
// every record its walk writes; unless both bits end up set the verify needs
// no binning scatter (ramcrc_replay_verify_device, k_bin_count).
constexpr uint32_t kHardAll = 3u;
__device__ __forceinline__ uint32_t replay_hard(uint32_t pos, uint32_t len, uint32_t hdr)
{
    const u32x4 r = {0u, pos, len, hdr};
    if (replay_other(r))
        return kHardAll;
    if ((hdr & (0x3f | kRecOverlong)) != RAMCRC_LOG_ENTRY_TYPE_OBJ || len < kObjHeaderBytes)
        return 0u;   // nothing to scan
    const uint32_t s16 = (pos + 1 + ((hdr >> 6) & 3) + 1 + 4) & 15;   // S mod 16
    const uint32_t steps = (s16 + (len - 4) + 127) / 128;             // entry_steps
    if (len - 4 < 4 || steps <= 1)
        return 2u;   // one window (or bytewise): the tiny path
    // (bit 2: more than two windows -- the direct multi-window path then
    // takes the general loop instead of the two-window ring)
    return steps <= 2 ? 1u : (steps <= uint32_t(kTinyK) ? 5u : kHardAll | 4u);
}
#ifndef RAMCRC_ENT_NT
#define RAMCRC_ENT_NT 1
#endif
#ifndef RAMCRC_PU
#define RAMCRC_PU 2   // A/B on the config-3 mix, 1 KiB and 4 KiB entries: 2 < 1, 3, 4, 6, 8
#endif
constexpr int kPU = RAMCRC_PU;             // ping-pong depth (pipelined bins)
#ifndef RAMCRC_TINY_TRIM
#define RAMCRC_TINY_TRIM 1   // tiny phase: 64-bit-shift head masks, saturating row bases
#endif
#ifndef RAMCRC_TINY_CF
#define RAMCRC_TINY_CF 1     // tiny phase: conflict-free column-major table (tiny_run_cf)
#endif
#ifndef RAMCRC_TINY_SAFE
#define RAMCRC_TINY_SAFE 1    // tiny_run_cf: unclamped window loads when every window of a q is page-safe
#endif
#ifndef RAMCRC_TINY_OVL
#define RAMCRC_TINY_OVL 1   // tiny phase: round 0's windows in flight while the table is built
#endif
constexpr uint32_t kNoIdx = 0xFFFFFFFFu;   // empty slot
#ifndef RAMCRC_SPLIT
#define RAMCRC_SPLIT 1   // k_entries: tiny and long phases on separate workgroups when a batch has both
#endif
#ifndef RAMCRC_SPLIT_KAPPA
#define RAMCRC_SPLIT_KAPPA 256   // a tiny window in long-phase work units, x 1024
#endif
constexpr uint64_t kSplitKappa = RAMCRC_SPLIT_KAPPA;
#ifndef RAMCRC_OCTET_COST
#define RAMCRC_OCTET_COST 4
#endif
constexpr uint64_t kOctetCost = RAMCRC_OCTET_COST;   // per-octet overhead in step units (work split)
#ifndef RAMCRC_AGE_SKEW
#define RAMCRC_AGE_SKEW 140
#endif
#ifndef RAMCRC_AGE_SKEW_REC
#define RAMCRC_AGE_SKEW_REC 80
#endif
// long bins: share of a wave of age rank r (slot / 4) in 1/2000 of an equal
// share: 2000 + skew * (3 - 2 r), i.e. +-21 % at the outer ranks for skew
// 140.  Same-box A/B (profiles/r03/long/ab_skew*.txt): plain batches gain up
// to skew 120-160 (config-3 mix +4 % over 80), replay verify (records mode)
// loses from 120 on (-3 %), so records mode keeps 80.
constexpr int kAgeSkew = RAMCRC_AGE_SKEW, kAgeSkewRec = RAMCRC_AGE_SKEW_REC;
__host__ __device__ constexpr uint64_t age_weight(uint32_t r, int skew)
{
    return uint64_t(2000 + skew * (3 - 2 * int(r)));
}
static_assert(RAMCRC_ENT_WAVES % 4 == 0, "age ranks of four waves");
#ifndef RAMCRC_BIN_PER
#define RAMCRC_BIN_PER 4
#endif
constexpr int kBinPer = RAMCRC_BIN_PER;    // entries per thread per tile (count/scatter)
#ifndef RAMCRC_BIN_ONE
#define RAMCRC_BIN_ONE 1   // k_bin_one for batches of <= 1 tile per workgroup (A/B: 0)
#endif
#ifndef RAMCRC_BIN_RESCUE
#define RAMCRC_BIN_RESCUE 1   // the guarded scatter after every k_bin_one (A/B only: 0 = none,
                              // an aborted k_bin_one then leaves its batch unbinned)
#endif
#ifndef RAMCRC_BIN_SLICES
#define RAMCRC_BIN_SLICES 8   // k_bin_one: histogram copies (workgroup i adds to copy i % 8: its XCD's)
#endif
constexpr int kBinSlices = RAMCRC_BIN_SLICES;
#ifndef RAMCRC_COUNT_PF
#define RAMCRC_COUNT_PF 1   // k_bin_count, records: next tile's records in flight (A/B: 0)
#endif
#ifndef RAMCRC_BIN_WGS_PER_CU
#define RAMCRC_BIN_WGS_PER_CU 8
#endif
constexpr uint64_t kBinWgsPerCu = RAMCRC_BIN_WGS_PER_CU;   // binning grid cap per CU

#ifndef RAMCRC_TINY_PF
// tiny rounds: the next round's windows loaded into registers while this one
// is hashed -- 0 never, 1 always, 2 records batches only (replay)
#define RAMCRC_TINY_PF 2
#endif
#ifndef RAMCRC_TINY_LSEL
// tiny windows: per-lane v_perm selectors instead of a v_alignbyte per dword
// -- 0 never, 1 always, 2 where the round loop has no register prefetch
#define RAMCRC_TINY_LSEL 2
#endif
#ifndef RAMCRC_TINY_DM
#define RAMCRC_TINY_DM 1   // records batches whose objects all span 2 .. kTinyK windows: no scatter
#endif
#ifndef RAMCRC_TINY_M2
#define RAMCRC_TINY_M2 1   // tiny_multi: bin 2 with two-window buffers and a ring of four
#endif
#ifndef RAMCRC_TINY_REGEO
#define RAMCRC_TINY_REGEO 1   // prefetching tiny loop: window geometry re-swizzled from the owner
#endif
#ifndef RAMCRC_TINY_T3
#define RAMCRC_TINY_T3 1   // tiny windows: tail masks on dword 3 only when every window ends at >= 96
#endif
#ifndef RAMCRC_TINY_MED3
#define RAMCRC_TINY_MED3 1   // tiny window tail clamp as one v_med3 per dword
#endif
#ifndef RAMCRC_TINY_HM
#define RAMCRC_TINY_HM 1   // 8-lane group XOR: third step by DPP row_half_mirror (0: ds_swizzle)
#endif
// XOR of the 8 lanes of a lane group (lanes 8g .. 8g + 7), in every lane:
// quad permutes for lane ^ 1 and ^ 2; then every lane of a quad holds the
// quad's XOR, and row_half_mirror (lane i of a half-row reads lane 7 - i)
// brings in the other quad's -- a VALU op, where the ds_swizzle it replaces
// was an LDS-pipe round trip per window.
__device__ __forceinline__ uint32_t group8_xor_all(uint32_t R)
{
    R ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(R), 0xB1, 0xF, 0xF, false));   // lane ^ 1
    R ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(R), 0x4E, 0xF, 0xF, false));   // lane ^ 2
#if RAMCRC_TINY_HM
    R ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(R), 0x141, 0xF, 0xF, false));  // row_half_mirror
#else
    R ^= uint32_t(__builtin_amdgcn_ds_swizzle(int(R), 0x1F | (4 << 10)));           // lane ^ 4
#endif
    return R;
}

constexpr uint32_t kTinyRow0 = 3;            // tiny phase: row of distance m is m + 3
constexpr uint32_t kLdsTiny = 132 * 1024;    // tiny phase: X^m(byte), m = -3..128
static_assert(kLdsTiny <= kLdsEntries, "k_entries' LDS holds the tiny phase's table");

__device__ __forceinline__ void fill_long(uint8_t* lds)
{
    constexpr uint32_t kRepItems = 4 * 256 * 8;   // as fill_replicated
    constexpr uint32_t kPlain = sizeof(DeviceTables::LongTabs) / 16;
    constexpr uint32_t kR = kRepItems / kEntWaves / kWaveSize;   // 8 per thread at 1024 threads
    constexpr uint32_t kP = (kPlain + kEntWaves * kWaveSize - 1) / (kEntWaves * kWaveSize);
    static_assert(kRepItems % (kEntWaves * kWaveSize) == 0, "rep items per thread");
    const OpTable& op = g_tab.stride_small;
    const uint4* src = reinterpret_cast<const uint4*>(&g_tab.lt);
    uint32_t v[kR];
    uint4 w[kP];
#pragma unroll
    for (uint32_t j = 0; j < kR; j++) {
        const uint32_t idx = threadIdx.x + j * blockDim.x;
        v[j] = op.t[idx >> 11][(idx >> 3) & 255];
    }
#pragma unroll
    for (uint32_t j = 0; j < kP; j++) {
        const uint32_t i = threadIdx.x + j * blockDim.x;
        w[j] = src[i < kPlain ? i : 0];
    }
#pragma unroll
    for (uint32_t j = 0; j < kR; j++) {
        const uint32_t idx = threadIdx.x + j * blockDim.x;
        const uint32_t k = idx >> 11, bv = (idx >> 3) & 255, q = idx & 7;
        const uint32_t off = (k >> 1) * 65536 + bv * 256 + (k & 1) * 128 + q * 16;
        *reinterpret_cast<uint4*>(lds + off) = make_uint4(v[j], v[j], v[j], v[j]);
    }
    uint4* dst = reinterpret_cast<uint4*>(lds + kX4Off);
#pragma unroll
    for (uint32_t j = 0; j < kP; j++) {
        const uint32_t i = threadIdx.x + j * blockDim.x;
        if (i < kPlain)
            dst[i] = w[j];
    }
}

// The counters a binning sequence (k_bin_count -> k_bin_scatter -> k_entries)
// accumulates come in two copies selected by the sequence's parity: sequence
// p counts into copy p while its k_bin_count zeroes copy p ^ 1 for the next
// sequence.  The host flips the parity only once k_bin_count is enqueued, so a
// sequence abandoned after that point (a failed later launch) leaves the next
// one a clean copy; nothing depends on a later kernel of the same sequence
// having run.  k_entries re-checks the layout against what the scatter wrote
// (cursor == count for every bin) before it touches a sorted slot.
struct BinCounters {
    uint64_t cursor[kNB];     // scatter cursors, relative to start
    uint32_t hist[kNB];       // entry counts
    uint32_t nlarge;          // large buffers the count pass left to k_chunks (skip_large)
    uint32_t ninact;          // inactive records (records mode: not checked here)
    uint32_t nother;          // records mode: records k_obj_compare has work for (replay_other)
    uint32_t arrive;          // k_bin_one: workgroups past their histogram atomics
    uint32_t flag;            // k_bin_one: 0, then kBinGo (last arrival) or kBinAbort (a stall)
    uint32_t wide;            // fused replay, direct multi-window path: some object of 3 .. kTinyK windows
    uint32_t hs[kBinSlices][kNB];   // k_bin_one: histogram per slice of workgroups
    uint32_t arr[kBinSlices];       // k_bin_one: arrivals per slice
};

constexpr uint32_t kBinGo = 1, kBinAbort = 2;   // BinCounters::flag: k_bin_one's vote

struct BinTable {
    uint64_t start[kNB];      // first sorted slot of the bin (multiple of 8)
    uint64_t count[kNB];      // entries in the bin
    uint64_t items[kNB + 1];  // exclusive prefix of octets * kmax: work units
    uint64_t kcost[kNB];      // steps charged per octet of the bin (its largest step count)
    uint64_t direct_n;        // nonzero: every entry of this kTable batch is tiny; the tiny
                              // phase reads the caller's table in place (nothing scattered)
    uint64_t direct_multi;    // nonzero: every active record of this records batch is an
                              // object of 2 .. kTinyK windows (bin 2 holds them all); the
                              // multi-window tiny phase reads the record table in place
    uint64_t direct_multi_k2; // ... and none spans more than two windows (the two-window ring)
    BinCounters ctr[2];       // per parity; copy p ^ 1 is zeroed by sequence p's k_bin_count
    uint64_t rescues;         // k_bin_one launches that aborted and were binned by the guarded scatter
};

struct Sorted {
    BinTable* bt;
    u32x4* desc;       // {S lo, S hi, E lo, E hi} per sorted slot
    uint32_t* idx;     // original index; kNoIdx for padding slots
    uint32_t* init;    // initial state per sorted slot (when the batch has one)
    uint32_t* status;  // context status word (bit 2: inconsistent bin layout)
    uint64_t cap;      // sorted slots allocated
    uint32_t par;      // counter copy of this sequence
    uint32_t one;      // host: the sequence was binned by k_bin_one (no scatter launch)
};

// First window of an entry in k_entries: its 128-byte line, so that every
// group load is exactly one cache line -- unless the 4 init bytes at S would
// cross into the second window (S within 3 bytes of the line end); then the
// 16-byte piece of S, as everywhere else.
__device__ __forceinline__ uint64_t line_base(uint64_t S)
{
    return (S & (kStep - 1)) > kStep - 4 ? (S & ~uint64_t(15)) : (S & ~uint64_t(kStep - 1));
}

__device__ __forceinline__ uint64_t entry_steps_line(uint64_t S, uint64_t E)
{
    return (E - line_base(S) + kStep - 1) / kStep;
}

__device__ __forceinline__ uint64_t entry_steps(uint64_t S, uint64_t E)
{
    return (E - (S & ~uint64_t(15)) + kStep - 1) / kStep;
}

// Bin 0: n < 4 (bytewise).  Bins 1..32: exactly that many steps.  Above:
// four bins per octave of the step count.
__device__ __forceinline__ int bin_of(uint64_t S, uint64_t E)
{
    if (E - S < 4)
        return 0;
    const uint64_t K = entry_steps(S, E);
    if (K <= 32)
        return int(K);
    const int m = 63 - __builtin_clzll(K);
    return 33 + 4 * (m - 5) + int((K >> (m - 2)) & 3);
}

__device__ __forceinline__ uint64_t bin_kmax(int b)
{
    if (b <= 32)
        return b == 0 ? 1 : uint64_t(b);
    const int m = (b - 33) / 4 + 5, f = (b - 33) % 4;
    return (uint64_t(5 + f) << (m - 2)) - 1;
}

// One LDS atomic per distinct bin of a wave instead of one per lane (log
// entries fall into a handful of bins, so per-lane atomics serialise).
// Returns this lane's rank among the wave's lanes of the same bin; *base_lane
// receives the previous counter value for the lane's bin.
__device__ __forceinline__ uint32_t wave_bin_add(uint32_t* h, int b, bool active, uint32_t& base)
{
    uint64_t todo = __ballot(active);
    const int lane = threadIdx.x & (kWaveSize - 1);
    uint32_t rank = 0;
    base = 0;
    while (todo) {
        const int leader = int(__builtin_ctzll(todo));
        const int lb = __shfl(b, leader, kWaveSize);
        const uint64_t same = __ballot(active && b == lb);
        uint32_t old = 0;
        if (lane == leader)
            old = atomicAdd(&h[lb], uint32_t(__popcll(same)));
        old = __shfl(old, leader, kWaveSize);
        if (active && b == lb) {
            base = old;
            rank = uint32_t(__popcll(same & ((1ull << lane) - 1)));
        }
        todo &= ~same;
    }
    return rank;
}

// The histogram pass.  It counts entries only: an earlier form also kept the
// largest step count of each log-scale bin with an LDS atomicMax issued,
// lane-masked, between the wave_bin_add loops, and on gfx950 that histogram
// came out wrong in about a quarter of the batches that had log-scale bins
// (entries of bin 33 counted under bins 34-40, 0 of 72 batches once either
// the atomicMax or the ds_bpermute-based wave_bin_add was removed,
// tools/diag_plan_skip.py).  A phantom entry left a
// bin's octet of padding slots only, whose interior loop bound Kmin - 1 then
// wrapped: the k_entries hang of round 2.  Each log-scale bin's work estimate
// now uses the bin's upper bound (bin_kmax).
// sum (nullable; records mode, ramcrc_replay_verify_device): the walk's
// replay_hard bits.  Bit 0 clear: every record is inactive or a one-window
// object, so the histogram is "all tiny" without reading the table -- the
// scatter then publishes the direct path, which re-checks every record (a
// record that is not tiny refuses the launch), and the plan and compare
// kernels find nothing.  Bit 1 clear: every record is inactive or an object
// of 2 .. kTinyK windows -- "all in bin 2", the direct multi-window path,
// which re-checks the same way.
template <int kMode>
__global__ __launch_bounds__(kThreads) void k_bin_count(BatchDesc d, Sorted so, int skip_large,
                                                        const uint32_t* sum)
{
    __shared__ uint32_t h[kNB];
    __shared__ uint32_t nlarge, ninact, nother;
    BinCounters& ctr = so.bt->ctr[so.par];
    if (blockIdx.x == 0) {
        // the next sequence's counters (see BinCounters)
        BinCounters& nx = so.bt->ctr[so.par ^ 1];
        for (int t = threadIdx.x; t < kNB; t += blockDim.x) {
            nx.cursor[t] = 0;
            nx.hist[t] = 0;
        }
        for (int t = threadIdx.x; t < kBinSlices * kNB; t += blockDim.x)
            nx.hs[t / kNB][t % kNB] = 0;
        for (int t = threadIdx.x; t < kBinSlices; t += blockDim.x)
            nx.arr[t] = 0;
        if (threadIdx.x == 0) {
            nx.nlarge = 0;
            nx.ninact = 0;
            nx.nother = 0;
            nx.wide = 0;
            nx.arrive = 0;
            nx.flag = 0;
        }
    }
    // the fused replay's summary (replay_hard bits over every walk record):
    // no record beyond one window -- all in bin 1, the direct tiny path; none
    // but objects of 2 .. kTinyK windows -- all in bin 2, the direct
    // multi-window path (bin_layout tells them apart by the bin)
    const uint32_t sv = sum ? *sum : 3u;
    if (!(sv & 1u) || (RAMCRC_TINY_DM && kTinyK >= 2 && !(sv & 2u))) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            ctr.hist[(sv & 1u) ? 2 : 1] = uint32_t(entry_count<kMode>(d));
            ctr.wide = (sv & 4u) ? 1u : 0u;
        }
        return;
    }
    for (int t = threadIdx.x; t < kNB; t += blockDim.x)
        h[t] = 0;
    if (threadIdx.x == 0) {
        nlarge = 0;
        ninact = 0;
        nother = 0;
    }
    __syncthreads();
    const uint64_t tile = uint64_t(blockDim.x) * kBinPer;
    const uint64_t n = entry_count<kMode>(d);
    // Records (replay batches of up to ~40M): the next tile's records are in
    // flight while this tile's segment status words are read and binned.
    // Order per tile: status loads (their records arrived last tile), then the
    // next tile's record loads, then the wait for the status words only.
    constexpr bool kPf = kMode == kRecords && RAMCRC_COUNT_PF;
    [[maybe_unused]] u32x4 nr[kBinPer];
    if constexpr (kPf) {
#pragma unroll
        for (int q = 0; q < kBinPer; q++) {
            const uint64_t i = uint64_t(blockIdx.x) * tile + uint64_t(q) * blockDim.x + threadIdx.x;
            nr[q] = i < n ? d.rec[i] : u32x4{0u, 0u, 0u, 0u};
        }
    }
    for (uint64_t base = uint64_t(blockIdx.x) * tile; base < n; base += uint64_t(gridDim.x) * tile) {
        uint64_t S[kBinPer], E[kBinPer];
        bool act[kBinPer], oth[kBinPer];
        if constexpr (kPf) {
            u32x4 cur[kBinPer];
            uint32_t st[kBinPer];
#pragma unroll
            for (int q = 0; q < kBinPer; q++) {
                cur[q] = nr[q];
                const uint64_t i = base + uint64_t(q) * blockDim.x + threadIdx.x;
                st[q] = i < n ? d.seg_status[cur[q].x].x : 0u;
            }
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t nb = base + uint64_t(gridDim.x) * tile;
#pragma unroll
            for (int q = 0; q < kBinPer; q++) {
                const uint64_t i = nb + uint64_t(q) * blockDim.x + threadIdx.x;
                nr[q] = i < n ? d.rec[i] : u32x4{0u, 0u, 0u, 0u};
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < kBinPer; q++) {
                const uint64_t i = base + uint64_t(q) * blockDim.x + threadIdx.x;
                S[q] = E[q] = 0;
                act[q] = i < n && record_range_st(d, cur[q], st[q], S[q], E[q]);
                oth[q] = i < n && replay_other(cur[q]);
            }
        } else {
#pragma unroll
        for (int q = 0; q < kBinPer; q++) {   // all loads first
            const uint64_t i = base + uint64_t(q) * blockDim.x + threadIdx.x;
            S[q] = E[q] = 0;
            oth[q] = false;
            if constexpr (kMode == kRecords) {
                // (the record read once: its range and whether k_obj_compare needs it)
                if (i < n) {
                    const u32x4 r = d.rec[i];
                    act[q] = record_range(d, r, S[q], E[q]);
                    oth[q] = replay_other(r);
                } else {
                    act[q] = false;
                }
            } else {
                act[q] = i < n && buffer_range<kMode>(d, i, S[q], E[q]);
            }
        }
        }
        uint32_t big = 0, inact = 0, other = 0;
#pragma unroll
        for (int q = 0; q < kBinPer; q++) {
            const bool large = skip_large && is_large(E[q] - S[q]);
            big += act[q] && large;
            inact += !act[q] && base + uint64_t(q) * blockDim.x + threadIdx.x < n;
            other += oth[q];
            const bool active = act[q] && !large;
            const int b = active ? bin_of(S[q], E[q]) : 0;
            uint32_t unused;
            wave_bin_add(h, b, active, unused);
        }
        if (__ballot(big != 0)) {   // rare: large buffers are few
            if (big)
                atomicAdd(&nlarge, big);
        }
        if (kMode == kRecords && __ballot(inact != 0)) {
            if (inact)
                atomicAdd(&ninact, inact);
        }
        if (kMode == kRecords && __ballot(other != 0)) {
            if (other)
                atomicAdd(&nother, other);
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < kNB; t += blockDim.x)
        if (h[t])
            atomicAdd(&ctr.hist[t], h[t]);
    if (threadIdx.x == 0 && nlarge)
        atomicAdd(&ctr.nlarge, nlarge);
    if (threadIdx.x == 0 && ninact)
        atomicAdd(&ctr.ninact, ninact);
    if (threadIdx.x == 0 && nother)
        atomicAdd(&ctr.nother, nother);
}

// Bin layout from the histogram, computed by every k_bin_scatter workgroup
// for itself (no separate scan launch): threads 0..255 take one bin each and
// run parallel exclusive scans of the slot counts and of the work units.
// Workgroup 0 also publishes the layout k_entries reads (start, items, kcost)
// and empties the padding slots of each bin's last octet.  Every thread of
// the block calls this (it synchronises).
struct BinScratch {
    uint64_t start[kNB], count[kNB];
    uint64_t wpos[4], witem[4];
    uint32_t direct, multi;
};

// Returns false (uniformly) when the histogram asks for more sorted slots
// than are allocated -- possible only with a corrupted histogram; the layout
// is then published empty, the status bit set, and nothing is scattered.
// direct_n: the table size when the batch may take the direct tiny path
// (kTable mode), else 0.  When every entry of such a batch is tiny (bins 0-1
// hold all of them), the layout is published empty with direct_n set and
// nothing is scattered: k_entries' tiny phase reads the caller's (off, len,
// init) in place, in index order.
// A counter another workgroup of the same launch may have added to
// (k_bin_one): read at the coherence point, not from this XCD's L2.
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool bin_layout(const Sorted& so, BinScratch& sc, bool publish,
                                          uint64_t direct_n, const uint32_t* hist = nullptr,
                                          uint64_t multi_n = 0)
{
    BinTable* bt = so.bt;
    const BinCounters& ctr = bt->ctr[so.par];
    const int b = threadIdx.x, lane = b & 63, w = b >> 6;
    if (threadIdx.x == 0) {
        const uint64_t inact = ld_agent(&ctr.ninact);
        sc.direct = direct_n && uint64_t(hist ? hist[0] : ld_agent(&ctr.hist[0])) +
                                        (hist ? hist[1] : ld_agent(&ctr.hist[1])) + inact == direct_n;
        // multi_n (records batches): every active record in bin 2 -- the
        // direct multi-window path reads the record table in place
        sc.multi = !sc.direct && multi_n &&
                   uint64_t(hist ? hist[2] : ld_agent(&ctr.hist[2])) + inact == multi_n;
    }
    __syncthreads();
    const bool direct = sc.direct, multi = sc.multi;
    if (publish && threadIdx.x == 0) {
        bt->direct_n = direct ? direct_n : 0;
        bt->direct_multi = multi ? multi_n : 0;
        bt->direct_multi_k2 = multi && !ld_agent(&ctr.wide);   // bin 2 proper: two windows at most
    }
    uint64_t cnt = 0, kc = 0, ps = 0, is = 0, pos_c = 0, item_c = 0;
    if (b < 256) {
        if (b < kNB) {
            cnt = direct || multi ? 0 : (hist ? hist[b] : ld_agent(&ctr.hist[b]));
            kc = b <= 32 ? uint64_t(b == 0 ? 1 : b) : bin_kmax(b);
        }
        const uint64_t oct = (cnt + kG - 1) / kG;
        pos_c = oct * kG;
        item_c = b > kTinyK && b >= 2 ? oct * (kc + kOctetCost) : 0;   // bins 0..kTinyK: tiny phases
        ps = pos_c;
        is = item_c;
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {
            const uint64_t a1 = __shfl_up(ps, s, kWaveSize);
            const uint64_t a2 = __shfl_up(is, s, kWaveSize);
            if (lane >= s) {
                ps += a1;
                is += a2;
            }
        }
        if (lane == 63) {
            sc.wpos[w] = ps;
            sc.witem[w] = is;
        }
    }
    __syncthreads();
    const bool ok = sc.wpos[0] + sc.wpos[1] + sc.wpos[2] + sc.wpos[3] <= so.cap;
    if (b < kNB) {
        uint64_t pb = 0, ib = 0;
        for (int j = 0; j < w; j++) {
            pb += sc.wpos[j];
            ib += sc.witem[j];
        }
        const uint64_t start = ok ? pb + ps - pos_c : 0, items = ok ? ib + is - item_c : 0;
        sc.start[b] = start;
        sc.count[b] = ok ? cnt : 0;
        if (publish) {
            bt->start[b] = start;
            bt->count[b] = ok ? cnt : 0;
            bt->items[b] = items;
            bt->kcost[b] = kc + kOctetCost;
            if (b == kNB - 1)
                bt->items[kNB] = ok ? items + item_c : 0;
        }
    }
    if (!ok) {
        if (publish && threadIdx.x == 0)
            atomicOr(so.status, kStatusSticky | kStatusBins);
        return false;
    }
    __syncthreads();
    if (publish) {
        for (int t = threadIdx.x; t < kNB * kG; t += blockDim.x) {
            const int bb = t / kG, j = t % kG;
            const uint64_t c = sc.count[bb];
            const uint64_t slot = c + uint64_t(j);
            if ((c % kG) && slot < (c + kG - 1) / kG * kG) {
                so.desc[sc.start[bb] + slot] = u32x4{0u, 0u, 0u, 0u};
                so.idx[sc.start[bb] + slot] = kNoIdx;
            }
        }
    }
    return true;
}

// rescue: the guarded scatter after a k_bin_one (see there): nothing to do
// when k_bin_one's vote went kBinGo; otherwise the histogram is the sum of
// k_bin_one's slices, which every workgroup of it added to before it voted.
template <int kMode>
__global__ __launch_bounds__(kThreads) void k_bin_scatter(BatchDesc d, Sorted so, int skip_large,
                                                          int rescue)
{
    __shared__ uint32_t cnt[kNB];
    __shared__ uint64_t base[kNB];
    __shared__ BinScratch sc;
    __shared__ uint32_t tot[kNB];
    __shared__ uint32_t vote;
    BinCounters& ctr = so.bt->ctr[so.par];
    if (rescue) {
        // one load per workgroup (k_bin_one has ended: the flag is final); a
        // load per thread put 250K same-address loads on the fabric (5 us)
        if (threadIdx.x == 0)
            vote = ld_agent(&ctr.flag);
        __syncthreads();
        if (vote == kBinGo)
            return;
        for (int t = threadIdx.x; t < kNB; t += blockDim.x) {
            uint32_t all = 0;
#pragma unroll
            for (int j = 0; j < kBinSlices; j++)
                all += ld_agent(&ctr.hs[j][t]);
            tot[t] = all;
            if (blockIdx.x == 0)
                ctr.hist[t] = all;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0)
            atomicAdd(reinterpret_cast<unsigned long long*>(&so.bt->rescues), 1ull);
    }
    for (int t = threadIdx.x; t < kNB; t += blockDim.x)
        cnt[t] = 0;
    __syncthreads();
    if (!bin_layout(so, sc, blockIdx.x == 0,
                    (kMode == kTable || kMode == kRecords) && RAMCRC_TINY_CF ? entry_count<kMode>(d) : 0,
                    rescue ? tot : nullptr,
                    kMode == kRecords && RAMCRC_TINY_DM && kTinyK >= 2 ? entry_count<kMode>(d) : 0))
        return;   // corrupted histogram: nothing is scattered, k_entries refuses
    if (sc.direct || sc.multi)
        return;   // all tiny / all of 2 .. kTinyK windows: k_entries reads the table in place
    unsigned long long* cursor = reinterpret_cast<unsigned long long*>(ctr.cursor);
    const uint64_t tile = uint64_t(blockDim.x) * kBinPer;
    const uint64_t n = entry_count<kMode>(d);
    for (uint64_t t0 = uint64_t(blockIdx.x) * tile; t0 < n; t0 += uint64_t(gridDim.x) * tile) {
        uint64_t S[kBinPer], E[kBinPer];
        int b[kBinPer];
        uint32_t lp[kBinPer];
        bool act[kBinPer];
#pragma unroll
        for (int q = 0; q < kBinPer; q++) {
            const uint64_t i = t0 + uint64_t(q) * blockDim.x + threadIdx.x;
            S[q] = E[q] = 0;
            act[q] = i < n && buffer_range<kMode>(d, i, S[q], E[q]);
        }
#pragma unroll
        for (int q = 0; q < kBinPer; q++) {
            const bool active = act[q] && !(skip_large && is_large(E[q] - S[q]));
            b[q] = active ? bin_of(S[q], E[q]) : 0;
            uint32_t wbase;
            const uint32_t rank = wave_bin_add(cnt, b[q], active, wbase);
            lp[q] = wbase + rank;
            if (!active)
                b[q] = -1;
        }
        __syncthreads();
        for (int t = threadIdx.x; t < kNB; t += blockDim.x)
            if (cnt[t]) {
                base[t] = atomicAdd(&cursor[t], (unsigned long long)cnt[t]);
                cnt[t] = 0;
            }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kBinPer; q++) {
            // a slot past the bin's count (a histogram that disagrees with
            // this pass) is not written; the cursor still counts it, so
            // k_entries sees cursor != count and refuses the launch
            if (b[q] >= 0 && base[b[q]] + lp[q] < sc.count[b[q]]) {
                const uint64_t i = t0 + uint64_t(q) * blockDim.x + threadIdx.x;
                const uint64_t pos = sc.start[b[q]] + base[b[q]] + lp[q];
                so.desc[pos] = u32x4{uint32_t(S[q]), uint32_t(S[q] >> 32), uint32_t(E[q]),
                                     uint32_t(E[q] >> 32)};
                so.idx[pos] = uint32_t(i);
                if (d.init)
                    so.init[pos] = d.init[i];
            }
        }
        __syncthreads();
    }
}

// One-launch binning for batches of at most one tile per workgroup, with the
// grid expected resident at once (bin_begin checks both): each workgroup loads
// its tile once, ranks every entry inside its bin with the same wave_bin_add
// as the count pass, and takes its range of each bin with one returning
// atomic on the histogram -- the value the two-launch path's scatter cursor
// would give.  After a grid-wide arrival every workgroup lays the bins out
// from the now complete histogram and writes its descriptors from registers.
// Saves the scatter's second read of the table.
//
// The arrival cannot be guaranteed: another context's kernels on another
// stream (a k_entries workgroup takes a whole CU; a second k_bin_one takes
// the other half) or a preempted queue can keep part of the grid from being
// dispatched while the rest waits.  So the wait is a vote, never a
// precondition: the last arrival tries to turn the flag from 0 to kBinGo, a
// waiter that has seen no arrival anywhere in the grid for kBinStallTicks
// tries to turn it from 0 to kBinAbort, and the one compare-and-swap that
// wins decides for every workgroup, including those dispatched later.  On
// abort nothing is scattered; the guarded scatter launched after every
// k_bin_one (k_bin_scatter with `rescue`) exits at once on kBinGo and
// otherwise bins the batch the two-launch way from the histogram k_bin_one
// completed.  A grid that cannot all be resident therefore costs one stall
// period and a second read of the table, never a wrong or refused launch.
#ifndef RAMCRC_BIN_SLEEP
#define RAMCRC_BIN_SLEEP 4   // s_sleep between polls (x 64 cycles)
#endif
#ifndef RAMCRC_BIN_STALL_US
#define RAMCRC_BIN_STALL_US 30   // k_bin_one: abort after this long with no arrival in the grid
#endif
// No fences: on this 8-XCD part an agent-scope release / acquire writes back
// / invalidates the XCD's L2 (per thread), which cost more than the whole
// two-launch binning.  Everything that crosses workgroups here is an atomic
// (the histogram adds, performed before the wave passes s_waitcnt, the
// arrival counts, the flag, and bin_layout's reads of the histogram).
constexpr uint64_t kBinStallTicks = uint64_t(RAMCRC_BIN_STALL_US) * 100;   // 100 MHz clock
__device__ __forceinline__ uint32_t bin_arrivals(const BinCounters& ctr)
{
    uint32_t a = 0;
#pragma unroll
    for (int j = 0; j < kBinSlices; j++)
        a += __hip_atomic_load(&ctr.arr[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return a;
}

__device__ __forceinline__ uint32_t bin_vote(BinCounters& ctr, uint32_t want)
{
    uint32_t expect = 0;
    __hip_atomic_compare_exchange_strong(&ctr.flag, &expect, want, __ATOMIC_RELAXED,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return expect ? expect : want;   // the value that won
}

// Two-level arrival: a workgroup counts itself in its slice (workgroups
// i % kBinSlices), the last of a slice counts the slice in `arrive`, the last
// slice votes kBinGo (one counter for the whole grid serialised its ~1,000
// arrivals: ~5 us).  Returns true when kBinGo won the vote.  The clock is the
// 100 MHz s_memrealtime; a stall measured across a preemption only makes the
// abort (the slower, always correct path) more likely.
__device__ __forceinline__ bool grid_arrive(BinCounters& ctr, uint32_t nwg)
{
    __shared__ uint32_t all_in;
    __builtin_amdgcn_s_waitcnt(0);   // this wave's histogram atomics are performed
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t sl = blockIdx.x % kBinSlices;
        const uint32_t in_sl = nwg / kBinSlices + (sl < nwg % kBinSlices ? 1u : 0u);
        const uint32_t nsl = nwg < uint32_t(kBinSlices) ? nwg : uint32_t(kBinSlices);
        bool last = __hip_atomic_fetch_add(&ctr.arr[sl], 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT) + 1 == in_sl;
        if (last)
            last = __hip_atomic_fetch_add(&ctr.arrive, 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT) + 1 == nsl;
        uint32_t f;
        if (last) {
            f = bin_vote(ctr, kBinGo);
        } else {
            uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t seen = bin_arrivals(ctr);
            while ((f = __hip_atomic_load(&ctr.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0) {
                const uint64_t now = __builtin_amdgcn_s_memrealtime();
                if (now - t0 > kBinStallTicks) {
                    const uint32_t a = bin_arrivals(ctr);
                    if (a == seen) {
                        f = bin_vote(ctr, kBinAbort);   // nobody arrived for a whole period
                        break;
                    }
                    seen = a;
                    t0 = now;
                }
                __builtin_amdgcn_s_sleep(RAMCRC_BIN_SLEEP);
            }
        }
        all_in = f == kBinGo;
    }
    __syncthreads();
    return all_in;
}

template <int kMode>
__global__ __launch_bounds__(kThreads) void k_bin_one(BatchDesc d, Sorted so, int skip_large,
                                                      uint32_t straggler)
{
    __shared__ uint32_t h[kNB];
    __shared__ uint64_t base[kNB];
    __shared__ uint32_t nlarge, ninact, nother;
    __shared__ BinScratch sc;
    BinCounters& ctr = so.bt->ctr[so.par];
    if (blockIdx.x == 0) {
        BinCounters& nx = so.bt->ctr[so.par ^ 1];   // the next sequence's counters
        for (int t = threadIdx.x; t < kNB; t += blockDim.x) {
            nx.cursor[t] = 0;
            nx.hist[t] = 0;
        }
        for (int t = threadIdx.x; t < kBinSlices * kNB; t += blockDim.x)
            nx.hs[t / kNB][t % kNB] = 0;
        for (int t = threadIdx.x; t < kBinSlices; t += blockDim.x)
            nx.arr[t] = 0;
        if (threadIdx.x == 0) {
            nx.nlarge = 0;
            nx.ninact = 0;
            nx.nother = 0;
            nx.wide = 0;
            nx.arrive = 0;
            nx.flag = 0;
        }
    }
    for (int t = threadIdx.x; t < kNB; t += blockDim.x)
        h[t] = 0;
    if (threadIdx.x == 0) {
        nlarge = 0;
        ninact = 0;
        nother = 0;
    }
    __syncthreads();
    const uint64_t n = entry_count<kMode>(d);
    const uint64_t t0 = uint64_t(blockIdx.x) * blockDim.x * kBinPer;
    uint64_t S[kBinPer], E[kBinPer];
    bool act[kBinPer], oth[kBinPer];
    uint32_t in0[kBinPer];
#pragma unroll
    for (int q = 0; q < kBinPer; q++) {   // all loads first
        const uint64_t i = t0 + uint64_t(q) * blockDim.x + threadIdx.x;
        S[q] = E[q] = 0;
        oth[q] = false;
        if constexpr (kMode == kRecords) {
            if (i < n) {
                const u32x4 r = d.rec[i];
                act[q] = record_range(d, r, S[q], E[q]);
                oth[q] = replay_other(r);
            } else {
                act[q] = false;
            }
        } else {
            act[q] = i < n && buffer_range<kMode>(d, i, S[q], E[q]);
        }
        in0[q] = d.init && i < n ? d.init[i] : 0u;
    }
    int b[kBinPer];
    uint32_t lp[kBinPer];
    uint32_t big = 0, inact = 0, other = 0;
#pragma unroll
    for (int q = 0; q < kBinPer; q++) {
        const bool large = skip_large && is_large(E[q] - S[q]);
        big += act[q] && large;
        inact += !act[q] && t0 + uint64_t(q) * blockDim.x + threadIdx.x < n;
        other += oth[q];
        const bool active = act[q] && !large;
        b[q] = active ? bin_of(S[q], E[q]) : 0;
        uint32_t wbase;
        const uint32_t rank = wave_bin_add(h, b[q], active, wbase);
        lp[q] = wbase + rank;
        if (!active)
            b[q] = -1;
    }
    if (__ballot(big != 0) && big)
        atomicAdd(&nlarge, big);
    if (kMode == kRecords && __ballot(inact != 0) && inact)
        atomicAdd(&ninact, inact);
    if (kMode == kRecords && __ballot(other != 0) && other)
        atomicAdd(&nother, other);
    __syncthreads();
    const int sl = int(blockIdx.x % kBinSlices);
    for (int t = threadIdx.x; t < kNB; t += blockDim.x)
        base[t] = h[t] ? atomicAdd(&ctr.hs[sl][t], h[t]) : 0u;
    if (threadIdx.x == 0 && nlarge)
        atomicAdd(&ctr.nlarge, nlarge);
    if (threadIdx.x == 0 && ninact)
        atomicAdd(&ctr.ninact, ninact);
    if (threadIdx.x == 0 && nother)
        atomicAdd(&ctr.nother, nother);
    // (straggler: test hook, one workgroup more than launched, which never comes)
    if (!grid_arrive(ctr, gridDim.x + straggler))
        return;   // aborted: the guarded scatter bins the batch
    constexpr bool kDirect = (kMode == kTable || kMode == kRecords) && RAMCRC_TINY_CF;
    if constexpr (kDirect) {
        // Every entry tiny (the direct path: nothing to scatter)?  Bins 0 and
        // 1 and the inactive count decide it -- 17 loads instead of the 8 x 161
        // below -- and then only workgroup 0 has work left: publishing the
        // (empty) layout.
        __shared__ uint32_t all_tiny;
        if (threadIdx.x < 2) {
            uint32_t all = 0;
#pragma unroll
            for (int j = 0; j < kBinSlices; j++)
                all += ld_agent(&ctr.hs[j][threadIdx.x]);
            h[threadIdx.x] = all;
        }
        __syncthreads();
        if (threadIdx.x == 0)
            all_tiny = uint64_t(h[0]) + h[1] + ld_agent(&ctr.ninact) == n;
        __syncthreads();
        if (all_tiny) {
            if (blockIdx.x == 0) {
                if (threadIdx.x < 2)
                    ctr.hist[threadIdx.x] = h[threadIdx.x];
                bin_layout(so, sc, true, n, h);   // direct: reads bins 0 and 1 only
                for (int t = threadIdx.x; t < kNB; t += blockDim.x)
                    ctr.cursor[t] = sc.count[t];
            }
            return;
        }
    }
    // totals, and this workgroup's place behind the earlier slices (reading
    // the slices here beat having the last arrival publish the totals)
    for (int t = threadIdx.x; t < kNB; t += blockDim.x) {
        uint32_t all = 0, before = 0;
#pragma unroll
        for (int j = 0; j < kBinSlices; j++) {
            const uint32_t v = ld_agent(&ctr.hs[j][t]);
            before += j < sl ? v : 0u;
            all += v;
        }
        h[t] = all;
        base[t] += before;
        if (blockIdx.x == 0)
            ctr.hist[t] = all;
    }
    __syncthreads();
    const bool ok = bin_layout(so, sc, blockIdx.x == 0,
                               (kMode == kTable || kMode == kRecords) && RAMCRC_TINY_CF ? n : 0, h);
    if (blockIdx.x == 0)   // what k_entries checks: every bin holds what was placed in it
        for (int t = threadIdx.x; t < kNB; t += blockDim.x)
            ctr.cursor[t] = sc.count[t];
    if (!ok || sc.direct)
        return;
#pragma unroll
    for (int q = 0; q < kBinPer; q++) {
        if (b[q] >= 0 && base[b[q]] + lp[q] < sc.count[b[q]]) {
            const uint64_t i = t0 + uint64_t(q) * blockDim.x + threadIdx.x;
            const uint64_t pos = sc.start[b[q]] + base[b[q]] + lp[q];
            so.desc[pos] = u32x4{uint32_t(S[q]), uint32_t(S[q] >> 32), uint32_t(E[q]),
                                 uint32_t(E[q] >> 32)};
            so.idx[pos] = uint32_t(i);
            if (d.init)
                so.init[pos] = in0[q];
        }
    }
}


// Mask and init-inject the 16 bytes of lane piece `a` of entry [S, E): one
// 64-bit clamp per piece, then 32-bit arithmetic per word.
__device__ __forceinline__ int clamp32(int64_t x)
{
    return x < -32 ? -32 : (x > 32 ? 32 : int(x));
}

__device__ __forceinline__ uint32_t fix_word32(uint32_t w, int ds, int de, uint32_t init)
{
    const int lo = min(max(ds, 0), 4), hi = min(max(de, 0), 4);
    const uint32_t mhi = uint32_t((1ull << (8 * hi)) - 1);
    const uint32_t mlo = uint32_t((1ull << (8 * lo)) - 1);
    w &= mhi & ~mlo;
    const int dd = -ds;   // word address - S
    const uint32_t inj =
        uint32_t((uint64_t(init) << 24) >> (24 + 8 * min(max(dd, -3), 3)));
    return w ^ ((dd > -4 && dd < 4) ? inj : 0u);
}

__device__ __forceinline__ u32x4 fix_piece(u32x4 w, uint64_t a, uint64_t S, uint64_t E,
                                           uint32_t init)
{
    const int ds = clamp32(int64_t(S - a)), de = clamp32(int64_t(E - a));
    w.x = fix_word32(w.x, ds, de, init);
    w.y = fix_word32(w.y, ds - 4, de - 4, init);
    w.z = fix_word32(w.z, ds - 8, de - 8, init);
    w.w = fix_word32(w.w, ds - 12, de - 12, init);
    return w;
}

// Lane piece -> window end: fold the four word slots with X^4, then the
// group's eight lanes with X^16, X^32, X^64 (a shuffle butterfly).  Every lane
// of the group returns the entry's raw state relative to the end of its last
// 128-byte window; the caller removes the zero padding with x^(-8 pad).
#ifndef RAMCRC_PROBE_FOLD
#define RAMCRC_PROBE_FOLD 0   // A/B only (WRONG results): 1 no fold lookups, 2 conflict-free fold lookups
#endif
#ifndef RAMCRC_PROBE_MASK
#define RAMCRC_PROBE_MASK 0   // A/B only (WRONG results): long-phase head/tail steps unmasked
#endif
__device__ __forceinline__ uint32_t group_fold(const uint8_t* lds, int gl, uint32_t u0,
                                               uint32_t u1, uint32_t u2, uint32_t u3)
{
#if RAMCRC_PROBE_FOLD == 1
    return u0 ^ u1 ^ u2 ^ u3 ^ uint32_t(__shfl_xor(int(u0), 1, kWaveSize));
#elif RAMCRC_PROBE_FOLD == 2
    auto pa = [&](uint32_t off, uint32_t v) {
        const uint32_t* t = reinterpret_cast<const uint32_t*>(lds + off);
        const uint32_t l = threadIdx.x & 31;
        return t[l] ^ t[256 + l] ^ t[512 + l] ^ t[768 + l] ^ v;
    };
    uint32_t z = pa(kX4Off, u0) ^ u1;
    z = pa(kX4Off, z) ^ u2;
    z = pa(kX4Off, z) ^ u3;
    z = pa(kX4Off, z);
#pragma unroll
    for (int lvl = 0; lvl < 3; lvl++) {
        const uint32_t other = __shfl_xor(z, 1 << lvl, kWaveSize);
        z = pa(kX4Off + (1 + lvl) * 4096, z) ^ other;
    }
    return z;
#else
    // X^12(u0) ^ X^8(u1) ^ X^4(u2) ^ u3 as a two-level tree (the two X^4
    // lookups are independent); the piece's final X^4 is left to the unpad
    // constant (xinv4), so the fold is three dependent lookups deep, not four.
    const uint32_t a = plain_apply(lds, kX4Off, u0) ^ u1;
    const uint32_t b = plain_apply(lds, kX4Off, u2) ^ u3;
    uint32_t z = plain_apply(lds, kX8Off, a) ^ b;
#pragma unroll
    for (int lvl = 0; lvl < 3; lvl++) {
        const uint32_t other = __shfl_xor(z, 1 << lvl, kWaveSize);
        const bool upper = (gl >> lvl) & 1;
        const uint32_t lower_v = upper ? other : z;
        const uint32_t upper_v = upper ? z : other;
        z = plain_apply(lds, kX4Off + (1 + lvl) * 4096, lower_v) ^ upper_v;
    }
    return z;
#endif
}

// Head word at distance ds = S - (word address): drop the bytes before S and
// inject the initial state into the four bytes at S.
__device__ __forceinline__ uint32_t keep_lo(int c);
__device__ __forceinline__ uint32_t head_word(uint32_t w, int ds, uint32_t init)
{
    const uint32_t inj = uint32_t((uint64_t(init) << 24) >> (24 - 8 * min(max(ds, -3), 3)));
    return (w & ~keep_lo(ds)) ^ ((ds > -4 && ds < 4) ? inj : 0u);
}

// Byte mask of a word whose first c bytes (clamped to 0..4) are kept.
__device__ __forceinline__ uint32_t keep_lo(int c)
{
    c = min(max(c, 0), 4);
    return c >= 4 ? 0xFFFFFFFFu : (1u << (8 * c)) - 1u;
}

// XOR of the 8 lanes of each lane group, valid in lanes 0-3 of the group
// (DPP: quad swaps, then the other quad of the 16-lane row; no LDS traffic).
__device__ __forceinline__ uint32_t group8_xor(uint32_t v)
{
    v ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
    v ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
    v ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x12C, 0xF, 0xF, false));  // row_ror:12 (lane + 4)
    return v;
}

// Entries of at most one 128-byte window (bins 0-1; 100-byte log entries are
// here): no Horner step and no per-entry multiply.  Byte b at distance m from
// the entry end contributes X^m(b), read from a 132 x 256 LDS table (rows for
// m <= 0 are zero), so a lane does 16 lookups for its 16 bytes and the group
// XORs its 8 lanes.  Round r of a wave covers 64 sorted
// slots; lane L owns slot 64 r + L: it loads that descriptor (one coalesced
// 1 KiB load per round instead of eight group-redundant ones), and at the end
// folds in the slot's initial state and stores its result.  Group g hashes
// the entries of lanes 8 g .. 8 g + 7 in turn, reading each owner's window
// (base, offset, length) by swizzle within the group.  Descriptors are loaded
// two rounds ahead and data one round ahead, so a wave's rounds overlap their
// memory latency with the previous round's lookups.
struct TinyOwn {
    uint64_t S, A;        // entry start; its 16-byte piece
    uint32_t geo;         // len (bits 0-7) | (S - A) << 8 for len >= 4 in bin 1; else 0
    uint32_t len, ix, init;
};

template <int q>
__device__ __forceinline__ uint32_t swz_from(uint32_t v)
{
    // lane (lane & 0x18) | q within each 32-lane half: lane q of this group
    return uint32_t(__builtin_amdgcn_ds_swizzle(int(v), 0x18 | (q << 5)));
}

template <int q = 0, class F>
__device__ __forceinline__ void static_for8(F&& f)
{
    if constexpr (q < 8) {
        f(std::integral_constant<int, q>{});
        static_for8<q + 1>(f);
    }
}

// Probe builds only (RAMCRC_STAMPS=1, tools/stamps.py): lane 0 of every wave
// records the 100 MHz real-time clock at k_entries' phase boundaries.
#ifndef RAMCRC_STAMPS
#define RAMCRC_STAMPS 0
#endif
#if RAMCRC_STAMPS
constexpr int kStampWaves = 8192, kStampSlots = 8;
__device__ unsigned long long g_stamps[kStampWaves * kStampSlots];
#define RAMCRC_STAMP(k)                                                                       \
    do {                                                                                      \
        const uint32_t sw_ = blockIdx.x * kEntWaves + threadIdx.x / kWaveSize;                \
        if ((threadIdx.x & (kWaveSize - 1)) == 0 && sw_ < uint32_t(kStampWaves))              \
            g_stamps[sw_ * kStampSlots + (k)] = __builtin_amdgcn_s_memrealtime();             \
    } while (0)
#define RAMCRC_STAMP_ONCE(k, flag) \
    do {                           \
        if (flag) {                \
            RAMCRC_STAMP(k);       \
            flag = false;          \
        }                          \
    } while (0)
#else
#define RAMCRC_STAMP_ONCE(k, flag) \
    do {                           \
        (void)(flag);              \
    } while (0)
#define RAMCRC_STAMP(k) \
    do {                \
    } while (0)
#endif

// The tiny phases with conflict-free table lookups (RAMCRC_TINY_CF): the
// window-relative table below puts a lookup's LDS bank on its window position,
// whatever the data byte.  Lane u of a group holds the window dwords u, u + 8,
// u + 16, u + 24 (window offsets 32 j + 4 u), so the 8 lanes of a group read
// rows 4 apart; each group takes the bytes of its dwords in a rotated order
// (byte (k + g) & 3 at instruction k, g the group's index in its 32-lane
// half), which puts the 4 groups of a half on the 4 residue classes: the 32
// lanes of a ds_read_b32 half hit 32 banks.  Bytes outside the entry are
// masked to 0, and X^m(0) = 0.
//
// tiny_run_cf: bins 0-1, entries of one 128-byte window (all 100-byte log
// entries).  tiny_multi: bins 2 .. kTinyK, entries of 2 .. kTinyK windows
// (objects of about 129 .. 500 B): window by window with Horner between them,
//   acc = X^e_w(acc) ^ R_w,
// R_w the group's sum over window w's bytes at their distance from the
// window's end e_w (128 for all but the last), X^e (e >= 4) four lookups in the
// same table by lanes gl & 3 and two quad swaps; an entry whose last window
// would hold only 1 .. 3 bytes stops a window early and its owner takes those
// bytes bytewise.  (The short-bin loop of entries_run spends an octet's head
// masks, fold and unpad multiply -- about 600 VALU per octet of 2-step entries
// -- where this spends the windows.)
//
// Round r of a wave covers 64 sorted slots; lane L owns slot 64 r + L: it loads
// that slot's descriptor two rounds ahead (one coalesced load per round instead
// of eight group-redundant ones; tiny_multi derives the entry geometry from it
// one round later), and at the end folds in the slot's initial state and
// stores the result.  Group g hashes the entries
// of lanes 8 g .. 8 g + 7 in turn, reading each owner's window (base, offset,
// length) by swizzle within the group; tiny_run_cf loads a round's windows one
// round ahead, tiny_multi an entry's windows one entry ahead.
struct TinyRaw {
    u32x4 dd;            // sorted descriptor {S, E}, or {off, len} on the direct path
    uint32_t ix, init;
};

struct TinyCf {
    uint64_t S;
    // E - A (bits 0-9; 0: nothing to hash, or bytewise), S - A (10-13), window
    // page-safe (14), E - S (16-25); A = S rounded down to 16
    uint32_t geo;
    uint32_t ix, init;
};

// windows hashed for an entry of geometry geo (tiny_multi: the last 1 .. 3
// bytes past a window go bytewise, as X^e needs e >= 4)
__device__ __forceinline__ uint32_t tk_tail(uint32_t geo)
{
    const uint32_t t = geo & 127u;
    return geo > 128 && t != 0 && t < 4 ? t : 0u;
}

__device__ __forceinline__ uint32_t tk_windows(uint32_t geo)
{
    return ((geo & 0x3FFu) - tk_tail(geo) + 127u) >> 7;
}

// The tiny phases' LDS holds X^(128 - q)(b) for window
// position q at ((q >> 6) << 16) | (b << 8) | ((q & 63) << 2) -- the data byte
// is address byte 1, so one v_perm forms an address from a per-lane constant
// -- and X^-128 (4 x 256 words) after it.  A window's bytes are summed at their
// distance from the window's end, whatever the entry; the owner lane moves its
// entry's sum to the entry end with X^e(X^-128(.)) (8 lookups per slot instead
// of per-window row arithmetic in every lane).  Masked bytes are 0, and
// X^m(0) = 0.
constexpr uint32_t kTwInvOff = 131072;
constexpr uint32_t kLdsTinyWr = kTwInvOff + 4096;
static_assert(kLdsTinyWr <= kLdsEntries, "k_entries' LDS holds the tiny phases' tables");

__device__ __forceinline__ uint32_t tw_addr(uint32_t q, uint32_t b)
{
    return ((q >> 6) << 16) | (b << 8) | ((q & 63) << 2);
}

__device__ __forceinline__ void tiny_fill_wr(uint8_t* lds)
{
    // 8192 chunks of 16 B, chunk (h, b, c) = words 128 (255 - b) + 64 h + 4 c .. of
    // g_tab.post (X^m(b) at 128 (255 - b) + 128 - m), then the X^-128 table
    constexpr uint32_t kPos = 8192, kAll = kPos + 256;
    constexpr uint32_t kPer = (kAll + kEntWaves * kWaveSize - 1) / (kEntWaves * kWaveSize);
    const uint4* post = reinterpret_cast<const uint4*>(g_tab.post);
    const uint4* inv = reinterpret_cast<const uint4*>(&g_tab.xinv128);
    uint4 v[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t i = threadIdx.x + j * (kEntWaves * kWaveSize);
        if (i < kPos) {
            const uint32_t h = i >> 12, b = (i >> 4) & 255, c = i & 15;
            v[j] = post[(128 * (255 - b) + 64 * h) / 4 + c];
        } else if (i < kAll) {
            v[j] = inv[i - kPos];
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t i = threadIdx.x + j * (kEntWaves * kWaveSize);
        if (i < kAll)
            *reinterpret_cast<uint4*>(lds + 16 * i) = v[j];
    }
}

#ifndef RAMCRC_TINY_GEN
#define RAMCRC_TINY_GEN 1   // tiny tables built in LDS from 8 basis words per row (0: copied from g_tab)
#endif
#if RAMCRC_TINY_GEN
// The tiny phases' tables built in place instead of copied: X^m is linear, so
// row q of X^(128 - q)(b) is the XOR of the basis words twb[q][k] over the set
// bits k of b.  Thread t takes row q = t % 128 and the 32 columns b0 .. b0 + 31,
// b0 = 32 (t / 128): T[b0] from bits 5-7, then T[b0 + i] = T[b0 + (i & (i - 1))]
// ^ twb[q][ctz i] -- 31 XORs -- and 32 stores at immediate offsets (a wave's
// 64 rows land on 32 banks).  Threads 0 .. 31 then build X^-128 the same way.
// The copy it replaces moved 132 KiB per CU through the L2 (33 MB per launch
// over the chip; 4.3 us of a 35 us 1M x 100 B launch, profiles/r04/ab).
// (split in two so that a caller can put loads of its own between them: the
// basis words' loads, then the build once they have landed)
struct TinyBasis {
    uint4 lo, hi, a, c;
};

__device__ __forceinline__ TinyBasis tiny_basis_load()
{
    TinyBasis t;
    const uint32_t q = threadIdx.x & 127;
    const uint4* bp = reinterpret_cast<const uint4*>(g_tab.twb[q]);
    t.lo = bp[0];
    t.hi = bp[1];
    t.a = t.c = make_uint4(0u, 0u, 0u, 0u);
    if (threadIdx.x < 32) {   // X^-128: table j = t / 8, columns 32 (t % 8) ..
        const uint4* ip = reinterpret_cast<const uint4*>(g_tab.twib[threadIdx.x >> 3]);
        t.a = ip[0];
        t.c = ip[1];
    }
    return t;
}

__device__ __forceinline__ void tiny_fill_build(uint8_t* lds, const TinyBasis& tb)
{
    static_assert(kEntWaves * kWaveSize == 1024, "one (row, column block) per thread");
    const uint32_t q = threadIdx.x & 127, b0 = 32 * (threadIdx.x >> 7);
    const uint32_t B[8] = {tb.lo.x, tb.lo.y, tb.lo.z, tb.lo.w, tb.hi.x, tb.hi.y, tb.hi.z, tb.hi.w};
    const uint32_t iv[8] = {tb.a.x, tb.a.y, tb.a.z, tb.a.w, tb.c.x, tb.c.y, tb.c.z, tb.c.w};
    const bool inv = threadIdx.x < 32;
    uint32_t T[32];
    T[0] = ((b0 >> 5) & 1 ? B[5] : 0u) ^ ((b0 >> 6) & 1 ? B[6] : 0u) ^ ((b0 >> 7) & 1 ? B[7] : 0u);
#pragma unroll
    for (int i = 1; i < 32; i++)
        T[i] = T[i & (i - 1)] ^ B[__builtin_ctz(i)];
    uint8_t* row = lds + (((q >> 6) << 16) | (b0 << 8) | ((q & 63) << 2));
#pragma unroll
    for (int i = 0; i < 32; i++)
        *reinterpret_cast<uint32_t*>(row + 256 * i) = T[i];
    if (inv) {
        const uint32_t c0 = 32 * (threadIdx.x & 7);
        uint32_t U[32];
        U[0] = ((c0 >> 5) & 1 ? iv[5] : 0u) ^ ((c0 >> 6) & 1 ? iv[6] : 0u) ^ ((c0 >> 7) & 1 ? iv[7] : 0u);
#pragma unroll
        for (int i = 1; i < 32; i++)
            U[i] = U[i & (i - 1)] ^ iv[__builtin_ctz(i)];
        uint32_t* dst = reinterpret_cast<uint32_t*>(lds + kTwInvOff) + 256 * (threadIdx.x >> 3) + c0;
#pragma unroll
        for (int i = 0; i < 32; i++)
            dst[i] = U[i];
    }
}

__device__ __forceinline__ void tiny_fill_gen(uint8_t* lds)
{
    tiny_fill_build(lds, tiny_basis_load());
}
#endif

// Per-lane address constants: byte k of a rotated dword (window position
// 32 j + 4 u + ((k + g4) & 3)) of dword pair j >> 1; + 128 for odd j.
struct TwRows {
    uint32_t lr[2][4];
    __device__ TwRows(uint32_t gl, uint32_t g4)
    {
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
            for (int k = 0; k < 4; k++)
                lr[h][k] = (uint32_t(h) << 16) | (16 * gl + 4 * ((uint32_t(k) + g4) & 3));
    }
};

// Per-lane v_perm selectors for tiny_win_wr<true>: lookup k of a dword takes
// its byte (k + g4) & 3 straight into address bits 8-15, which replaces the
// v_alignbyte rotation per dword (4 VGPRs for 32 VALU per round).
struct TwSel {
    uint32_t sel[4];
    __device__ TwSel() {}
    __device__ explicit TwSel(uint32_t g4)
    {
#pragma unroll
        for (int k = 0; k < 4; k++)
            sel[k] = 0x0C020000u | ((4u + ((uint32_t(k) + g4) & 3)) << 8);
    }
};

// The group's sum over one window's bytes in [sa, e), byte b at position o
// as X^(128 - o)(b) (relative to the window's end; all 8 lanes get it).
// kTail3: the caller knows e >= 96 for every window of the wave, so dwords
// 0-2 (window offsets below 96) need no tail mask
template <bool kLsel = false, bool kTail3 = false>
__device__ __forceinline__ uint32_t tiny_win_wr(const uint8_t* lds, const u32x4& wv, uint32_t sa,
                                                uint32_t e, const TwRows& rw, uint32_t gl, uint32_t g4,
                                                const TwSel& ts = TwSel())
{
    // tail: dword j keeps its bytes before e, clamp(e - 32 j - 4 u, 0, 4)
    const int z = 32 - 8 * int(e) + 32 * int(gl);   // bits to drop from dword 0's top
    // head: window bytes before sa lie in dword 0 of lanes 0-3
    const uint32_t hd = uint32_t(min(max(8 * (int(sa) - 4 * int(gl)), 0), 32));
    const uint32_t ws[4] = {wv.x, wv.y, wv.z, wv.w};
    uint32_t v[16];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        uint32_t keep = 0xFFFFFFFFu;
        if (!kTail3 || j == 3) {
#if RAMCRC_TINY_MED3
            // one v_med3 after the add (the compiler's max/add/min is three ops)
            uint32_t sh;
            asm("v_med3_i32 %0, %1, 0, 32" : "=v"(sh) : "v"(z + 256 * j));
#else
            const uint32_t sh = uint32_t(min(max(z + 256 * j, 0), 32));
#endif
            keep = uint32_t(uint64_t(0xFFFFFFFFu) >> sh);
        }
        if (j == 0)
            keep &= uint32_t(~uint64_t(0) << hd);
        const uint32_t xb = ws[j] & keep;
        if constexpr (kLsel) {
            // lookup k takes byte (k + g4) & 3 (conflict-free banks) through
            // the lane's own selector instead of a rotated copy of the dword
#pragma unroll
            for (int k = 0; k < 4; k++)
                v[4 * j + k] = *reinterpret_cast<const uint32_t*>(
                    lds + __builtin_amdgcn_perm(xb, rw.lr[j >> 1][k], ts.sel[k]) + 128 * (j & 1));
        } else {
            const uint32_t xr = __builtin_amdgcn_alignbyte(xb, xb, g4);   // conflict-free banks
#pragma unroll
            for (int k = 0; k < 4; k++)
                v[4 * j + k] = *reinterpret_cast<const uint32_t*>(
                    lds + __builtin_amdgcn_perm(xr, rw.lr[j >> 1][k], 0x0C020000u | ((4u + uint32_t(k)) << 8)) +
                    128 * (j & 1));
        }
    }
    const uint32_t t0 = xor3(v[0], v[1], v[2]), t1 = xor3(v[3], v[4], v[5]);
    const uint32_t t2 = xor3(v[6], v[7], v[8]), t3 = xor3(v[9], v[10], v[11]);
    const uint32_t t4 = xor3(v[12], v[13], v[14]);
    uint32_t R = xor3(xor3(t0, t1, t2), xor3(t3, t4, v[15]), 0u);
    R = group8_xor_all(R);
    return R;
}

__device__ __forceinline__ void tiny_fill(uint8_t* lds)
{
#if RAMCRC_TINY_GEN
    tiny_fill_gen(lds);
#else
    tiny_fill_wr(lds);
#endif
}

// X^m(v) for 4 <= m <= 128 (byte k at distance m - k), and X^-128(v)
__device__ __forceinline__ uint32_t tw_shift(const uint8_t* lds, uint32_t v, uint32_t m)
{
    auto t = [&](uint32_t q, uint32_t b) { return *reinterpret_cast<const uint32_t*>(lds + tw_addr(q, b)); };
    return xor3(t(128 - m, v & 0xFF), t(129 - m, (v >> 8) & 0xFF), t(130 - m, (v >> 16) & 0xFF)) ^
           t(131 - m, v >> 24);
}

__device__ __forceinline__ uint32_t tw_inv128(const uint8_t* lds, uint32_t v)
{
    auto t = [&](uint32_t k, uint32_t b) {
        return *reinterpret_cast<const uint32_t*>(lds + kTwInvOff + 4 * (256 * k + b));
    };
    return xor3(t(0, v & 0xFF), t(1, (v >> 8) & 0xFF), t(2, (v >> 16) & 0xFF)) ^ t(3, v >> 24);
}

template <bool kPF>
__device__ __forceinline__ bool tiny_run_cf(const BatchDesc& d, const Sorted& so, uint8_t* lds,
                                            bool bad, uint32_t blk, uint32_t nblk, bool need_table)
{
    const uint64_t direct_n = so.bt->direct_n;   // all tiny: the caller's table, in place
    if (!direct_n && so.bt->start[2] == so.bt->start[0]) {
        // no entry of at most one window (uniform: every wave exits); the
        // multi-window phase still needs the table
        if (need_table) {
            tiny_fill(lds);
            return !__syncthreads_or(bad);
        }
        return true;
    }
    const int lane = threadIdx.x & (kWaveSize - 1);
    const uint32_t gl = uint32_t(lane) & 7;
    const uint32_t g4 = (uint32_t(lane) >> 3) & 3;
    const uint64_t wave = uint64_t(blk) * kEntWaves +
                          __builtin_amdgcn_readfirstlane(threadIdx.x / kWaveSize);
    const uint64_t nwaves = uint64_t(nblk) * kEntWaves;
    const uint64_t s0 = direct_n ? 0 : so.bt->start[0], s1 = direct_n ? direct_n : so.bt->start[2];
    const uint64_t rounds = (s1 - s0 + 63) / 64;
    const bool finalize = d.flags & RAMCRC_FINALIZE;
    const uint64_t dummy = reinterpret_cast<uint64_t>(so.bt);
    typedef const __attribute__((address_space(1))) uint32_t g32;

    auto load_own = [&](uint64_t r) -> TinyOwn {
        TinyOwn o;
        const uint64_t sl = s0 + r * 64 + uint32_t(lane);
        u32x4 dd = {0u, 0u, 0u, 0u};
        o.ix = kNoIdx;
        o.init = 0xFFFFFFFFu;
        if (r < rounds && sl < s1) {
            if (direct_n) {   // kTable: buffer sl = base + off[sl], len[sl]; records: record sl
                uint64_t S, E;
                bool act = true;
                if (d.rec) {
                    act = buffer_range<kRecords>(d, sl, S, E);
                } else {
                    S = reinterpret_cast<uint64_t>(d.base) + d.off[sl];
                    E = S + d.len[sl];
                }
                if (act)
                    dd = u32x4{uint32_t(S), uint32_t(S >> 32), uint32_t(E), uint32_t(E >> 32)};
                o.ix = act ? uint32_t(sl) : kNoIdx;
                if (d.init)
                    o.init = d.init[sl];
                if (act && E - S >= 4 && E - (S & ~uint64_t(15)) > kStep) {
                    // not tiny after all: the histogram lied; refuse, write nothing
                    atomicOr(so.status, kStatusSticky | kStatusBins);
                    o.ix = kNoIdx;
                }
            } else {
                dd = so.desc[sl];
                o.ix = so.idx[sl];
                if (d.init)
                    o.init = so.init[sl];
            }
        }
        o.S = (uint64_t(dd.y) << 32) | dd.x;
        const uint64_t E = (uint64_t(dd.w) << 32) | dd.z;
        const uint32_t len = uint32_t(E - o.S);   // <= 128 in bins 0-1
        const uint64_t A = o.S & ~uint64_t(15);   // the window; not kept (registers)
        o.geo = (o.ix != kNoIdx && len >= 4) ? (len | (uint32_t(o.S - A) << 8)) : 0u;
        // bit 12: the whole window [A, A + 128) lies in pages that hold entry
        // bytes (or, with nothing to hash, in the bin table), so its dwords
        // can be read unclamped
        const bool safe = !o.geo || ((A + 127) >> 12) == ((E - 1) >> 12);
        o.geo |= (safe ? (1u << 12) : 0u) | (len << 16);   // len again in bits 16-23
        return o;
    };
    // the group's eight windows: dwords gl + 8 j of each owner's window.
    // Bytes outside the entry are masked, so a dword past E may hold
    // anything: when all eight windows of a q stay inside pages that hold
    // entry bytes (bit 12 of geo), the dwords are read as they are; otherwise
    // a dword that starts at or past E loads the entry's last dword instead,
    // so no load leaves the entry's last dword.
    auto issue = [&](const TinyOwn& o, u32x4 (&w)[8], uint32_t (&geo)[8], uint32_t& st) {
        st = d.vstat && o.ix != kNoIdx ? load_u32_any(o.S - 4) : 0u;
        static_for8([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            geo[q] = swz_from<q>(o.geo);
            const uint64_t Sq = (uint64_t(swz_from<q>(uint32_t(o.S >> 32))) << 32) |
                                swz_from<q>(uint32_t(o.S));
            // nothing to hash: the window loads read valid memory (the bin table)
            const uint64_t A = (geo[q] & 0xFFF) ? (Sq & ~uint64_t(15)) : dummy;
            [[maybe_unused]] const uint64_t au = A + 4 * gl;
            u32x4 v;
            if (RAMCRC_TINY_SAFE && __builtin_amdgcn_ballot_w64(!((geo[q] >> 12) & 1)) == 0) {
                // every window of this q is page-safe: plain loads, immediate offsets
                v.x = *reinterpret_cast<g32*>(au);
                v.y = *reinterpret_cast<g32*>(au + 32);
                v.z = *reinterpret_cast<g32*>(au + 64);
                v.w = *reinterpret_cast<g32*>(au + 96);
            } else {
                const uint32_t e = ((geo[q] >> 8) & 0xF) + (geo[q] & 0xFF);   // E - A (0: empty)
                const int el = (max(int(e) - 1, 0) & ~3) - int(4 * gl);   // last dword, from 4 u
                v.x = *reinterpret_cast<g32*>(au + min(0, el));
                v.y = *reinterpret_cast<g32*>(au + min(32, el));
                v.z = *reinterpret_cast<g32*>(au + min(64, el));
                v.w = *reinterpret_cast<g32*>(au + min(96, el));
            }
            w[q] = v;
        });
    };

    // RAMCRC_TINY_OVL: the table's basis words are loaded first, round 0's
    // windows issued as soon as its owners are known, and the table built
    // while those loads are in flight (the build waits for the basis alone)
    constexpr bool kOvl = RAMCRC_TINY_OVL && RAMCRC_TINY_GEN;
#if RAMCRC_TINY_GEN
    TinyBasis tb;
    if constexpr (kOvl)
        tb = tiny_basis_load();
#endif
    uint64_t r = wave;
    TinyOwn o0 = load_own(r), o1 = load_own(r + nwaves);
    u32x4 wc[8];
    uint32_t gc[8], sc;
#if RAMCRC_TINY_GEN
    if constexpr (kOvl) {
        issue(o0, wc, gc, sc);
        tiny_fill_build(lds, tb);
    } else {
        tiny_fill(lds);
    }
#else
    tiny_fill(lds);
#endif
    const TwRows rw(gl, g4);
    // without the register prefetch the selectors fit (RAMCRC_TINY_LSEL 2)
    // with the prefetch, the windows' geometry is swizzled again from the
    // owner in the compute (RAMCRC_TINY_REGEO) so that the selectors and the
    // second window body fit in the registers
    constexpr bool kRegeo = kPF && RAMCRC_TINY_REGEO;
    constexpr bool kLean = !kPF || kRegeo;
    constexpr bool kLsel = RAMCRC_TINY_LSEL == 2 ? kLean : bool(RAMCRC_TINY_LSEL);
    TwSel ts;
    if constexpr (kLsel)
        ts = TwSel(g4);
    if (__syncthreads_or(bad))
        return false;
    RAMCRC_STAMP(5);
    bool first_round = true;
    if constexpr (!kOvl)
        issue(o0, wc, gc, sc);
    for (; r < rounds; r += nwaves) {
        const TinyOwn o2 = load_own(r + 2 * nwaves);
        u32x4 wn[8];
        uint32_t gn[8], sn = 0;
        if constexpr (kPF) {
            if (r + nwaves < rounds)
                issue(o1, wn, gn, sn);
        }
        uint32_t mine = 0;
        static_for8([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            const uint32_t g = kRegeo ? swz_from<q>(o0.geo) : gc[q];
            const uint32_t sa = (g >> 8) & 0xF;
            const uint32_t e = sa + (g & 0xFF);           // window-relative end, <= 128
            // (a wave-uniform branch: entries of 81 B or more skip most tail masks)
            const bool t3 = RAMCRC_TINY_T3 && kLean && __builtin_amdgcn_ballot_w64(e < 96) == 0;
            const uint32_t R = t3 ? tiny_win_wr<kLsel, true>(lds, wc[q], sa, e, rw, gl, g4, ts)
                                  : tiny_win_wr<kLsel, false>(lds, wc[q], sa, e, rw, gl, g4, ts);
            mine = gl == uint32_t(q) ? R : mine;
        });
        // own slot: the initial state (byte k at distance len - k), or bytewise
        if (o0.ix != kNoIdx) {
            uint32_t R;
            const uint32_t n = (o0.geo >> 16) & 0xFF;   // the entry's length
            if (n >= 4) {
                // the window sum moved from the window's end to the entry's end,
                // e = S - A + n >= 4 bytes into the window
                const uint32_t e = ((o0.geo >> 8) & 0xF) + n;
                R = tw_shift(lds, tw_inv128(lds, mine), e) ^ tw_shift(lds, o0.init, n);
            } else {
                R = o0.init;
                for (uint32_t k = 0; k < n; k++)
                    R = *reinterpret_cast<const uint32_t*>(
                            lds + tw_addr(127, (R ^ *(const gu8*)(o0.S + k)) & 0xFF)) ^ (R >> 8);
            }
            const uint32_t Rf = finalize ? ~R : R;
            d.out[o0.ix] = Rf;
            if (d.vstat && Rf != sc)
                atomicAdd(&d.vstat[d.rec[o0.ix].x].bad_objects, 1u);
        }
        RAMCRC_STAMP_ONCE(6, first_round);
        o0 = o1;
        o1 = o2;
        if constexpr (kPF) {
            sc = sn;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                wc[q] = wn[q];
                gc[q] = gn[q];
            }
        } else {
            // the next round's windows straight into the spent buffer: the
            // other waves of the SIMD cover their latency
            if (r + nwaves < rounds)
                issue(o0, wc, gc, sc);
        }
    }
    return true;
}

// bins 2 .. kTinyK (see above): one entry per q as in tiny_run_cf, all K
// windows of a group's entry loaded while earlier ones are hashed: a ring of
// kDepth buffers of kK windows, the entry kDepth - 1 ahead loaded at each q.
// Bin 2 (entries of at most two windows: the objects of 128-byte values) runs
// with kK = 2 and a ring of 4 -- three entries in flight per group for the
// registers the general loop spends on two buffers of four windows; bins 3 ..
// kTinyK with kK = kTinyK and two buffers.
// kDirect: a records batch read in place (BinTable::direct_multi), record i
// at slot i; a record that is not an object of 2 .. kTinyK windows refuses the
// launch (the summary that chose this path was wrong), as the direct tiny
// path does.
template <int kK, int kDepth, bool kDirect = false>
__device__ __forceinline__ void tiny_multi_run(const BatchDesc& d, const Sorted& so, const uint8_t* lds,
                                               uint32_t blk, uint32_t nblk, uint64_t s0, uint64_t s1)
{
    static_assert(kDepth >= 2 && 8 % kDepth == 0, "tiny_multi: ring index q % kDepth must be static");
    if (s0 == s1)
        return;   // uniform
    const int lane = threadIdx.x & (kWaveSize - 1);
    const uint32_t gl = uint32_t(lane) & 7;
    const uint32_t g4 = (uint32_t(lane) >> 3) & 3;
    const uint64_t wave = uint64_t(blk) * kEntWaves +
                          __builtin_amdgcn_readfirstlane(threadIdx.x / kWaveSize);
    const uint64_t nwaves = uint64_t(nblk) * kEntWaves;
    const uint64_t rounds = (s1 - s0 + 63) / 64;
    if (wave >= rounds)
        return;   // uniform
    const bool finalize = d.flags & RAMCRC_FINALIZE;
    const uint64_t dummy = reinterpret_cast<uint64_t>(so.bt);
    typedef const __attribute__((address_space(1))) uint32_t g32;

    auto load_raw = [&](uint64_t r) -> TinyRaw {
        TinyRaw w;
        const uint64_t sl = s0 + r * 64 + uint32_t(lane);
        const bool in = r < rounds && sl < s1;
        if constexpr (kDirect) {
            uint64_t S = 0, E = 0;
            bool act = in && record_range(d, d.rec[sl], S, E);
            if (act) {
                const uint64_t k = entry_steps(S, E);
                if (k < 2 || k > uint64_t(kTinyK)) {
                    atomicOr(so.status, kStatusSticky | kStatusBins);   // refuse, write nothing
                    act = false;
                }
            }
            w.dd = u32x4{uint32_t(S), uint32_t(S >> 32), uint32_t(E), uint32_t(E >> 32)};
            w.ix = act ? uint32_t(sl) : kNoIdx;
            w.init = d.init && in ? d.init[sl] : 0xFFFFFFFFu;
        } else {
            const uint64_t sc = in ? sl : s0;
            w.dd = so.desc[sc];
            const uint32_t ix = so.idx[sc];
            w.ix = in ? ix : kNoIdx;
            w.init = d.init ? so.init[sc] : 0xFFFFFFFFu;
        }
        return w;
    };
    auto own_of = [&](const TinyRaw& w) -> TinyCf {
        TinyCf o;
        o.ix = w.ix;
        o.init = w.init;
        uint64_t S = (uint64_t(w.dd.y) << 32) | w.dd.x, E = (uint64_t(w.dd.w) << 32) | w.dd.z;
        if (o.ix == kNoIdx)
            S = E = dummy;
        o.S = S;
        const uint32_t len = uint32_t(E - S);
        const uint64_t A = S & ~uint64_t(15);
        o.geo = (len >= 4 ? uint32_t(E - A) : 0u) | (uint32_t(S - A) << 10) | (len << 16);
        return o;
    };
    // the owner's stored object checksum (records mode) and the word holding
    // the entry's last three bytes (its bytewise tail), a round ahead
    auto own_loads = [&](const TinyCf& o, uint32_t& st, uint32_t& tw) {
        st = d.vstat && o.ix != kNoIdx ? load_u32_any(o.S - 4) : 0u;
        const uint64_t E = o.S + ((o.geo >> 16) & 0x3FF);
        const uint64_t a = o.ix != kNoIdx ? E - 3 : dummy;   // entries here hold >= 113 bytes
        const uint64_t b = o.ix != kNoIdx ? E - 1 : dummy;
        const uint32_t w0 = *reinterpret_cast<g32*>(a & ~uint64_t(3));
        const uint32_t w1 = *reinterpret_cast<g32*>(b & ~uint64_t(3));
        tw = __builtin_amdgcn_alignbyte(w1, w0, uint32_t(a) & 3);   // bytes E - 3, E - 2, E - 1
    };
    const TwRows rw(gl, g4);
    // the windows of the entry (geo, S) into w: window k is [A + 128 k, + 128);
    // a dword at or past the window's last entry byte reads that byte's dword
    auto load_entry = [&](uint32_t geo, uint64_t S, u32x4 (&w)[kK]) {
        const uint32_t K = tk_windows(geo);
        const uint32_t el = (geo & 0x3FF) - tk_tail(geo) - 128 * (K - 1);   // last window's end
        const uint64_t au = (S & ~uint64_t(15)) + 4 * gl;
#pragma unroll
        for (int k = 0; k < kK; k++) {
            if (uint32_t(k) < K) {
                const uint32_t e = uint32_t(k) + 1 == K ? el : 128u;
                const int lim = (max(int(e) - 1, 0) & ~3) - int(4 * gl);
                const uint64_t aw = au + 128 * uint64_t(k);
                w[k].x = *reinterpret_cast<g32*>(aw + min(0, lim));
                w[k].y = *reinterpret_cast<g32*>(aw + min(32, lim));
                w[k].z = *reinterpret_cast<g32*>(aw + min(64, lim));
                w[k].w = *reinterpret_cast<g32*>(aw + min(96, lim));
            }
        }
    };
    // entry qe of the round whose owners are `on` (swizzled from lane 8g + qe)
    auto load_q = [&](auto qc, const TinyCf& on, bool valid, uint32_t& gq, u32x4 (&w)[kK]) {
        constexpr int qe = decltype(qc)::value;
        uint32_t g = swz_from<qe>(on.geo);
        g = valid ? g : 0u;
        const uint64_t Sn = (uint64_t(swz_from<qe>(uint32_t(on.S >> 32))) << 32) | swz_from<qe>(uint32_t(on.S));
        gq = g;
        load_entry(g, Sn, w);
    };

    uint64_t r = wave;
    TinyRaw w1 = load_raw(r + nwaves);
    TinyCf o0 = own_of(load_raw(r));
    uint32_t sc, tc;
    own_loads(o0, sc, tc);
    u32x4 buf[kDepth][kK];
    uint32_t gq[kDepth];
    // the ring's first kDepth - 1 entries
    static_for8([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (j < kDepth - 1)
            load_q(jc, o0, true, gq[j], buf[j]);
    });
    for (; r < rounds; r += nwaves) {
        const TinyRaw w2 = load_raw(r + 2 * nwaves);
        const TinyCf o1 = own_of(w1);   // loaded a round ago
        const bool more = r + nwaves < rounds;
        uint32_t sn = 0, tn = 0;
        own_loads(o1, sn, tn);
        uint32_t mine = 0;
        static_for8([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            // the group's entry kDepth - 1 ahead: of this round, or of the next
            {
                constexpr int qn = q + kDepth - 1;
                constexpr int bn = qn % kDepth;
                if constexpr (qn < 8)
                    load_q(std::integral_constant<int, qn>{}, o0, true, gq[bn], buf[bn]);
                else
                    load_q(std::integral_constant<int, qn - 8>{}, o1, more, gq[bn], buf[bn]);
            }
            constexpr int bq = q % kDepth;
            const uint32_t geo = gq[bq];
            const uint32_t K = tk_windows(geo);
            const uint32_t el = (geo & 0x3FF) - tk_tail(geo) - 128 * (K - 1);
            // window sums at their distance from their window's end; Horner with
            // X^128 between windows: acc is relative to the last window's end
            uint32_t acc = tiny_win_wr(lds, buf[bq][0], (geo >> 10) & 0xF,
                                       K > 1 ? 128u : (K ? el : 0u), rw, gl, g4);
#pragma unroll
            for (int k = 1; k < kK; k++) {
                if (__builtin_amdgcn_ballot_w64(uint32_t(k) < K)) {   // uniform
                    const uint32_t e = uint32_t(k) + 1 == K ? el : 128u;
                    const uint32_t R = tiny_win_wr(lds, buf[bq][k], 0, uint32_t(k) < K ? e : 0u, rw, gl, g4);
                    // X^128(acc) by lanes gl & 3 (byte gl & 3 at distance 128 - (gl & 3))
                    const uint32_t kk = gl & 3;
                    uint32_t X = *reinterpret_cast<const uint32_t*>(lds + tw_addr(kk, (acc >> (8 * kk)) & 0xFF));
                    X ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(X), 0xB1, 0xF, 0xF, false));
                    X ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(X), 0x4E, 0xF, 0xF, false));
                    acc = uint32_t(k) < K ? (X ^ R) : acc;
                }
            }
            mine = gl == uint32_t(q) ? acc : mine;
        });
        // own slot: the initial state X^(n - tail)(init) in steps of at most 128,
        // then the tail bytewise
        if (o0.ix != kNoIdx) {
            const uint32_t n = (o0.geo >> 16) & 0x3FF, tail = tk_tail(o0.geo);
            const uint32_t K = tk_windows(o0.geo);
            const uint32_t el = (o0.geo & 0x3FF) - tail - 128 * (K - 1);   // >= 4
            uint32_t v = o0.init, m = n - tail;
            while (m > 128) {
                const uint32_t st = m - 128 >= 4 ? 128u : m - 4;
                v = tw_shift(lds, v, st);
                m -= st;
            }
            // the windows' sum moved from the last window's end to E - tail
            uint32_t R = tw_shift(lds, tw_inv128(lds, mine), el) ^ tw_shift(lds, v, m);
            for (uint32_t k = 3 - tail; k < 3; k++)   // bytes E - tail .. E - 1
                R = *reinterpret_cast<const uint32_t*>(lds + tw_addr(127, (R ^ (tc >> (8 * k))) & 0xFF)) ^
                    (R >> 8);
            const uint32_t Rf = finalize ? ~R : R;
            d.out[o0.ix] = Rf;
            if (d.vstat && Rf != sc)
                atomicAdd(&d.vstat[d.rec[o0.ix].x].bad_objects, 1u);
        }
        o0 = o1;
        w1 = w2;
        sc = sn;
        tc = tn;
    }
}

__device__ __forceinline__ void tiny_multi(const BatchDesc& d, const Sorted& so, const uint8_t* lds,
                                           uint32_t blk, uint32_t nblk)
{
    if constexpr (kTinyK >= 2) {
        if (RAMCRC_TINY_DM && so.bt->direct_multi) {
            if (RAMCRC_TINY_M2 && kTinyK > 2 && so.bt->direct_multi_k2)
                tiny_multi_run<2, 4, true>(d, so, lds, blk, nblk, 0, so.bt->direct_multi);
            else
                tiny_multi_run<kTinyK, 2, true>(d, so, lds, blk, nblk, 0, so.bt->direct_multi);
            return;
        }
        const uint64_t s0 = so.bt->start[2], s1 = so.bt->start[kTinyK + 1];
        if (s0 == s1)
            return;   // uniform
        if constexpr (RAMCRC_TINY_M2 && kTinyK > 2) {
            const uint64_t s2 = so.bt->start[3];
            tiny_multi_run<2, 4>(d, so, lds, blk, nblk, s0, s2);
            tiny_multi_run<kTinyK, 2>(d, so, lds, blk, nblk, s2, s1);
        } else {
            tiny_multi_run<kTinyK, 2>(d, so, lds, blk, nblk, s0, s1);
        }
    }
}

// Entries of two or more 128-byte steps (bins >= 2).  One octet (8 entries,
// one per lane group) at a time:
//   step 0 (head)          start mask and init injection, precomputed per octet;
//   steps 1 .. Kmin-2      interior for every entry of the octet: no masks,
//                          unconditional loads, kPU-deep ping-pong prefetch;
//   steps Kmin-1 .. Koct-1 tail: end mask, lanes past their entry frozen.
// The head and the first two tail loads are issued with the interior ones, the
// next octet's descriptor is prefetched, and the previous octet's fold runs
// after this octet's loads are in flight.  The unpad multiply x^(-8 pad) is
// batched: lane gl of a group keeps the fold of octet gl of the current eight,
// and one wave-wide multiply finishes 64 entries.  Waves split the bins by
// estimated work (steps + kOctetCost per octet).
//
// kSmall: bins 2 .. kSmallK (whole octets loaded one ahead); otherwise bins
// kSmallK+1 and up.  Two instantiations keep the register allocation of the
// long-entry loop free of the short-entry loop's state.
template <bool kSmall>
__device__ __forceinline__ void entries_run(const BatchDesc& d, const Sorted& so, const uint8_t* lds,
                                            uint32_t blk, uint32_t nblk)
{
    constexpr int kT = kTinyK > kSmallK ? kTinyK : kSmallK;
    constexpr int b0 = kSmall ? (kTinyK > 1 ? kTinyK + 1 : 2) : kT + 1, b1 = kSmall ? kSmallK + 1 : kNB;
    if (b0 >= b1)
        return;
    const uint64_t* s_items = reinterpret_cast<const uint64_t*>(lds + kBinOff);   // kNB + 1
    const uint64_t* s_start = s_items + (kNB + 1);                                // kNB
    const uint32_t* s_cost = reinterpret_cast<const uint32_t*>(s_start + kNB);    // kNB
    if (s_items[b0] == s_items[b1])
        return;   // no entry in this phase's bins (uniform)
    const uint32_t* xinv = reinterpret_cast<const uint32_t*>(lds + kXinvOff);

    const int lane = threadIdx.x & (kWaveSize - 1);
    const int g = lane >> 3, gl = lane & 7;
    const RepOp op(lane);
    const uint64_t wave = uint64_t(blk) * kEntWaves +
                          __builtin_amdgcn_readfirstlane(threadIdx.x / kWaveSize);
    const uint64_t nwaves = uint64_t(nblk) * kEntWaves;
    const uint64_t I0 = s_items[b0], T = s_items[b1] - I0;
    const bool finalize = d.flags & RAMCRC_FINALIZE;
    const uint64_t dummy = reinterpret_cast<uint64_t>(so.bt);   // device memory, 16 B aligned

    // batched unpad: lane gl holds octet gl of the current batch of eight
    uint32_t bY = 0, bPad = 0, bIx = kNoIdx, bSt = 0;
    int nb = 0;
    auto flush_batch = [&]() {
        const uint32_t R = mulmod_horner(bY, xinv[bPad & 255]);
        if (bIx != kNoIdx) {
            const uint32_t Rf = finalize ? ~R : R;
            d.out[bIx] = Rf;
            if (d.vstat && Rf != bSt)   // ObjectManager::replaySegment's check (:659-663)
                atomicAdd(&d.vstat[d.rec[bIx].x].bad_objects, 1u);
        }
        bIx = kNoIdx;
        nb = 0;
    };
    // deferred fold of the previous octet
    bool pend = false;
    uint32_t pu0 = 0, pu1 = 0, pu2 = 0, pu3 = 0, ppad = 0, pix = kNoIdx, pst = 0;
    auto flush = [&]() {
        if (pend) {
            const uint32_t Y = group_fold(lds, gl, pu0, pu1, pu2, pu3);
            if (gl == nb) {
                bY = Y;
                bPad = ppad;
                bIx = pix;
                bSt = pst;
            }
            pend = false;
            if (++nb == kG)
                flush_batch();
        }
    };

    // the octets whose first work unit lies in [lo, hi)
    auto run = [&](const uint64_t lo, const uint64_t hi) {
        for (int b = b0; b < b1; b++) {
            const uint64_t ib = s_items[b], ie = s_items[b + 1];
            if (ie <= lo || ib == ie)
                continue;
            if (ib >= hi)
                break;
            const uint64_t cost = s_cost[b];
            const uint64_t oa = ((lo > ib ? lo : ib) - ib + cost - 1) / cost;
            const uint64_t ob = ((hi < ie ? hi : ie) - ib + cost - 1) / cost;
            const uint64_t sb = s_start[b];
            if (oa >= ob)
                continue;
            if constexpr (kSmall) {
                // Exact bins of at most kSmallK steps: the whole octet is loaded
                // one octet ahead, so the load latency hides behind the previous
                // octet's steps and fold instead of stalling every octet.
                const uint32_t K = uint32_t(b);
                struct Oct {
                    uint64_t S, E;
                    uint32_t init, ix, steps, st, st1;   // st, st1: dwords around the stored checksum
                    u32x4 w[kSmallK + 1];
                };
                auto load_oct = [&](uint64_t o, Oct& t) {
                    const uint64_t sl = sb + o * kG + g;
                    const u32x4 dd = so.desc[sl];
                    t.ix = so.idx[sl];
                    t.init = d.init ? so.init[sl] : 0xFFFFFFFFu;
                    t.S = (uint64_t(dd.y) << 32) | dd.x;
                    t.E = (uint64_t(dd.w) << 32) | dd.z;
                    t.steps = t.ix != kNoIdx ? uint32_t(entry_steps_line(t.S, t.E)) : 0u;   // K or K+1
                    const uint64_t A = line_base(t.S);
                    const uint64_t p0 = A + gl * 16;
                    const uint64_t safe = t.steps ? A : dummy;
                    t.st = t.st1 = 0u;   // joined at use: a join here would wait for them
                    if (d.vstat && t.steps) {
                        typedef const __attribute__((address_space(1))) uint32_t g32s;
                        const uint64_t sa = (t.S - 4) & ~uint64_t(3);
                        t.st = *reinterpret_cast<g32s*>(sa);
                        t.st1 = *reinterpret_cast<g32s*>(sa + 4);
                    }
    #pragma unroll
                    for (int k = 0; k <= kSmallK; k++) {
                        const uint64_t a = p0 + uint64_t(k) * kStep;
                        if (k <= int(K))
                            t.w[k] = load16(t.steps && a < t.E ? a : safe);
                    }
                };
                Oct cur, nxt;
                load_oct(oa, cur);
                for (uint64_t o = oa; o < ob; o++) {
                    if (o + 1 < ob)
                        load_oct(o + 1, nxt);
                    const uint64_t A = line_base(cur.S);
                    const uint64_t p0 = A + gl * 16;
                    uint32_t u0 = 0, u1 = 0, u2 = 0, u3 = 0;
                    {
                        const int off = int(uint32_t(cur.S - A)) - 16 * gl;
                        u32x4 w = cur.w[0];
                        w.x = head_word(w.x, off, cur.init);
                        w.y = head_word(w.y, off - 4, cur.init);
                        w.z = head_word(w.z, off - 8, cur.init);
                        w.w = head_word(w.w, off - 12, cur.init);
                        op.apply4(lds, u0, u1, u2, u3, w);
                    }
                    const int64_t erel = int64_t(cur.E - p0);
    #pragma unroll
                    for (int k = 1; k <= kSmallK; k++) {
                        if (k <= int(K)) {
                            const int64_t de64 = erel - int64_t(k) * int64_t(kStep);
                            const int de = int(de64 < 0 ? 0 : (de64 > 16 ? 16 : de64));
                            u32x4 w = cur.w[k];
                            w.x &= keep_lo(de);
                            w.y &= keep_lo(de - 4);
                            w.z &= keep_lo(de - 8);
                            w.w &= keep_lo(de - 12);
                            const bool live = uint32_t(k) < cur.steps;
                            uint32_t v0 = u0, v1 = u1, v2 = u2, v3 = u3;
                            op.apply4(lds, v0, v1, v2, v3, w);
                            u0 = live ? v0 : u0;
                            u1 = live ? v1 : u1;
                            u2 = live ? v2 : u2;
                            u3 = live ? v3 : u3;
                        }
                    }
                    pend = true;
                    pu0 = u0;
                    pu1 = u1;
                    pu2 = u2;
                    pu3 = u3;
                    ppad = uint32_t((A + uint64_t(cur.steps) * kStep) - cur.E);
                    pix = cur.ix;
                    pst = __builtin_amdgcn_alignbyte(cur.st1, cur.st, uint32_t(cur.S - 4) & 3);
                    flush();
                    cur = nxt;
                }
            }
        }
    };
    // One octet of a long bin b: 8 entries, one per lane group.
    auto octet = [&](const u32x4 dd, const uint32_t ix, const uint32_t init, const int b) {
            const uint64_t S = (uint64_t(dd.y) << 32) | dd.x;
            const uint64_t E = (uint64_t(dd.w) << 32) | dd.z;
            const uint32_t steps = ix != kNoIdx ? uint32_t(entry_steps_line(S, E)) : 0u;
            const uint64_t A = line_base(S);   // windows on 128-byte lines
            const uint64_t p0 = A + gl * 16;
            // longest / shortest entry of the octet (padding slots excluded)
            uint32_t Koct, Kmin;
            if (b <= 32) {
                // exact bin b: a step count is b or b + 1 (line_base(S) lies
                // at most 112 bytes before the 16-byte piece of S)
                const bool hi = __ballot(steps == uint32_t(b) + 1) != 0;
                const bool lo1 = __ballot(steps == uint32_t(b)) != 0;
                Koct = hi ? uint32_t(b) + 1 : (lo1 ? uint32_t(b) : 0u);
                Kmin = lo1 ? uint32_t(b) : uint32_t(b) + 1;
            } else {
                uint32_t kmax32 = steps, kmin32 = steps ? steps : 0xFFFFFFFFu;
#pragma unroll
                for (int s = 8; s < 64; s <<= 1) {
                    kmax32 = max(kmax32, uint32_t(__shfl_xor(kmax32, s, kWaveSize)));
                    kmin32 = min(kmin32, uint32_t(__shfl_xor(kmin32, s, kWaveSize)));
                }
                Koct = __builtin_amdgcn_readfirstlane(kmax32);
                Kmin = __builtin_amdgcn_readfirstlane(kmin32);   // >= 2
            }
            if (Koct == 0)
                return;   // an octet of padding slots only: none in a consistent layout
                          // (each bin's last octet holds >= 1 entry), but Kmin - 1
                          // would bound the interior loop at 2^32 steps
            const uint32_t kt0 = Kmin - 1;   // first tail step (>= 1)
            const uint64_t safe = steps ? A : dummy;

            // loads: head, first two tail steps, first kPU interior steps
            const gu32x4* pb = gptr16(steps ? p0 : dummy);
            const uint64_t bstride = steps ? kStep / 16 : 0;
#if RAMCRC_ENT_NT
            auto ldf = [&](uint64_t k) -> u32x4 { return __builtin_nontemporal_load(pb + k * bstride); };
#else
            auto ldf = [&](uint64_t k) -> u32x4 { return pb[k * bstride]; };
#endif
            auto ldt = [&](uint32_t k) -> u32x4 {   // tail step: lanes past E read a safe word
                const uint64_t a = p0 + uint64_t(k) * kStep;
                return load16(k < steps && a < E ? a : safe);
            };
            const u32x4 wh = ldf(0);
            const u32x4 wt0 = ldt(kt0);
            const u32x4 wt1 = ldt(kt0 + 1 < Koct ? kt0 + 1 : kt0);
            u32x4 Abuf[kPU], Bbuf[kPU];
#pragma unroll
            for (int j = 0; j < kPU; j++)
                Abuf[j] = ldf(1 + j < kt0 ? 1 + j : 0);
            // the stored checksum (records mode) behind the data loads; read at
            // the octet's end
            // (its two dwords are loaded here and joined at the octet's end:
            // joining them here would wait for every load above before the
            // previous octet's fold, exposing one memory latency per octet)
            typedef const __attribute__((address_space(1))) uint32_t g32s;
            uint32_t sw0 = 0u, sw1 = 0u;
            if (d.vstat && steps) {
                const uint64_t sa = (S - 4) & ~uint64_t(3);
                sw0 = *reinterpret_cast<g32s*>(sa);
                sw1 = *reinterpret_cast<g32s*>(sa + 4);
            }
            __builtin_amdgcn_sched_barrier(0);
            flush();

            uint32_t u0 = 0, u1 = 0, u2 = 0, u3 = 0;
            auto stepf = [&](const u32x4& w) { op.apply4(lds, u0, u1, u2, u3, w); };
            // head: keep bytes >= S, inject init at S .. S+3 (masks and
            // v_perm selectors from the LDS table of the piece's offset)
            if (RAMCRC_PROBE_MASK) {
                stepf(wh);
            } else {
                const int off = int(uint32_t(S - A)) - 16 * gl;   // S - p0
                const int c = min(max(off, -4), 16) + 4;
                const u32x4* ht = reinterpret_cast<const u32x4*>(lds + kHeadOff) + 2 * c;
                const u32x4 m = ht[0], sl = ht[1];
                u32x4 w;
                w.x = (wh.x & m.x) ^ __builtin_amdgcn_perm(init, 0u, sl.x);
                w.y = (wh.y & m.y) ^ __builtin_amdgcn_perm(init, 0u, sl.y);
                w.z = (wh.z & m.z) ^ __builtin_amdgcn_perm(init, 0u, sl.z);
                w.w = (wh.w & m.w) ^ __builtin_amdgcn_perm(init, 0u, sl.w);
                stepf(w);
            }
            // interior
            uint32_t k = 1;
            for (; k + 2 * kPU <= kt0; k += 2 * kPU) {
#pragma unroll
                for (int j = 0; j < kPU; j++)
                    Bbuf[j] = ldf(k + kPU + j);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < kPU; j++)
                    stepf(Abuf[j]);
#pragma unroll
                for (int j = 0; j < kPU; j++)
                    Abuf[j] = ldf(k + 2 * kPU + j < kt0 ? k + 2 * kPU + j : 0);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < kPU; j++)
                    stepf(Bbuf[j]);
            }
#pragma unroll
            for (int j = 0; j < kPU; j++)
                if (k + j < kt0)
                    stepf(Abuf[j]);
            if (k + kPU < kt0) {
#pragma unroll
                for (int j = 0; j < kPU; j++)
                    Bbuf[j] = ldf(k + kPU + j < kt0 ? k + kPU + j : 0);
#pragma unroll
                for (int j = 0; j < kPU; j++)
                    if (k + kPU + j < kt0)
                        stepf(Bbuf[j]);
            }
            // tail: keep bytes < E (masks from the LDS table of the bytes
            // left).  Every entry of the octet is live at step kt0; at
            // kt0 + 1 the ones that have ended take one more step of zeros
            // (no select: their padding grows by 128 bytes, < 256); the
            // ragged steps of log-scale bins freeze ended entries.
            const uint64_t trel64 = E - (p0 + uint64_t(kt0) * kStep);   // > 0 for live lanes
            const int trel = int(trel64 > 1024 && int64_t(trel64) > 0 ? 1024 : int64_t(trel64));
            const u32x4* tt = reinterpret_cast<const u32x4*>(lds + kTailOff);
            auto stepm = [&](u32x4 w, int de) {
                if (!RAMCRC_PROBE_MASK) {
                    const u32x4 m = tt[min(max(de, 0), 16)];
                    w.x &= m.x;
                    w.y &= m.y;
                    w.z &= m.z;
                    w.w &= m.w;
                }
                stepf(w);
            };
            stepm(wt0, trel);
            uint32_t eff = steps;   // steps the group ran for this entry
            if (kt0 + 1 < Koct) {
                stepm(wt1, trel - int(kStep));
                eff = steps > kt0 + 2 ? steps : kt0 + 2;
            }
            const int64_t erel = int64_t(E - p0);
            for (uint32_t kk = kt0 + 2; kk < Koct; kk++) {   // ragged octets (log-scale bins)
                const int64_t de64 = erel - int64_t(kk) * int64_t(kStep);
                const uint32_t p0v = u0, p1v = u1, p2v = u2, p3v = u3;
                stepm(ldt(kk), int(de64 < 0 ? 0 : (de64 > 16 ? 16 : de64)));
                const bool live = kk < steps;
                u0 = live ? u0 : p0v;
                u1 = live ? u1 : p1v;
                u2 = live ? u2 : p2v;
                u3 = live ? u3 : p3v;
            }

            pend = true;
            pu0 = u0;
            pu1 = u1;
            pu2 = u2;
            pu3 = u3;
            ppad = uint32_t((A + uint64_t(eff) * kStep) - E);
            pix = ix;
            pst = __builtin_amdgcn_alignbyte(sw1, sw0, uint32_t(S - 4) & 3);
    };

    // Work split.  Waves given equal shares of the long bins finish in the
    // order they were created (phase stamps, tools/stamps.py, 1M x 4 KiB:
    // the four oldest waves of a workgroup -- one per SIMD -- end at 564 us,
    // the next four at 588, then 617, the youngest four at 657: each SIMD
    // issues by age).  Each workgroup's share is therefore split among its
    // waves by age rank (slot / 4): older waves get age_weight(rank) / 2000 of
    // an equal share.  The octets of a wave's range form one stream: the next
    // octet's descriptor is always fetched one octet ahead, across bin
    // boundaries too.  (Taking part of the share from a counter instead -- one
    // LDS counter per workgroup or one device counter -- cost 1.6-2.7x, about
    // 1-2 us per chunk; DESIGN.md section 5.4, profiles/r03/long.)
    if constexpr (kSmall) {
        run(I0 + T * wave / nwaves, I0 + T * (wave + 1) / nwaves);
    } else {
        const uint64_t P0 = I0 + T * blk / nblk, PT = I0 + T * (blk + 1) / nblk - P0;
        const uint32_t slot = __builtin_amdgcn_readfirstlane(threadIdx.x / kWaveSize);
        // cumulative weight of the slots before `slot` (4 slots per age rank)
        const int skew = d.vstat ? kAgeSkewRec : kAgeSkew;
        auto cum = [&](uint32_t sl) -> uint64_t {
            uint64_t c = 0;
#pragma unroll
            for (uint32_t r = 0; r < kEntWaves / 4; r++) {
                const uint32_t n = sl > 4 * r ? (sl - 4 * r < 4 ? sl - 4 * r : 4) : 0;
                c += uint64_t(n) * age_weight(r, skew);
            }
            return c;
        };
        const uint64_t tot = cum(kEntWaves);
        const uint64_t rlo = P0 + PT * cum(slot) / tot, rhi = P0 + PT * cum(slot + 1) / tot;
        struct Pos {
            int b;
            uint64_t o, ob, sb;
        };
        // first octet of [rlo, rhi) in bins >= bs
        auto seek = [&](int bs, Pos& p) -> bool {
            for (int b = bs; b < b1; b++) {
                const uint64_t ib = s_items[b], ie = s_items[b + 1];
                if (ie <= rlo || ib == ie)
                    continue;
                if (ib >= rhi)
                    return false;
                const uint64_t cost = s_cost[b];
                const uint64_t oa = ((rlo > ib ? rlo : ib) - ib + cost - 1) / cost;
                const uint64_t ob = ((rhi < ie ? rhi : ie) - ib + cost - 1) / cost;
                if (oa >= ob)
                    continue;
                p.b = b;
                p.o = oa;
                p.ob = ob;
                p.sb = s_start[b];
                return true;
            }
            return false;
        };
        // the octet after p: in its bin, else the first of the next bins
        auto advance = [&](Pos& p) -> bool {
            if (p.o + 1 < p.ob) {
                p.o++;
                return true;
            }
            return seek(p.b + 1, p);
        };
        Pos cur;
        bool have = seek(b0, cur);
        u32x4 nd = {0u, 0u, 0u, 0u};
        uint32_t nix = kNoIdx, ninit = 0xFFFFFFFFu;
        auto fetch = [&](const Pos& p) {
            const uint64_t sl = p.sb + p.o * kG + g;
            nd = so.desc[sl];
            nix = so.idx[sl];
            if (d.init)
                ninit = so.init[sl];
        };
        if (have)
            fetch(cur);
        while (have) {
            const u32x4 dd = nd;
            const uint32_t ix = nix, init = ninit;
            const int b = cur.b;
            Pos nxt = cur;
            have = advance(nxt);
            if (have)   // prefetch the next octet's descriptor
                fetch(nxt);
            octet(dd, ix, init, b);
            cur = nxt;
        }
    }
    flush();
    if (nb)
        flush_batch();
}

// The long-phase tables into the LDS, then the short and the long bins over
// workgroups blk of nblk.  Refuses (status bits) on an inconsistent layout.
__device__ __forceinline__ void long_phase(const BatchDesc& d, const Sorted& so, uint8_t* lds, bool bad,
                                           uint32_t blk, uint32_t nblk)
{
    fill_long(lds);
    uint64_t* s_items = reinterpret_cast<uint64_t*>(lds + kBinOff);   // kNB + 1
    uint64_t* s_start = s_items + (kNB + 1);                          // kNB
    uint32_t* s_cost = reinterpret_cast<uint32_t*>(s_start + kNB);    // kNB
    for (int t = threadIdx.x; t <= kNB; t += blockDim.x) {
        s_items[t] = so.bt->items[t];
        if (t < kNB) {
            s_start[t] = so.bt->start[t];
            s_cost[t] = uint32_t(so.bt->kcost[t]);
        }
    }
    if (__syncthreads_or(bad)) {
        if (blockIdx.x == 0 && threadIdx.x == 0)
            atomicOr(so.status, kStatusSticky | kStatusBins);
        return;
    }
    RAMCRC_STAMP(2);
    entries_run<true>(d, so, lds, blk, nblk);
    RAMCRC_STAMP(3);
    entries_run<false>(d, so, lds, blk, nblk);
    RAMCRC_STAMP(4);
}

// Both phases in one launch (one LDS fill, one launch boundary): the exact
// short bins, then the pipelined long bins.  The phases are separate inlined
// loops, so the long-entry loop's registers are not shared with the short one.
__global__ __launch_bounds__(kEntWaves * kWaveSize, 1) void k_entries(BatchDesc d, Sorted so)
{
    static_assert(RAMCRC_TINY_CF, "k_entries runs the conflict-free tiny phases");
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsEntries];
    // Every bin must hold exactly the entries the scatter placed in it
    // (cursor == count): then every sorted slot this launch reads was written
    // by this sequence.  Checked at the first barrier of each phase, before
    // any slot's contents are used; a mismatch refuses the launch (no output
    // written, status bits kStatusSticky | kStatusBins, RAMCRC_EINTERNAL from
    // ramcrc_ctx_check) instead of walking stale slots.
    const bool bad = threadIdx.x < kNB &&
                     so.bt->ctr[so.par].cursor[threadIdx.x] != so.bt->count[threadIdx.x];
    auto refuse = [&]() {
        if (blockIdx.x == 0 && threadIdx.x == 0)
            atomicOr(so.status, kStatusSticky | kStatusBins);
    };
    RAMCRC_STAMP(0);
    const bool have_tk = kTinyK >= 2 && !so.bt->direct_n &&
                         (so.bt->direct_multi || so.bt->start[kTinyK + 1] != so.bt->start[2]);
    // Role split (round 5, RAMCRC_SPLIT): when a batch has both tiny and long
    // entries, workgroups < T run only the tiny phases (filling only their
    // table) and the others only the long phase, so the two overlap and no
    // workgroup waits for its slowest tiny wave before refilling its LDS.  T
    // follows the work: a tiny window costs kSplitKappa / 1024 long-phase work
    // units.  T = 0: both phases on every workgroup, in sequence.
    uint32_t T = 0;
    constexpr int kT = kTinyK > kSmallK ? kTinyK : kSmallK;
    if (RAMCRC_SPLIT && !so.bt->direct_n && so.bt->start[kTinyK + 1] != so.bt->start[0] &&
        so.bt->items[kNB] != so.bt->items[kT + 1]) {
        uint64_t win = so.bt->start[2] - so.bt->start[0];   // one window each
        for (int b = 2; b <= kTinyK; b++)
            win += (so.bt->start[b + 1] - so.bt->start[b]) * uint64_t(b);
        const uint64_t ct = win * kSplitKappa / 1024, cl = so.bt->items[kNB] - so.bt->items[kT + 1];
        T = uint32_t((uint64_t(gridDim.x) * ct + (ct + cl) / 2) / (ct + cl));
        T = T < 1 ? 1 : (T > gridDim.x - 1 ? gridDim.x - 1 : T);
    }
    const bool do_tiny = T == 0 || blockIdx.x < T, do_long = T == 0 || blockIdx.x >= T;
    const uint32_t tn = T ? T : gridDim.x;
    bool tiny_ok = true;
    if (do_tiny) {
        // records (replay) keep the register prefetch: without it their
        // tiny phase measured 3-4 % slower; table batches 5-7 % faster
        tiny_ok = (RAMCRC_TINY_PF == 2 ? d.rec != nullptr : bool(RAMCRC_TINY_PF))
                      ? tiny_run_cf<true>(d, so, lds, bad, blockIdx.x, tn, have_tk)
                      : tiny_run_cf<false>(d, so, lds, bad, blockIdx.x, tn, have_tk);
        if (tiny_ok && have_tk)
            tiny_multi(d, so, lds, blockIdx.x, tn);
    }
    RAMCRC_STAMP(1);
    if (!tiny_ok) {
        refuse();
        return;
    }
    if (!do_long)
        return;
    if (so.bt->items[2] == so.bt->items[kNB]) {   // every entry is tiny (or large on the batch path)
        if (__syncthreads_or(bad))
            refuse();
        return;
    }
    // the position table is dead (when this workgroup ran the tiny phases)
    __syncthreads();
    long_phase(d, so, lds, bad, blockIdx.x - T, gridDim.x - T);
}

// ------------------------------------------------------------ k_plan
template <int kMode>
__global__ __launch_bounds__(kThreads) void k_plan_count(BatchDesc d, Plan pl)
{
    __shared__ uint64_t wsum[kWavesPerGroup];
    if (plan_empty(pl))
        return;   // no large buffer: nothing reads local[] / group_pref[] of this launch
    // groups of kThreads entries, grid-stride (the grid is capped: a batch of
    // tens of millions of records launches few workgroups when it has no
    // large buffer and every one of them returns above)
    const uint64_t n = entry_count<kMode>(d);
    for (uint64_t grp = blockIdx.x; grp < pl.ngroups; grp += gridDim.x) {
        const uint64_t i = grp * kThreads + threadIdx.x;
        uint64_t c = 0;
        if (i < n) {   // local[] is still written for every i < d.n
            uint64_t S, E;
            buffer_range<kMode>(d, i, S, E);
            c = is_large(E - S) ? chunk_count(S, E, d.cshift) : 0;
        }
        // exclusive scan over the workgroup: in-wave inclusive scan, then waves
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        uint64_t x = c;
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {
            const uint64_t y = __shfl_up(x, s, kWaveSize);
            if (lane >= s)
                x += y;
        }
        if (lane == 63)
            wsum[w] = x;
        __syncthreads();
        uint64_t before = 0;
        for (int j = 0; j < w; j++)
            before += wsum[j];
        if (i < d.n)
            pl.local[i] = before + x - c;
        if (threadIdx.x == kThreads - 1)
            pl.group_pref[grp] = before + x;   // group total, scanned by k_plan_scan
        __syncthreads();   // wsum is reused by the next group
    }
}

__global__ __launch_bounds__(kThreads) void k_plan_scan(Plan pl)
{
    // single workgroup: exclusive scan of ngroups totals in place, [ngroups] = total
    __shared__ uint64_t wsum[kWavesPerGroup];
    __shared__ uint64_t carry_s;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        carry_s = 0;
        // stream-ordered before this launch's k_chunks; atomic so that a
        // sticky bit set concurrently by another stream's launch survives
        atomicAnd(pl.status, ~kStatusRefused);
        *pl.ticket = 0;
    }
    if (plan_empty(pl)) {
        if (threadIdx.x == 0)
            pl.group_pref[pl.ngroups] = 0;
        return;
    }
    __syncthreads();
    for (uint64_t base = 0; base < pl.ngroups; base += kThreads) {
        const uint64_t i = base + threadIdx.x;
        const uint64_t c = i < pl.ngroups ? pl.group_pref[i] : 0;
        uint64_t x = c;
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {
            const uint64_t y = __shfl_up(x, s, kWaveSize);
            if (lane >= s)
                x += y;
        }
        if (lane == 63)
            wsum[w] = x;
        __syncthreads();
        uint64_t before = carry_s;
        for (int j = 0; j < w; j++)
            before += wsum[j];
        if (i < pl.ngroups)
            pl.group_pref[i] = before + x - c;
        __syncthreads();
        if (threadIdx.x == kThreads - 1)
            carry_s = before + x;
        __syncthreads();
    }
    if (threadIdx.x == 0)
        pl.group_pref[pl.ngroups] = carry_s;
}

// Test hook (RAMCRC_OPT_TEST_DIRTY_BINS): corrupt the histogram of a binning
// sequence between its count and scatter passes, as a stale histogram would.
__global__ void k_test_dirty_bins(BinTable* bt, uint32_t par, uint32_t bin, uint32_t add)
{
    if (bin < kNB)
        bt->ctr[par].hist[bin] += add;
}

// ramcrc_ctx_check: take the sticky bits (1, 2) atomically; the old word goes
// to status[1] for the host to read.
__global__ void k_status_take(uint32_t* status)
{
    status[1] = atomicAnd(status, ~(kStatusSticky | kStatusBins));
}

// ------------------------------------------------------------ host side
thread_local int t_last_hip = 0;

#define HIPCHK(expr)                              \
    do {                                          \
        hipError_t e_ = (expr);                   \
        if (e_ != hipSuccess) {                   \
            t_last_hip = int(e_);                 \
            return RAMCRC_EHIP;                   \
        }                                         \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

}  // namespace

struct ramcrc_ctx {
    int device = 0;
    int ncu = 256;       // CUs the persistent grids are sized for (ramcrc_ctx_set_cus)
    int ncu_all = 256;   // CUs of the device
    std::recursive_mutex mu;   // recursive: the host entry points hold it across their inner device calls
    uint32_t* partials = nullptr;
    uint64_t partials_cap = 0;
    uint64_t* plan_local = nullptr;
    uint64_t plan_cap = 0;
    uint64_t* group_pref = nullptr;
    uint64_t group_cap = 0;
    uint32_t* status = nullptr;
    // small-entry binning
    BinTable* bins = nullptr;
    uint32_t bin_par = 0;   // counter copy of the next binning sequence (BinCounters)
    int fail_after_count = 0;   // RAMCRC_OPT_TEST_FAIL_AFTER_COUNT: abandon N sequences
    uint32_t dirty_bins = 0;    // RAMCRC_OPT_TEST_DIRTY_BINS: bin << 16 | count, once
    int bin_straggler = 0;      // RAMCRC_OPT_TEST_BIN_STRAGGLER: next k_bin_one waits in vain
    int bin_resident[5] = {-1, -1, -1, -1, -1};   // k_bin_one<mode> workgroups per CU (occupancy query)
    u32x4* sdesc = nullptr;
    uint32_t* sidx = nullptr;
    uint32_t* sinit = nullptr;
    uint64_t sorted_cap = 0;
    // per-object checksums of ramcrc_assemble_objects_device when d_out is NULL
    uint32_t* obj_out = nullptr;
    uint64_t obj_out_cap = 0;
    // ramcrc_segments_certify_device scratch (uint32 words)
    uint32_t* cert_scratch = nullptr;
    uint64_t cert_scratch_cap = 0;
    // host staging for ramcrc_batch_host / ramcrc_stream_host
    uint8_t* h_stage = nullptr;
    uint64_t h_stage_cap = 0;
    uint8_t* d_stage = nullptr;
    uint64_t d_stage_cap = 0;
    hipStream_t copy_stream = nullptr;
    hipStream_t compute_stream = nullptr;
    // parallel segment walk scratch: per part results, per segment flags / bases
    void* walk_parts = nullptr;
    uint64_t walk_parts_cap = 0;
    uint32_t* walk_fallback = nullptr;
    uint64_t walk_fallback_cap = 0;
    uint64_t* walk_base = nullptr;
    uint64_t walk_base_cap = 0;
    void* walk_recs = nullptr;
    uint64_t walk_recs_cap = 0;
    void* walk_pool = nullptr;            // A's records past a part's first 64
    uint64_t walk_pool_cap = 0;
    uint32_t* walk_pool_owner = nullptr;
    uint64_t walk_pool_owner_cap = 0;
    uint32_t* walk_blocks = nullptr;
    uint64_t walk_blocks_cap = 0;
    unsigned long long* walk_pool_used = nullptr;
    uint64_t walk_pool_used_cap = 0;
    uint32_t* walk_sum = nullptr;   // ramcrc_replay_verify_device: the walk's replay_hard summary
    uint64_t walk_sum_cap = 0;
    bool serial_walk = false;   // RAMCRC_OPT_SERIAL_WALK
    uint32_t walk_pshift = 0;   // RAMCRC_OPT_WALK_PART_SHIFT; 0: kPartShift
    // benchmark timing of the scan kernels
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_used, ev_free;
};

namespace {

int grow_device(void** p, uint64_t* cap, uint64_t need_elems, size_t elem)
{
    if (*cap >= need_elems && *p)
        return RAMCRC_OK;
    uint64_t n = need_elems < 1024 ? 1024 : need_elems;
    if (*p) {
        HIPCHK(hipDeviceSynchronize());
        HIPCHK(hipFree(*p));
        *p = nullptr;
        *cap = 0;
    }
    if (hipMalloc(p, n * elem) != hipSuccess) {
        *p = nullptr;
        return RAMCRC_ENOMEM;
    }
    *cap = n;
    return RAMCRC_OK;
}

int reserve_locked(ramcrc_ctx* c, uint64_t max_chunks, uint64_t max_entries)
{
    int rc = grow_device(reinterpret_cast<void**>(&c->partials), &c->partials_cap, max_chunks,
                         sizeof(uint32_t));
    if (rc)
        return rc;
    rc = grow_device(reinterpret_cast<void**>(&c->plan_local), &c->plan_cap, max_entries,
                     sizeof(uint64_t));
    if (rc)
        return rc;
    const uint64_t ngroups = (max_entries + kThreads - 1) / kThreads + 1;
    return grow_device(reinterpret_cast<void**>(&c->group_pref), &c->group_cap, ngroups,
                       sizeof(uint64_t));
}

// Upper bound of chunks for a general batch whose buffers live in device
// memory: every full chunk holds 256 KiB of distinct device bytes, plus at
// most two partial chunks per entry.
// Upper bound of chunks for a general batch whose buffers live in device
// memory: every full chunk holds 256 KiB of distinct device bytes, plus at
// most two partial chunks per entry.  Overlapping or host-mapped buffers can
// exceed it; k_chunks then sets status bit 0 and writes nothing (see
// ramcrc_ctx_reserve).
uint64_t default_chunk_bound(uint64_t n)
{
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess)
        total_b = 288ull << 30;
    return total_b / kChunk + 2 * n + 16;
}

Plan make_plan(ramcrc_ctx* c, uint64_t n)
{
    Plan pl{};
    pl.local = c->plan_local;
    pl.group_pref = c->group_pref;
    pl.ngroups = (n + kThreads - 1) / kThreads;
    pl.partials = c->partials;
    pl.partials_cap = c->partials_cap;
    pl.status = c->status;
    pl.ticket = reinterpret_cast<unsigned long long*>(c->status + 2);   // 8-byte aligned
    return pl;
}

// Bracket the byte-scan kernel with events when benchmark timing is on.
// Timing-only events: no system-scope fence (cache writeback/invalidate)
// when they are reached, which otherwise puts a ~6 us bubble into the
// stream at every record (two per batch: 16 % of a 1M x 100 B step).  The
// elapsed time is read only after the stream is synchronised.
constexpr unsigned kTimerEventFlags = hipEventDisableSystemFence;

#ifndef RAMCRC_EXT_TIMING
#define RAMCRC_EXT_TIMING 1
#endif
// Times the one launch of its scope.  With RAMCRC_EXT_TIMING the two events
// ride in the kernel's own dispatch (hipExtLaunchKernelGGL start/stop
// events): no separate event packets, so no stream bubble before and after
// the kernel; otherwise they are recorded around it.
struct ScanTimer {
    ramcrc_ctx* c;
    hipStream_t s;
    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    ScanTimer(ramcrc_ctx* ctx, hipStream_t stream) : c(ctx), s(stream)
    {
        if (!c->timing)
            return;
        if (!c->ev_free.empty()) {
            ev = c->ev_free.back();
            c->ev_free.pop_back();
        } else if (hipEventCreateWithFlags(&ev.first, kTimerEventFlags) != hipSuccess ||
                   hipEventCreateWithFlags(&ev.second, kTimerEventFlags) != hipSuccess) {
            ev = {nullptr, nullptr};
            return;
        }
        if (!RAMCRC_EXT_TIMING)
            (void)hipEventRecord(ev.first, s);
    }
    template <typename F, typename... Args>
    void launch(F kernel, dim3 grid, dim3 block, Args... args)
    {
        if (RAMCRC_EXT_TIMING && ev.first)
            hipExtLaunchKernelGGL(kernel, grid, block, 0, s, ev.first, ev.second, 0, args...);
        else
            hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
    }
    ~ScanTimer()
    {
        if (!ev.first)
            return;
        if (!RAMCRC_EXT_TIMING)
            (void)hipEventRecord(ev.second, s);
        c->ev_used.push_back(ev);
    }
};

int reserve_sorted(ramcrc_ctx* c, uint64_t n)
{
    const uint64_t need = n + uint64_t(kG) * kNB;
    if (c->sorted_cap >= need)
        return RAMCRC_OK;
    uint64_t cap = c->sorted_cap;
    int rc = grow_device(reinterpret_cast<void**>(&c->sdesc), &cap, need, sizeof(u32x4));
    if (rc)
        return rc;
    cap = c->sorted_cap;
    rc = grow_device(reinterpret_cast<void**>(&c->sidx), &cap, need, sizeof(uint32_t));
    if (rc)
        return rc;
    cap = c->sorted_cap;
    rc = grow_device(reinterpret_cast<void**>(&c->sinit), &cap, need, sizeof(uint32_t));
    if (rc)
        return rc;
    c->sorted_cap = cap;
    return RAMCRC_OK;
}

// Small-entry path: bin by step count, scatter into bin order, scan.  A
// binning sequence is k_bin_count (bin_begin) ... k_bin_scatter, k_entries
// (bin_finish), or k_bin_one (bin_begin) ... k_entries for a batch of at most
// one tile per resident workgroup; the planned path runs its chunk kernels in
// between, so that they can exit at once when the count pass found no large
// buffer.
uint64_t bin_grid(const ramcrc_ctx* c, uint64_t n)
{
    // One tile per workgroup up to kBinWgsPerCu workgroups per CU: the binning
    // passes are latency-bound loads of 16 B per entry, and one 4-wave
    // workgroup per CU walking its tiles in turn kept one tile in flight.
    uint64_t grid = (n + uint64_t(kThreads) * kBinPer - 1) / (uint64_t(kThreads) * kBinPer);
    if (grid > uint64_t(c->ncu) * kBinWgsPerCu)
        grid = uint64_t(c->ncu) * kBinWgsPerCu;
    return grid;
}

template <int kMode>
int bin_begin(ramcrc_ctx* c, const BatchDesc& d, hipStream_t s, int skip_large, Sorted* so,
              const uint32_t* sum = nullptr)
{
    if (d.n >= (1ull << 32))
        return RAMCRC_EINVAL;   // sorted slots keep 32-bit entry indices
    int rc = reserve_sorted(c, d.n);
    if (rc)
        return rc;
    *so = Sorted{c->bins, c->sdesc, c->sidx, c->sinit, c->status, c->sorted_cap, c->bin_par, 0};
    // Every launch of this library checks its own error right after it (the
    // timed ScanTimer::launch calls included), so an error pending here was left
    // by a caller's own HIP call on this thread (torch's pointer probes leave
    // such errors behind).  It is recorded for ramcrc_last_hip_error and cleared,
    // not reported as this launch's failure.
    if (hipError_t stale = hipGetLastError(); stale != hipSuccess)
        t_last_hip = int(stale);
    // One launch when one tile per workgroup covers the batch and that grid
    // is resident at once (k_bin_one's arrival count needs every workgroup):
    // at most half the workgroups a CU holds, so that a second context's
    // k_bin_one on another stream fits beside it.  The dirty-histogram test
    // hook needs the two-launch path.
    const uint64_t tiles = (d.n + uint64_t(kThreads) * kBinPer - 1) / (uint64_t(kThreads) * kBinPer);
    int& resident = c->bin_resident[kMode];   // k_bin_one workgroups per CU (under c->mu)
    if (resident < 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_bin_one<kMode>, kThreads, 0) !=
            hipSuccess)
            nb = 0;
        resident = nb;
    }
    if (RAMCRC_BIN_ONE && !c->dirty_bins && !sum && tiles > 0 &&
        tiles <= uint64_t(c->ncu) * uint64_t(std::min(resident / 2, int(kBinWgsPerCu)))) {
        so->one = 1;
        hipLaunchKernelGGL(k_bin_one<kMode>, dim3(tiles), dim3(kThreads), 0, s, d, *so, skip_large,
                           c->bin_straggler ? 1u : 0u);
        c->bin_straggler = 0;
    } else {
        hipLaunchKernelGGL(k_bin_count<kMode>, dim3(bin_grid(c, d.n)), dim3(kThreads), 0, s, d,
                           *so, skip_large, sum);
    }
    HIPCHK(hipGetLastError());
    // enqueued: it zeroes the other copy, which the next sequence uses
    c->bin_par ^= 1u;
    return RAMCRC_OK;
}

template <int kMode>
int bin_finish(ramcrc_ctx* c, const BatchDesc& d, hipStream_t s, int skip_large, const Sorted& so)
{
    if (c->fail_after_count > 0) {   // test hook: a failure after k_bin_count
        c->fail_after_count--;
        return RAMCRC_EHIP;
    }
    if (c->dirty_bins) {   // test hook: a stale histogram
        hipLaunchKernelGGL(k_test_dirty_bins, dim3(1), dim3(1), 0, s, c->bins, so.par,
                           uint32_t(c->dirty_bins >> 16), uint32_t(c->dirty_bins & 0xFFFF));
        c->dirty_bins = 0;
        HIPCHK(hipGetLastError());
    }
    if (!so.one || RAMCRC_BIN_RESCUE) {
        // after k_bin_one: the guarded scatter (exits at once unless k_bin_one aborted)
        hipLaunchKernelGGL(k_bin_scatter<kMode>, dim3(bin_grid(c, d.n)), dim3(kThreads), 0, s, d,
                           so, skip_large, int(so.one));
        HIPCHK(hipGetLastError());
    }
    {
        ScanTimer t(c, s);
        t.launch(k_entries, dim3(c->ncu), dim3(kEntWaves * kWaveSize), d, so);
    }
    HIPCHK(hipGetLastError());
    return RAMCRC_OK;
}

template <int kMode>
int launch_binned(ramcrc_ctx* c, const BatchDesc& d, hipStream_t s, int skip_large)
{
    Sorted so;
    int rc = bin_begin<kMode>(c, d, s, skip_large, &so);
    if (rc)
        return rc;
    return bin_finish<kMode>(c, d, s, skip_large, so);
}

template <int kMode>
int launch_planned(ramcrc_ctx* c, const BatchDesc& d, hipStream_t s, const uint32_t** nother = nullptr,
                   const uint32_t* sum = nullptr)
{
    Sorted so;
    int rc = bin_begin<kMode>(c, d, s, 1, &so, sum);
    if (rc)
        return rc;
    if (nother)
        *nother = &so.bt->ctr[so.par].nother;
    Plan pl = make_plan(c, d.n);
    pl.nlarge = &so.bt->ctr[so.par].nlarge;
    const uint64_t gcap = uint64_t(4) * c->ncu;
    hipLaunchKernelGGL(k_plan_count<kMode>, dim3(uint32_t(pl.ngroups < gcap ? pl.ngroups : gcap)),
                       dim3(kThreads), 0, s, d, pl);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_plan_scan, dim3(1), dim3(kThreads), 0, s, pl);
    HIPCHK(hipGetLastError());
    {
        ScanTimer t(c, s);
        t.launch(k_chunks<kMode>, dim3(c->ncu), dim3(kThreads), d, pl, uint64_t(0));
    }
    HIPCHK(hipGetLastError());
    const uint64_t cw = (d.n + 255) / 256, ccap = uint64_t(16) * c->ncu;
    if (d.n > kWideCombineMin)
        hipLaunchKernelGGL((k_combine<kMode, true>), dim3(uint32_t(cw < ccap ? cw : ccap)), dim3(256), 0, s,
                           d, pl, uint64_t(0));
    else
        hipLaunchKernelGGL((k_combine<kMode, false>), dim3((d.n + 3) / 4), dim3(256), 0, s, d, pl,
                           uint64_t(0));
    HIPCHK(hipGetLastError());
    return bin_finish<kMode>(c, d, s, 1, so);
}

// ------------------------------------------------------------ segment walk
// Segment::checkMetadataIntegrity (src/Segment.cc:758-800) on the device: one
// wavefront per segment.  The walk is a pointer chase through length-prefixed
// entries (|EntryHeader|length 1-4 B|payload|, src/Segment.h:99-112): latency,
// not bandwidth, bounds it, so everything is arranged to keep one hop short.
//  * The chase reads only LDS.  The segment is staged through 16 KiB windows
//    (coalesced 1 KiB wave loads); while one window is walked the next one is
//    already in flight in registers.  Consecutive windows overlap by 16 bytes,
//    so an entry header and its length bytes (<= 5 B, read as 8) never
//    straddle two windows.  An entry that jumps past the prefetched window
//    reloads at its header: payload bytes of large entries are never fetched.
//  * The metadata checksum is off the chase.  A hop only parks its entry in
//    one lane; every 64 hops the wave checksums the 64 parked header+length
//    byte strings in parallel -- lane j: raw(0, bytes_j) moved past the bytes
//    of the entries after it (x^(8d) from a table, one GF(2) multiply) --
//    XORs them across the wave and folds the batch into the running state:
//    raw(s, A||B) = X^|B|(raw(s, A)) ^ raw(0, B).
// Complete entries are appended to the record table 64 at a time (one atomic
// per 64 records).
constexpr uint32_t kWalkWin = 16384;                          // bytes per window
constexpr uint32_t kWalkStep = kWalkWin - 16;                 // window advance
constexpr int kWalkPer = int(kWalkWin / 16 / kWaveSize);      // 16-byte units per lane
constexpr uint32_t kWalkMeta = 5 * kWaveSize;                 // metadata bytes per batch, max

struct WalkDesc {
    const uint8_t* base;
    uint64_t stride;
    uint64_t capacity;
    uint64_t nseg;
    const ramcrc_seg_cert* certs;
    ramcrc_seg_status* status;
    u32x4* entries;
    uint64_t cap;
    unsigned long long* n_entries;
    const uint32_t* only;   // nullable: walk only the segments with only[seg] != 0
    uint64_t* seg_base;     // nullable: per segment, the first slot of its records
    uint32_t* sum;          // nullable: ORed with the written records' replay_hard bits
};

// CRC32C update by the m (1..4) bytes in the low end of v; t[j][b] = X^(j+1)(b).
__device__ __forceinline__ uint32_t crc_small(const uint32_t* t, uint32_t c, uint32_t v, uint32_t m)
{
    const uint32_t x = c ^ v;
    uint32_t r = m >= 4 ? 0u : (c >> (8 * m));
#pragma unroll
    for (uint32_t k = 0; k < 4; k++)
        if (k < m)
            r ^= t[(m - 1 - k) * 256 + ((x >> (8 * k)) & 0xFF)];
    return r;
}

// Issue the loads of window [wbase, wbase + kWalkWin) of a segment (lane l:
// units l + 64 k) as buffer loads whose descriptor ends at the segment's
// capacity: units past it read as zero with no branch, as Segment::copyOut
// leaves bytes past the segment's end.
__device__ __forceinline__ void walk_issue(u32x4 (&r)[kWalkPer], uint64_t sb, uint64_t wbase,
                                           uint64_t capacity, int lane)
{
    const uint64_t base = rfl64(sb + wbase);
    const uint32_t nrec =
        __builtin_amdgcn_readfirstlane(uint32_t(wbase < capacity ? capacity - wbase : 0));
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), (short)0, int(nrec),
                                          0x00020000);
#pragma unroll
    for (int k = 0; k < kWalkPer; k++)
        r[k] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, uint32_t(lane + kWaveSize * k) * 16, 0, 0);
}

__device__ __forceinline__ void walk_store(uint8_t* win, const u32x4 (&r)[kWalkPer], int lane)
{
#pragma unroll
    for (int k = 0; k < kWalkPer; k++)
        *reinterpret_cast<u32x4*>(win + (lane + kWaveSize * k) * 16) = r[k];
}

__global__ __launch_bounds__(kWaveSize) void k_seg_walk(WalkDesc w)
{
    __shared__ __attribute__((aligned(16))) uint8_t win[2][kWalkWin];
    __shared__ __attribute__((aligned(16))) uint32_t tab[4 * 256];
    __shared__ uint32_t xm[kWalkMeta + 1];
    fill_plain(reinterpret_cast<uint8_t*>(tab), 0, &g_tab.pos[1 + kTinyRow0][0], 4 * 256);
    for (uint32_t t = threadIdx.x; t <= kWalkMeta; t += blockDim.x)
        xm[t] = g_tab.xmeta[t];
    __syncthreads();
    const int lane = threadIdx.x;
    uint32_t hard = 0;   // replay_hard bits of the records this wave wrote (w.sum)

    for (uint64_t seg = blockIdx.x; seg < w.nseg; seg += gridDim.x) {
        if (w.only && !w.only[seg])
            continue;   // walked by the parallel walk (uniform per workgroup)
        const uint64_t sb = reinterpret_cast<uint64_t>(w.base) + seg * w.stride;
        const ramcrc_seg_cert cert = w.certs[seg];
        // Two passes: the first counts the records, one atomic allocates them,
        // the second writes them -- so every segment's records are contiguous
        // and in offset order (the parallel walk's are too).
        unsigned long long rbase = 0, rdone = 0, rtotal = 0;
        for (int pass = 0; pass < 2; pass++) {
        uint32_t pos = 0, crc = 0xFFFFFFFFu, count = 0, flags = 0;
        // Parked entries: lane j holds entry j of the current batch of 64 --
        // its offset and the 4 bytes from its header on.  Its length is
        // recovered at the flush from the offset of the entry after it
        // (len = next - pos - 1 - lengthBytes, mod 2^32), so a hop parks two
        // values, not four.
        uint32_t rpos = 0, rq = 0;
        uint32_t ns = 0;

        // Fold the parked entries' header + length bytes into crc and append
        // the first nrec of them to the record table.
        // tail: the offset after the last parked entry (its `next`).
        auto flush = [&](uint32_t nrec, uint32_t tail) {
            const uint32_t pn = __shfl_down(rpos, 1, kWaveSize);
            const uint32_t nxt = lane + 1 == int(ns) ? tail : pn;
            const uint32_t hdr = rq & 0xFF, lb = (hdr >> 6) + 1;
            const uint32_t rlen = nxt - rpos - 1 - lb;
            // a payload past 2^32 (carry out of the reference's uint32_t
            // offset) is unreadable: kRecOverlong
            const uint32_t rinfo = hdr | (rlen > ~(rpos + 1 + lb) ? kRecOverlong : 0u);
            uint32_t m = 0, r = 0;
            if (lane < int(ns)) {
                m = 1 + lb;
                r = crc_small(tab, 0u, hdr | (rlen << 8), m < 4 ? m : 4);
                if (m == 5)
                    r = crc_small(tab, r, rlen >> 24, 1);
            }
            uint32_t incl = m;   // inclusive prefix of the byte counts
#pragma unroll
            for (int s = 1; s < kWaveSize; s <<= 1) {
                const uint32_t y = __shfl_up(incl, s, kWaveSize);
                if (lane >= s)
                    incl += y;
            }
            const uint32_t total = __shfl(incl, kWaveSize - 1, kWaveSize);
            uint32_t c = lane < int(ns) ? mulmod_horner(r, xm[total - incl]) : 0u;
#pragma unroll
            for (int s = 1; s < kWaveSize; s <<= 1)
                c ^= __shfl_xor(c, s, kWaveSize);
            crc = mulmod_horner(crc, xm[total]) ^ c;
            if (nrec && pass == 0) {
                rtotal += nrec;
            } else if (nrec) {
                const unsigned long long b = rbase + rdone;
                if (lane < int(nrec) && b + lane < w.cap) {
                    w.entries[b + lane] = u32x4{uint32_t(seg), rpos, rlen, rinfo};
                    hard |= w.sum ? replay_hard(rpos, rlen, rinfo) : 0u;
                }
                rdone += nrec;
            }
            ns = 0;
        };

        // window state: win[cur] holds [wb, wb + kWalkWin); pf is loading
        // [wb + kWalkStep, ...)
        int cur = 0;
        uint32_t wb = 0;
        u32x4 pf[kWalkPer];
        __syncthreads();   // the previous segment's LDS reads are done
        walk_issue(pf, sb, 0, w.capacity, lane);
        walk_store(win[0], pf, lane);
        walk_issue(pf, sb, kWalkStep, w.capacity, lane);
        __syncthreads();

        // The chase: every value below is wave-uniform (scalar registers).
        // The outer loop moves windows, flushes full batches and stops the
        // walk; the inner loop is the hop itself -- one LDS read and a few
        // scalar operations -- and runs while the entry header stays inside
        // the window, the batch has room and the cycle bound is not reached.
        const uint32_t cap32 = uint32_t(w.capacity);
        const uint32_t limit = cert.segment_length < cap32 ? cert.segment_length : cap32;
        uint32_t steps = 0, tail = 0;
        bool overrun = false;
        while (pos < limit) {
            // deterministic walk below the capacity: more steps than bytes means
            // a repeated position, i.e. the reference's loop never ends
            if (steps >= cap32) {
                flags |= RAMCRC_SEG_CYCLE;
                break;
            }
            if (pos - wb > kWalkWin - 8) {   // (a position below wb wraps: reload)
                const uint64_t nb = uint64_t(wb) + kWalkStep;
                if (uint64_t(pos) >= nb && uint64_t(pos) - nb <= kWalkWin - 8) {
                    walk_store(win[cur ^ 1], pf, lane);   // the prefetched window
                    cur ^= 1;
                    wb = uint32_t(nb);
                } else {                                    // a jump: reload at the header
                    wb = pos & ~15u;
                    walk_issue(pf, sb, wb, w.capacity, lane);
                    walk_store(win[cur], pf, lane);
                }
                __syncthreads();
                walk_issue(pf, sb, uint64_t(wb) + kWalkStep, w.capacity, lane);
            }
            if (ns == uint32_t(kWaveSize))
                flush(ns, pos);
            const uint32_t* w32 = reinterpret_cast<const uint32_t*>(win[cur]);
            // hop while pos - wb <= span (header + 7 bytes inside the window, pos
            // below the limit) and the batch and the cycle bound have room
            const uint64_t wend = uint64_t(wb) + (kWalkWin - 8);
            const uint32_t last = limit - 1 < wend ? limit - 1 : uint32_t(wend);
            const uint32_t span = last - wb;
            // the batch and the cycle bound: at most nsmax - ns hops
            uint32_t nsmax = uint32_t(kWaveSize);
            if (cap32 - steps < nsmax - ns)
                nsmax = ns + (cap32 - steps);
            const uint32_t ns0 = ns;
            uint32_t next;
            for (;;) {
                const uint32_t o = pos - wb;
                const uint32_t d0 = __builtin_amdgcn_readfirstlane(w32[o >> 2]);
                const uint32_t d1 = __builtin_amdgcn_readfirstlane(w32[(o >> 2) + 1]);
                const uint64_t q = ((uint64_t(d1) << 32) | d0) >> (8 * (o & 3));
                const uint32_t t = (uint32_t(q) >> 6) & 3;   // getLengthBytes() - 1
                // len = the t + 1 bytes after the header: one s_bfe_u64, field
                // {offset 8, width 8 t + 8}
                uint32_t fld;
                uint64_t len64;
                asm("s_lshl_b32 %0, %2, 19\n\ts_add_u32 %0, %0, 0x80008\n\ts_bfe_u64 %1, %3, %0"
                    : "=&s"(fld), "=s"(len64) : "s"(t), "s"(q) : "scc");
                // uint32_t arithmetic, as the reference (a wrap is legal)
                next = pos + t + 2 + uint32_t(len64);
                const bool mine = lane == int(ns);   // park: one compare, two selects
                rpos = mine ? pos : rpos;
                rq = mine ? uint32_t(q) : rq;
                ns++;
                // the next header leaves the window or the limit (this also
                // covers next > capacity and a wrapped next)
                if (next - wb > span)
                    break;
                if (ns == nsmax)   // the batch is full, or the cycle bound
                    break;
                pos = next;
            }
            steps += ns - ns0;
            tail = next;
            if (next > cap32) {
                // the last hop's header and length were checksummed; that
                // entry is not a record
                flags |= RAMCRC_SEG_PAST_CAPACITY;
                overrun = true;
                break;
            }
            pos = next;
        }
        count = steps - (overrun ? 1u : 0u);
        if (ns)
            flush(overrun ? ns - 1 : ns, tail);
        if (pass == 0) {
            unsigned long long b = 0;
            if (lane == 0 && rtotal)
                b = atomicAdd(w.n_entries, rtotal);
            rbase = __shfl(b, 0, kWaveSize);
            if (lane == 0 && w.seg_base)
                w.seg_base[seg] = rbase;
            if (rtotal == 0)
                pass = 1;   // nothing to write: the second pass is this one
        }
        if (rbase + rtotal > w.cap)
            flags |= RAMCRC_SEG_TABLE_FULL;
        if (pass == 0)
            continue;
        const uint32_t fin = ~crc_small(tab, crc, cert.segment_length, 4);
        if (!(flags & (RAMCRC_SEG_PAST_CAPACITY | RAMCRC_SEG_CYCLE))) {
            if (pos > cert.segment_length)
                flags |= RAMCRC_SEG_PAST_LENGTH;
            else if (fin != cert.checksum)
                flags |= RAMCRC_SEG_BAD_CHECKSUM;
            else if (!(flags & RAMCRC_SEG_TABLE_FULL))
                flags |= RAMCRC_SEG_OK;   // records dropped: not verified, never OK
        }
        if (lane == 0) {
            ramcrc_seg_status st;
            st.flags = flags;
            st.checksum = fin;
            st.entries = count;
            st.bad_objects = 0;
            w.status[seg] = st;
        }
        }   // pass
    }
    {
        const uint32_t hw = (__ballot(hard & 1u) ? 1u : 0u) | (__ballot(hard & 2u) ? 2u : 0u) |
                           (__ballot(hard & 4u) ? 4u : 0u);
        if (w.sum && hw && lane == 0)
            atomicOr(w.sum, hw);
    }
}

// ------------------------------------------------- parallel segment walk
// The walk of Segment::checkMetadataIntegrity (src/Segment.cc:758-800) is a
// chain: entry i+1 starts where entry i's length says.  One wave chasing it
// through a whole 8 MiB segment (k_seg_walk) is latency-bound at ~160 ns a
// hop, and a 512-segment batch is only 512 chains.  Here every segment is cut
// into 64 KiB parts and the chain is found in every part at once:
//
//  A0 k_walk_sync   per part k >= 1 (one wave): the first offset in the part
//                   from which kSyncHops consecutive hops each land on a
//                   header of a valid LogEntryType (src/LogEntryTypes.h:29-68,
//                   type < 12) inside the segment -- a guess of where the
//                   chain enters the part.  Candidates are tested 512 at a
//                   time, all hops of all live candidates issued together.
//  A  k_walk_parts  per part (one lane): the reference's walk from the guess
//                   (part 0: from offset 0) until it leaves the part or
//                   reaches min(certificate length, capacity): entries,
//                   the raw CRC of their header + length bytes, exit offset.
//  B  k_walk_fix    per segment (one wave): the true chain, part by part in
//                   order.  A part is accepted when the chain arrives exactly
//                   at its guess (the walk is deterministic, so its result is
//                   then the reference's); a part the chain skips is ignored;
//                   otherwise the part is walked again from the true offset.
//                   The accepted parts' metadata CRCs are combined with
//                   raw(0, A||B) = X^|B|(raw(0, A)) ^ raw(0, B), the status is
//                   written and the segment's records are allocated.
//  C  k_walk_emit   per accepted part (one lane): walk again, writing the
//                   records in order at their final slots.
// A segment whose chain wraps the reference's uint32_t offset (it would then
// walk backwards, or forever) or needs too many re-walks is handed to the
// serial walker k_seg_walk, which implements those semantics.  The result of
// every segment -- flags, checksum, entry count, records -- equals the serial
// walk's (tests/test_gpu_segments.py runs both against the oracle).
#ifndef RAMCRC_PART_SHIFT
#define RAMCRC_PART_SHIFT 16
#endif
constexpr uint32_t kPartShift = RAMCRC_PART_SHIFT;  // default parts: 64 KiB
constexpr uint32_t kPartShiftMin = 13;               // smallest part (RAMCRC_OPT_WALK_PART_SHIFT)
constexpr uint32_t kNoStart = 0xFFFFFFFFu;
#ifndef RAMCRC_SYNC_HOPS
#define RAMCRC_SYNC_HOPS 6
#endif
#ifndef RAMCRC_SYNC_PER
#define RAMCRC_SYNC_PER 8
#endif
#ifndef RAMCRC_SYNC_STAGE_KIB
#define RAMCRC_SYNC_STAGE_KIB 7
#endif
constexpr int kSyncHops = RAMCRC_SYNC_HOPS;         // hops a guess must survive
constexpr int kSyncPer = RAMCRC_SYNC_PER;           // candidates per lane per round
constexpr uint32_t kSyncRound = kSyncPer * kWaveSize;   // 512 candidates
static_assert(kSyncPer % 4 == 0 && kSyncPer <= 32, "candidates per lane: whole dwords");
constexpr uint32_t kSyncSpan = 16384;               // candidate bytes searched per part
constexpr uint32_t kMeetMax = 4;                    // B's fast path: meets within 4 records
constexpr uint32_t kMeetHops = 3;                   // ... after at most 3 entries walked
constexpr uint32_t kRewalkBudget = 1u << 15;        // hops B may re-walk before falling back
// part flags
constexpr uint32_t kPartWalked = 1u, kPartWrap = 2u, kPartOverrun = 4u, kPartEmit = 8u;
constexpr uint32_t kPartSpill = 16u;   // A: more records than its scratch holds
constexpr uint32_t kPartChase = 32u;   // B: walked again; C walks it once more
constexpr uint32_t kPartHuge = 64u;    // A: an entry of 16 MiB or more (records hold 24-bit lengths)
constexpr uint32_t kMaxBlocks = 15;    // pool blocks per part: records 64 .. 1023 of A's walk
constexpr uint32_t kPartRec = 64;      // records A keeps per part (C copies them)

struct PartRes {
    uint32_t start;    // A0: guess (kNoStart: none); B: the true start of an emitting part
    uint32_t exit;     // A: offset where the part's walk stopped
    uint32_t count;    // A: entries (records)
    uint32_t nmeta;    // A: header + length bytes checksummed
    uint32_t raw;      // A: raw(0, those bytes)
    uint32_t flags;    // kPart*
    uint64_t rec;      // B: first record slot of the part
    uint32_t pre;      // B: entries walked before meeting the guessed chain (C walks them)
    uint32_t cut;      // B: junk entries at the head of the guessed chain (C skips them)
};

struct PWalk {
    const uint8_t* base;
    uint64_t stride;
    uint32_t capacity;
    uint32_t nparts;
    uint64_t nseg;
    const ramcrc_seg_cert* certs;
    ramcrc_seg_status* status;
    u32x4* entries;
    uint64_t cap;
    unsigned long long* n_entries;
    PartRes* parts;
    uint32_t* fallback;   // per segment: nonzero = walked by k_seg_walk
    uint64_t* seg_base;   // per segment: first record slot (B)
    uint2* recs;          // per part: kPartRec records of A's walk {offset, length << 8 | header}
    uint32_t pshift;      // log2 part bytes of this launch (from *geo when geo is set)
    const uint32_t* geo;  // the part shift k_walk_probe chose for this batch
    // A's records past the first kPartRec of a part: blocks of kPartRec from a
    // pool (one atomic per block), up to kMaxBlocks per part
    uint2* pool;
    uint32_t* pool_owner;            // per pool block: part * 16 + block number (1 ..)
    uint32_t* blocks;                // per part: kMaxBlocks pool block indices
    unsigned long long* pool_used;   // blocks taken (zeroed per launch)
    uint64_t pool_cap;               // pool blocks
    uint32_t* sum;                   // nullable: as WalkDesc::sum
};

typedef const __attribute__((address_space(1))) uint32_t gu32;

// The bytes from pos on (at least 5: the header and up to 4 length bytes), as
// Segment::copyOut would give them: bytes at or past the capacity read 0.
// Two aligned dword loads (pos < capacity, capacity % 16 == 0).
__device__ __forceinline__ uint64_t seg_peek(uint64_t seg, uint32_t pos, uint32_t capacity)
{
    const uint32_t a = pos & ~3u;
    const bool two = a + 4 < capacity;
    const uint32_t w0 = *reinterpret_cast<gu32*>(seg + a);
    uint32_t w1 = *reinterpret_cast<gu32*>(seg + (two ? a + 4 : a));
    w1 = two ? w1 : 0u;
    return ((uint64_t(w1) << 32) | w0) >> (8 * (pos & 3));
}

// raw CRC update by an entry's header + length bytes (2..5 of them, from q).
__device__ __forceinline__ uint32_t meta_update(const uint32_t* tab, uint32_t c, uint64_t q,
                                                uint32_t mbytes)
{
    c = crc_small(tab, c, uint32_t(q), mbytes < 4 ? mbytes : 4);
    if (mbytes == 5)
        c = crc_small(tab, c, uint32_t(q >> 32), 1);
    return c;
}

// x^(8d) for any 32-bit d.
__device__ __forceinline__ uint32_t xpow8_dev(uint32_t d)
{
    uint32_t r = ramcrc::kOne;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t b = (d >> (8 * j)) & 0xFF;
        if (b)
            r = r == ramcrc::kOne ? g_tab.xbyte[j][b] : mulmod_dev(r, g_tab.xbyte[j][b]);
    }
    return r;
}

__device__ __forceinline__ uint32_t walk_limit(const PWalk& w, uint64_t seg)
{
    const uint32_t len = w.certs[seg].segment_length;
    return len < w.capacity ? len : w.capacity;
}

// The part geometry of this batch: every walk kernel takes it from the word
// k_walk_probe wrote (the host sizes its grids and scratch for the smallest
// part the probe may choose).
__device__ __forceinline__ PWalk walk_geo(PWalk w)
{
    if (w.geo) {
        w.pshift = *w.geo;
        w.nparts = uint32_t((uint64_t(w.capacity) + (1ull << w.pshift) - 1) >> w.pshift);
    }
    return w;
}

// Part size per batch from the entry density.  A part should hold about 64
// entries: much fewer and the sync search (which stages the first 7 KiB of
// a part and chases 6 hops) mostly finds no header or chases far through
// global memory, and k_walk_fix re-walks the part; much more and the one-lane
// part walks get long (profiles/r04/parts: 8 KiB values 1.90 TB/s with 64 KiB
// parts, 3.85 with 512 KiB; 64 B values 1.25 with 64 KiB, 0.78 with 128 KiB).
// One wave: lane l walks the first kProbeHops entries of one of up to 64
// segments spread over the batch; the mean entry size m gives the shift
// round(log2(64 m)) within [kPartShift, kPartShiftMax].  A forced shift
// (RAMCRC_OPT_WALK_PART_SHIFT) is written as is.
constexpr uint32_t kPartShiftMax = 20;
constexpr int kProbeHops = 8;

// The replay summary word (PWalk::sum, replay_hard bits) only gains bits
// within a batch.  A wave reads it (coherently) and ORs only the bits it
// would add: with 1 KiB objects every wave has hard records, and 32K
// same-address atomics cost 175 us per batch when k_walk_copy made them
// (profiles/r05/replayfix).  No word: everything counts as seen.
__device__ __forceinline__ uint32_t walk_sum_seen(const uint32_t* sum)
{
    return sum ? __hip_atomic_load(sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kHardAll;
}

__global__ __launch_bounds__(kWaveSize) void k_walk_probe(PWalk w, uint32_t forced, uint32_t* geo)
{
    const int lane = threadIdx.x;
    const uint64_t ns = w.nseg < uint64_t(kWaveSize) ? w.nseg : uint64_t(kWaveSize);
    uint64_t dist = 0, hops = 0;
    if (!forced && uint64_t(lane) < ns) {
        const uint64_t seg = uint64_t(lane) * w.nseg / ns;
        const uint64_t sb = reinterpret_cast<uint64_t>(w.base) + seg * w.stride;
        const uint32_t limit = walk_limit(w, seg);
        uint32_t pos = 0;
        for (int hh = 0; hh < kProbeHops && pos < limit; hh++) {
            const uint64_t q = seg_peek(sb, pos, w.capacity);
            const Hop h = hop_of(q, pos);
            if (!plausible(q, h, w.capacity) || h.next > limit)
                break;
            dist += h.next - pos;
            hops++;
            pos = uint32_t(h.next);
        }
    }
#pragma unroll
    for (int o = 1; o < kWaveSize; o <<= 1) {
        dist += __shfl_xor(dist, o, kWaveSize);
        hops += __shfl_xor(hops, o, kWaveSize);
    }
    if (lane == 0) {
        // the batch's counters, zeroed here rather than by three memsets
        // ahead of this launch (each a few microseconds on the stream)
        *w.n_entries = 0;
        w.pool_used[0] = 0;
        if (w.sum)
            *w.sum = 0;
        uint32_t shift = kPartShift;
        if (forced) {
            shift = forced;
        } else if (hops) {
            const uint64_t t = 64 * (dist / hops);   // bytes of 64 entries
            uint32_t l = 63 - uint32_t(__builtin_clzll(t | 1));   // floor(log2 t)
            // round to nearest in log scale: up when t >= 2^l * sqrt(2)
            if (t * t >= (1ull << (2 * l)) * 2)
                l++;
            shift = l < kPartShift ? kPartShift : (l > kPartShiftMax ? kPartShiftMax : l);
        }
        *geo = shift;
    }
}

// A0: one wave per part k >= 1.  The part's first kSyncWin bytes are staged
// in LDS, so most candidate hops (the true chain's included, for entries of
// a few KiB) read LDS instead of waiting on global memory.
constexpr uint32_t kSyncStage = RAMCRC_SYNC_STAGE_KIB * 1024;   // staged bytes per wave
constexpr uint32_t kSyncWin = kSyncStage - 16;       // candidates / hops read from LDS below this
constexpr int kSyncWaves = 4;                        // waves per workgroup
#ifndef RAMCRC_SYNC_TYPES
#define RAMCRC_SYNC_TYPES 1   // k_walk_sync: survivors whose hops are all objects / tombstones first
#endif
constexpr uint64_t kSyncJunkKey = 1ull << 63;        // search key bit: a survivor of the other class

// Wave minimum through DPP (quad swaps, half-row and row mirrors, row
// broadcasts): the result is valid in lane 63 and returned uniform.
__device__ __forceinline__ uint32_t wave_min(uint32_t v)
{
    v = min(v, uint32_t(__builtin_amdgcn_update_dpp(-1, int(v), 0xB1, 0xF, 0xF, false)));   // quad_perm 1,0,3,2
    v = min(v, uint32_t(__builtin_amdgcn_update_dpp(-1, int(v), 0x4E, 0xF, 0xF, false)));   // quad_perm 2,3,0,1
    v = min(v, uint32_t(__builtin_amdgcn_update_dpp(-1, int(v), 0x141, 0xF, 0xF, false)));  // row_half_mirror
    v = min(v, uint32_t(__builtin_amdgcn_update_dpp(-1, int(v), 0x140, 0xF, 0xF, false)));  // row_mirror
    v = min(v, uint32_t(__builtin_amdgcn_update_dpp(-1, int(v), 0x142, 0xA, 0xF, false)));  // row_bcast:15
    v = min(v, uint32_t(__builtin_amdgcn_update_dpp(-1, int(v), 0x143, 0xC, 0xF, false)));  // row_bcast:31
    return uint32_t(__builtin_amdgcn_readlane(int(v), 63));
}

// One part of the sync search.  The certificate length is loaded with the
// stage and used a search later, so its latency is not exposed either.
struct SyncPart {
    uint64_t sb;       // segment base address
    uint32_t k;        // part number in the segment
    uint32_t B;        // first byte of the part
    uint32_t seglen;   // certificate segment length
};

__device__ __forceinline__ SyncPart sync_part(const PWalk& w, uint64_t i)
{
    SyncPart P;
    const uint64_t seg = i / w.nparts;
    P.k = uint32_t(i - seg * w.nparts);
    P.B = P.k << w.pshift;
    P.seglen = w.certs[seg].segment_length;
    P.sb = reinterpret_cast<uint64_t>(w.base) + seg * w.stride;
    return P;
}

#ifndef RAMCRC_SYNC_PF
#define RAMCRC_SYNC_PF 1   // stage loads of a wave's next part issued before this part's search
#endif
#ifndef RAMCRC_SYNC_STRICT
#define RAMCRC_SYNC_STRICT 1   // candidate hops past the walk limit or of empty entries end the candidate
#endif
#ifndef RAMCRC_SYNC_EARLY
#define RAMCRC_SYNC_EARLY 1   // stop at the end of the first round holding a survivor
#endif

__global__ __launch_bounds__(kSyncWaves * kWaveSize) void k_walk_sync(PWalk w0)
{
    const PWalk w = walk_geo(w0);
    __shared__ __attribute__((aligned(16))) uint8_t wins[kSyncWaves][kSyncStage];
    __shared__ uint16_t lists[kSyncWaves][kSyncRound];   // a round's first-hop survivors
    constexpr uint32_t kSU = kSyncStage / 1024;
    const int lane = threadIdx.x & (kWaveSize - 1);
    const int wv = threadIdx.x / kWaveSize;
    uint8_t* win = wins[wv];
    uint16_t* list = lists[wv];
    const uint64_t nwave = uint64_t(gridDim.x) * kSyncWaves;
    const uint64_t total = w.nseg * w.nparts;
    // stage [B, B + kSyncStage): bytes at or past the capacity are 0.  All
    // loads are issued before the first store (one memory latency, not one
    // per 1 KiB); with RAMCRC_SYNC_PF the loads of the wave's next part are
    // in flight while this part is searched.  The LDS is wave-private.
    u32x4 v[kSU];
    auto stage_load = [&](const SyncPart& P) {
#pragma unroll
        for (uint32_t u = 0; u < kSU; u++) {
            const uint64_t a = uint64_t(P.B) + u * 1024 + uint32_t(lane) * 16;
            v[u] = a + 16 <= w.capacity ? load16(P.sb + a) : u32x4{0u, 0u, 0u, 0u};
        }
    };
    uint64_t i = uint64_t(blockIdx.x) * kSyncWaves + wv;
    SyncPart nxt{};
    if (RAMCRC_SYNC_PF && i < total) {
        nxt = sync_part(w, i);
        if (nxt.k != 0)
            stage_load(nxt);
    }
    for (; i < total; i += nwave) {
        const SyncPart P = RAMCRC_SYNC_PF ? nxt : sync_part(w, i);
        const uint32_t B = P.B;
        const uint64_t sb = P.sb;
        const uint32_t limit = P.seglen < w.capacity ? P.seglen : w.capacity;   // walk_limit
        uint64_t end64 = uint64_t(B) + kSyncSpan;
        end64 = end64 < uint64_t(B) + (1ull << w.pshift) ? end64 : uint64_t(B) + (1ull << w.pshift);
        end64 = end64 < w.capacity ? end64 : w.capacity;
        const uint32_t end = uint32_t(end64 < limit ? end64 : limit);
        const bool search_part = P.k != 0 && end > B;   // part 0 starts at offset 0
        if (search_part) {
            if (!RAMCRC_SYNC_PF)
                stage_load(P);
#pragma unroll
            for (uint32_t u = 0; u < kSU; u++)
                *reinterpret_cast<u32x4*>(win + u * 1024 + uint32_t(lane) * 16) = v[u];
        }
        if (RAMCRC_SYNC_PF && i + nwave < total) {
            nxt = sync_part(w, i + nwave);
            if (nxt.k != 0)   // (also for a part past the segment length: not known yet)
                stage_load(nxt);
        }
        if (!search_part) {
            if (P.k != 0 && lane == 0)
                w.parts[i].start = kNoStart;
            continue;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // stores land before the reads
        auto peek_lds = [&](uint32_t p) -> uint64_t {   // the bytes from p (B <= p, p + 8 <= B + kSyncStage)
            const uint32_t o = p - B;
            const uint32_t* w32 = reinterpret_cast<const uint32_t*>(win + (o & ~3u));
            return ((uint64_t(w32[1]) << 32) | w32[0]) >> (8 * (o & 3));
        };
        auto peek = [&](uint32_t p) -> uint64_t {   // the bytes from p (>= B)
            return p - B + 8 <= kSyncStage ? peek_lds(p) : seg_peek(sb, p, w.capacity);
        };
        // Candidates in rounds of 512 from B.  A candidate survives when its
        // chain makes kSyncHops plausible hops (or reaches the limit).  A
        // junk header whose length happens to land on a real header survives
        // too, and then skips the real entries it jumps over.  The real first
        // entry h is two real entries ahead after two hops, while a junk chain
        // that lands on the real chain only after skipping some of it is
        // further ahead: the survivor whose second hop lands nearest is kept
        // (ties: the lower candidate; a junk chain that wins has met the real
        // chain within two entries, which k_walk_fix resolves in as many
        // hops).  The scan ends with the first round that holds a survivor
        // (RAMCRC_SYNC_EARLY; a junk survivor from an earlier position is then
        // met by k_walk_fix or its part walked again), or else at the nearest
        // first hop seen.  The guess only decides how much k_walk_fix re-walks,
        // never a result.  Replay A/B (profiles/r03/walk): stopping early cut
        // this kernel from 217 to 157 us on 1 KiB objects, but with the
        // permissive hop test alone it doubled k_walk_fix (more junk guesses);
        // with the strict test (RAMCRC_SYNC_STRICT) the step is 4.8 % faster.
        // Per round: lane l filters candidates c0 + 8 l + j (j < 8) four at a
        // time with byte-parallel (SWAR) tests on the words it holds
        // (first_hop4); the ~10 % that pass are listed in LDS and chased one
        // per lane, level by level (level 0 is the exact plausible() test),
        // and the wave minima are DPP reductions.  LDS-only: a hop
        // that leaves the staged window ends the candidate (no global round
        // trip for any lane); otherwise beyond-window hops read global memory.
        const bool kill4 = w.capacity <= (1u << 24);   // a 4-byte length ends past it
        const bool kill3 = w.capacity <= (1u << 23);   // so does a 3-byte one >= 2^23
        // The LDS-only instance has no global load: the waits a global peek
        // brings would also wait for the next part's stage loads.
        auto search = [&](auto lds_only_c, uint32_t to) -> uint32_t {
            constexpr bool lds_only = decltype(lds_only_c)::value;
            auto peek_any = [&](uint32_t p) -> uint64_t {
                if constexpr (lds_only)
                    return peek_lds(p);
                else
                    return peek(p);
            };
            const uint32_t wend = B + kSyncWin;   // peeks below wend stay in LDS
            uint64_t best = ~0ull;                // (position after two hops << 32) | candidate
            uint32_t bound = 0xFFFFFFFFu;         // nearest first hop of a survivor: h lies below it
            // (early stop: once a survivor of the preferred class is known)
            for (uint32_t c0 = B; c0 < to && c0 < bound && !(RAMCRC_SYNC_EARLY && best < kSyncJunkKey);
                 c0 += kSyncRound) {
                const uint32_t cl = c0 + uint32_t(lane) * kSyncPer;
                constexpr int kWords = (kSyncPer / 4 + 3) & ~1;
                uint32_t d[kWords];   // bytes [cl, cl + kSyncPer + 8) and up to 4 more
#pragma unroll
                for (int u = 0; u < kWords; u += 2) {
                    // (LDS-only: words past the window belong to candidates >= to, masked below)
                    const uint32_t pc = cl + 4 * u;
                    const uint64_t v = peek_any(lds_only && pc - B > kSyncStage - 8 ? B + kSyncStage - 8 : pc);
                    d[u] = uint32_t(v);
                    d[u + 1] = uint32_t(v >> 32);
                }
                uint32_t alive = 0;
#pragma unroll
                for (int g = 0; g < kSyncPer / 4; g++)
                    alive |= first_hop4(d[g], __builtin_amdgcn_alignbyte(d[g + 1], d[g], 3), kill4,
                                        kill3)
                             << (4 * g);
                alive &= to > cl ? (to - cl >= kSyncPer ? ~0u : (1u << (to - cl)) - 1u) : 0u;
                // survivors listed slot-major in LDS (offsets from c0)
                uint32_t total = 0;
#pragma unroll
                for (int j = 0; j < kSyncPer; j++) {
                    const uint64_t m = __ballot((alive >> j) & 1);
                    const uint32_t at = total + __builtin_amdgcn_mbcnt_hi(
                                                    uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
                    if ((alive >> j) & 1)
                        list[at] = uint16_t(uint32_t(lane) * kSyncPer + j);
                    total += uint32_t(__popcll(m));
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                for (uint32_t t0 = 0; t0 < total; t0 += kWaveSize) {
                    const bool have = t0 + uint32_t(lane) < total;
                    const uint32_t c = c0 + (have ? list[t0 + uint32_t(lane)] : 0u);
                    bool live = have;
                    bool junk = false;   // a hop whose entry is neither an object nor a tombstone
                    uint32_t p = c, first = 0, second = 0;
                    for (int hh = 0; hh < kSyncHops && __ballot(live && p < limit); hh++) {
                        if (live && p < limit) {   // (at the limit the walk ends: keep)
                            if (hh > 0 && lds_only && p >= wend) {
                                live = false;
                            } else {
                                const uint64_t q = peek_any(p);
                                const Hop h = hop_of(q, p);
                                // (guess heuristics, beyond plausible(): a real chain
                                // neither crosses the segment length nor holds an
                                // empty entry -- junk chains through structured
                                // object headers do both)
                                if (plausible(q, h, w.capacity) &&
                                    (!RAMCRC_SYNC_STRICT || (h.next <= limit && h.len != 0))) {
                                    p = uint32_t(h.next);
                                    const uint32_t ty = uint32_t(q) & 0x3F;
                                    junk = junk || (ty != RAMCRC_LOG_ENTRY_TYPE_OBJ &&
                                                    ty != RAMCRC_LOG_ENTRY_TYPE_OBJTOMB);
                                } else {
                                    live = false;
                                }
                            }
                        }
                        if (hh == 0)
                            first = p;
                        if (hh == 1)
                            second = p;
                    }
                    if (second == 0)
                        second = p;
                    if (first == 0)
                        first = p;
                    const uint32_t fb = wave_min(live ? first : 0xFFFFFFFFu);
                    bound = fb < bound ? fb : bound;
                    // nearest second hop, ties to the lower candidate; chains of
                    // objects and tombstones first (RAMCRC_SYNC_TYPES): a fixed
                    // object layout can hold a junk chain of another type that
                    // runs beside the real one at the same stride and never meets
                    // it, and then beats it on the second hop -- k_walk_fix then
                    // re-walks the whole part (128 B values: 0.37 ms per batch)
                    for (int cls = RAMCRC_SYNC_TYPES ? 0 : 1; cls < 2; cls++) {
                        const bool lc = live && (cls == 1 || !junk);
                        const uint32_t s2 = wave_min(lc ? second : 0xFFFFFFFFu);
                        if (s2 != 0xFFFFFFFFu) {
                            const uint64_t tie = __ballot(lc && second == s2);
                            const uint32_t lo = __popcll(tie) == 1
                                                    ? uint32_t(__builtin_amdgcn_readlane(int(c), __builtin_ctzll(tie)))
                                                    : wave_min(lc && second == s2 ? c : 0xFFFFFFFFu);
                            const uint64_t key = (RAMCRC_SYNC_TYPES && cls ? kSyncJunkKey : 0ull) |
                                                 (uint64_t(s2) << 32) | lo;
                            best = key < best ? key : best;
                            break;
                        }
                    }
                }
            }
            return best == ~0ull ? kNoStart : uint32_t(best);   // (bit 63, the class, dropped)
        };
        // entries of up to ~2 KiB: found with LDS reads alone; longer ones
        // (their chain leaves the window) by the general search
        const uint32_t lds_to = B + kSyncWin - 8 < end ? B + kSyncWin - 8 : end;
        uint32_t guess = search(std::true_type{}, lds_to);
        if (guess == kNoStart)
            guess = search(std::false_type{}, end);
        if (lane == 0)
            w.parts[i].start = guess;
    }
}

// The reference walk from `pos` while pos < stop (at most `budget` hops), as
// one lane: fills the part result (count, metadata bytes and raw CRC, exit,
// wrap / overrun flags) and hands every record to sink(index, offset,
// length, header byte).
// seg_peek on one segment.
struct GlobalPeek {
    uint64_t sb;
    uint32_t capacity;
    __device__ uint64_t operator()(uint32_t p) const { return seg_peek(sb, p, capacity); }
};

template <class Sink, class Peek>
__device__ __forceinline__ void walk_lane(const PWalk& w, const uint32_t* tab, uint32_t pos,
                                          uint32_t stop, PartRes& r, Sink&& sink, uint32_t budget,
                                          Peek&& peek)
{
    uint32_t count = 0, nmeta = 0, raw = 0, flags = kPartWalked, hops = 0;
    // The next header's load is issued before this entry's record store:
    // vmcnt counts stores too, so a wait for a load issued after a store
    // would also wait for the store to complete.
    uint64_t q = pos < stop ? peek(pos) : 0ull;
    while (pos < stop) {
        if (hops++ >= budget) {
            flags |= kPartWrap;   // out of budget: the serial walker takes the segment
            break;
        }
        const Hop h = hop_of(q, pos);
        raw = meta_update(tab, raw, q, h.mbytes);
        nmeta += h.mbytes;
        if (h.next > 0xFFFFFFFFull) {
            flags |= kPartWrap;
            break;
        }
        if (h.next > w.capacity) {
            flags |= kPartOverrun;
            break;
        }
        const uint32_t next = uint32_t(h.next);
        const uint64_t qn = next < stop ? peek(next) : 0ull;
        sink(count, pos, h.len, uint32_t(q) & 0xFF);
        count++;
        pos = next;
        q = qn;
    }
    r.exit = pos;
    r.count = count;
    r.nmeta = nmeta;
    r.raw = raw;
    r.flags = flags;
}

template <class Sink>
__device__ __forceinline__ void walk_lane(const PWalk& w, const uint32_t* tab, uint64_t seg,
                                          uint64_t sb, uint32_t pos, uint32_t stop, PartRes& r,
                                          Sink&& sink, uint32_t budget)
{
    walk_lane(w, tab, pos, stop, r, sink, budget, GlobalPeek{sb, w.capacity});
}

// B's re-walks are wave-uniform (every lane chases the same chain), so the
// wave stages the segment bytes around the chain in LDS, kFixWin at a time,
// and each hop reads LDS instead of waiting a memory round trip.
#ifndef RAMCRC_FIX_WIN_KIB
#define RAMCRC_FIX_WIN_KIB 16
#endif
constexpr uint32_t kFixWin = RAMCRC_FIX_WIN_KIB * 1024;
struct WinPeek {
    uint8_t* lds;
    uint64_t sb;
    uint32_t capacity;
    uint32_t wb;   // staged [wb, wb + kFixWin); kNoStart: nothing staged
    __device__ uint64_t operator()(uint32_t p)
    {
        if (wb == kNoStart || p < wb || ((p - wb) & ~3u) + 8 > kFixWin) {
            const uint32_t b = p & ~15u;
            const uint32_t l16 = (threadIdx.x & (kWaveSize - 1)) * 16;
            u32x4 v[kFixWin / 1024];
#pragma unroll
            for (uint32_t u = 0; u < kFixWin / 1024; u++) {
                const uint64_t a = uint64_t(b) + u * 1024 + l16;
                v[u] = a + 16 <= capacity ? load16(sb + a) : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (uint32_t u = 0; u < kFixWin / 1024; u++)
                *reinterpret_cast<u32x4*>(lds + u * 1024 + l16) = v[u];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            wb = b;
        }
        const uint32_t o = p - wb;
        const uint32_t* w32 = reinterpret_cast<const uint32_t*>(lds + (o & ~3u));
        return ((uint64_t(w32[1]) << 32) | w32[0]) >> (8 * (o & 3));
    }
};

struct NoSink {
    __device__ void operator()(uint32_t, uint32_t, uint32_t, uint32_t) const {}
};

// Records straight to the table (slots below the table's capacity).
struct TableSink {
    u32x4* out;
    uint64_t n;
    uint32_t seg;
    uint32_t* hard;   // nullable: ORed with the written records' replay_hard bits
    __device__ void operator()(uint32_t idx, uint32_t pos, uint32_t len, uint32_t hdr) const
    {
        if (idx < n) {
            out[idx] = u32x4{seg, pos, len, hdr};
            if (hard)
                *hard |= replay_hard(pos, len, hdr);
        }
    }
};

__device__ __forceinline__ void walk_tab_fill(uint32_t* tab)
{
    for (uint32_t t = threadIdx.x; t < 4 * 256; t += blockDim.x)
        tab[t] = g_tab.pos[1 + kTinyRow0 + t / 256][t % 256];
    __syncthreads();
}

// A: one lane per part.
// A keeps each lane's records (offset; length << 8 | header byte) in LDS
// while it chases, then the wave writes them part by part with coalesced
// stores: records stored by a lane one hop at a time would reach memory as
// partial lines.  A part with more than kPartRec records, or an entry of
// 16 MiB or more, is marked kPartSpill and walked again by C; its first
// kPartRec records still go to the scratch (B meets a misguessed chain within
// its first few entries), unless an entry's length does not fit a record.
__global__ __launch_bounds__(256) void k_walk_parts(PWalk w0)
{
    const PWalk w = walk_geo(w0);
    __shared__ uint32_t tab[4 * 256];
    __shared__ uint2 lrec[256][kPartRec];
    walk_tab_fill(tab);
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const bool valid = i < w.nseg * w.nparts;
    PartRes r{};
    uint2* mine = lrec[threadIdx.x];
    bool huge = false, lost = false;
    // a full block of this lane's records to its place: block 0 to the
    // part's scratch, later ones to pool blocks (a lane's 512 contiguous
    // bytes; the lines fill up in L2)
    auto put_block = [&](uint32_t b, uint32_t n) {
        uint2* dst = nullptr;
        if (b == 0) {
            dst = w.recs + i * kPartRec;
        } else if (b <= kMaxBlocks && !lost) {
            const unsigned long long k = atomicAdd(w.pool_used, 1ull);
            if (k < w.pool_cap) {
                dst = w.pool + k * kPartRec;
                w.blocks[i * kMaxBlocks + (b - 1)] = uint32_t(k);
                w.pool_owner[k] = uint32_t(i * 16 + b);
            }
        }
        if (!dst) {
            lost = true;   // C walks the part again
            return;
        }
        for (uint32_t e = 0; e < n; e += 2) {
            const uint2 a0 = mine[e], a1 = mine[e + 1];
            if (e + 1 < n)
                *reinterpret_cast<uint4*>(dst + e) = make_uint4(a0.x, a0.y, a1.x, a1.y);
            else
                dst[e] = a0;
        }
    };
    if (valid) {
        const uint64_t seg = i / w.nparts;
        const uint32_t k = uint32_t(i - seg * w.nparts);
        const uint32_t B = k << w.pshift;
        const uint32_t limit = walk_limit(w, seg);
        r = w.parts[i];
        const uint32_t start = k == 0 ? 0u : r.start;
        r.start = start;
        if (start == kNoStart || B >= limit) {
            r.flags = 0;
            r.count = r.nmeta = r.raw = 0;
            r.exit = start;
        } else {
            const uint32_t pend = uint32_t(uint64_t(B) + (1ull << w.pshift) < w.capacity
                                               ? uint64_t(B) + (1ull << w.pshift) : w.capacity);
            const uint64_t sb = reinterpret_cast<uint64_t>(w.base) + seg * w.stride;
            walk_lane(w, tab, seg, sb, start, pend < limit ? pend : limit, r,
                      [&](uint32_t idx, uint32_t pos, uint32_t len, uint32_t hdr) {
                          // a part of at most kPartRec records keeps them in LDS
                          // for the wave's coalesced flush below; a denser part
                          // writes every full block as it goes
                          if (idx == kPartRec)
                              put_block(0, kPartRec);
                          mine[idx & (kPartRec - 1)] = make_uint2(pos, (len << 8) | hdr);
                          huge = huge || len >= (1u << 24);
                          if (idx >= kPartRec && (idx & (kPartRec - 1)) == kPartRec - 1)
                              put_block(idx / kPartRec, kPartRec);
                      },
                      1u << w.pshift);
            if (r.count > kPartRec && (r.count & (kPartRec - 1)))
                put_block(r.count / kPartRec, r.count & (kPartRec - 1));
            if (r.count > kPartRec * (1 + kMaxBlocks) || huge || lost)
                r.flags |= kPartSpill;
            if (huge)
                r.flags |= kPartHuge;
        }
        w.parts[i] = r;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's LDS records
    const int lane = threadIdx.x & (kWaveSize - 1);
    const bool flush = valid && (r.flags & kPartWalked) && !(r.flags & kPartHuge) && r.count <= kPartRec;
    uint64_t todo = __ballot(flush);
    while (todo) {
        const int j = __builtin_ctzll(todo);
        todo &= todo - 1;
        const uint32_t n = __shfl(r.count, j, kWaveSize);
        const uint64_t dst = (i - uint64_t(lane) + uint64_t(j)) * kPartRec;
        const uint2* src = lrec[(threadIdx.x & ~63u) + uint32_t(j)];
        for (uint32_t e = uint32_t(lane); e < n; e += kWaveSize)
            w.recs[dst + e] = src[e];
    }
}

#ifdef RAMCRC_WALK_DEBUG
__device__ unsigned long long g_fixdbg[8];
#endif

// B: one wave per segment, lane k deciding part k of a chunk of 64.  A part
// is accepted as A walked it when the true chain arrives at its guess, or
// meets the guessed chain within kMeetHops entries at one of its first
// kMeetMax records (a junk guess whose length lands on the true chain: the
// common misguess); the true arrival offset of part k is the exit of part
// k-1 as A walked it, so every part is checked at once.  The parts that
// fail -- a guess that never meets, a part the chain jumps over, a part left
// unwalked -- are resolved in order by the whole wave (re-walked from the
// true offset through an LDS window), each resolution re-checking the part
// after it.  The accepted parts' metadata CRCs fold into the segment's with
// one GF(2) multiply per part, then the status is written and the records
// are allocated (one atomic per segment).
__global__ __launch_bounds__(kWaveSize) void k_walk_fix(PWalk w0)
{
    const PWalk w = walk_geo(w0);
    __shared__ uint32_t tab[4 * 256];
    __shared__ __attribute__((aligned(16))) uint8_t win[kFixWin];
    walk_tab_fill(tab);
    const int lane = threadIdx.x;
    for (uint64_t seg = blockIdx.x; seg < w.nseg; seg += gridDim.x) {
        const uint32_t limit = walk_limit(w, seg);
        const ramcrc_seg_cert cert = w.certs[seg];
        const uint64_t sb = reinterpret_cast<uint64_t>(w.base) + seg * w.stride;
        WinPeek wpeek{win, sb, w.capacity, kNoStart};
        PartRes* parts = w.parts + seg * w.nparts;
        // The true chain (wave-uniform): pos, the metadata CRC so far (raw
        // state from 0xFFFFFFFF), the records before the current chunk.
        uint32_t pos = 0, crc = 0xFFFFFFFFu, count = 0, rewalk = 0;
        bool overrun = false, fallback = false;
#ifdef RAMCRC_WALK_DEBUG
        uint32_t dbg_meet = 0, dbg_meet_hops = 0, dbg_chase = 0, dbg_miss = 0;
        bool fast = true;
        const uint64_t dbg_t0 = __builtin_amdgcn_s_memrealtime();
#endif
        // Fold the accepted parts of a chunk (one per lane) into crc in one
        // step: crc <- X^n(crc) ^ sum_j X^(suffix_j)(raw_j), suffix_j = the
        // metadata bytes of the accepted parts after j, n = all of them.
        auto fold = [&](bool acc, uint32_t nmeta, uint32_t raw) {
            const uint32_t nm = acc ? nmeta : 0u;
            uint32_t incl = nm;   // inclusive suffix sum over higher lanes
#pragma unroll
            for (int s = 1; s < kWaveSize; s <<= 1) {
                const uint32_t y = __shfl_down(incl, s, kWaveSize);
                if (lane + s < kWaveSize)
                    incl += y;
            }
            const uint32_t n_all = __shfl(incl, 0, kWaveSize);
            uint32_t c = acc ? mulmod_horner(raw, xpow8_dev(incl - nm)) : 0u;
#pragma unroll
            for (int s = 1; s < kWaveSize; s <<= 1)
                c ^= __shfl_xor(c, s, kWaveSize);
            crc = mulmod_horner(crc, xpow8_dev(n_all)) ^ c;
        };
        // Where the chain arriving at pe meets part k's guessed chain: after
        // `hops` (<= kMeetHops) entries walked from pe, at the guess's record
        // `cut` (0: the guess itself, up to kMeetMax); -1 when it does not.
        // The walked entries' header + length bytes: raw CRC wr over wn bytes.
        auto meet_at = [&](uint32_t k, uint32_t st, uint32_t fl, uint32_t gc, uint32_t pe,
                           uint32_t& wr, uint32_t& wn) -> int {
            wr = wn = 0;
            const uint64_t Ek = (uint64_t(k) << w.pshift) + (1ull << w.pshift);
            if (!(fl & kPartWalked) || (fl & kPartWrap) || uint64_t(pe) >= Ek)
                return -1;
            // the scratch holds a part's first kPartRec records (none when an
            // entry's length does not fit a record): met at its start only then
            const uint32_t gn = (fl & kPartHuge) ? 0u : (gc < kPartRec ? gc : kPartRec);
            const uint64_t base = (uint64_t(seg) * w.nparts + k) * kPartRec;
            uint32_t p = pe;
            for (uint32_t hh = 0;; hh++) {
                if (p == st)
                    return int(hh << 8);
                for (uint32_t c = 1; c <= kMeetMax && c < gn; c++)
                    if (w.recs[base + c].x == p)
                        return int((hh << 8) | c);
                if (hh == kMeetHops || p >= limit || uint64_t(p) >= Ek)
                    return -1;
                const uint64_t q = seg_peek(sb, p, w.capacity);
                const Hop h = hop_of(q, p);
                if (h.next > w.capacity)
                    return -1;
                wr = meta_update(tab, wr, q, h.mbytes);
                wn += h.mbytes;
                p = uint32_t(h.next);
            }
        };
        const uint32_t nlive =
            limit == 0 ? 0u : uint32_t((uint64_t(limit) + (1ull << w.pshift) - 1) >> w.pshift);
        for (uint32_t k0 = 0; k0 < nlive && !overrun && !fallback; k0 += kWaveSize) {
            const uint32_t k = k0 + uint32_t(lane);
            const bool in = k < nlive;
            PartRes r{};
            if (in)
                r = parts[k];
            const uint32_t gst = r.start;   // A's guess
            // per lane: ok (decided), emit (accepted: walked or met), the
            // meet to apply (mt >= 0; kResolved: totals already final), and
            // the exit handed to the next part
            constexpr int kResolved = -2;
            uint32_t ex = r.exit, wr = 0, wn = 0;
            int mt = -1;
            {
                uint32_t pe = __shfl_up(ex, 1, kWaveSize);
                pe = lane == 0 ? pos : pe;
                if (in)
                    mt = meet_at(k, gst, r.flags, r.count, pe, wr, wn);
                if (mt > 0)
                    r.start = pe;
            }
            bool ok = !in || mt >= 0, emit = in && mt >= 0;
            while (true) {
                // the first undecided part; every part before it is decided
                const uint64_t bad = __ballot(!ok);
                if (!bad)
                    break;
                const int j = int(__builtin_ctzll(bad));
                // an accepted part below it that overran ends the chain
                const uint64_t ovr = __ballot(emit && (r.flags & kPartOverrun));
                if (ovr && int(__builtin_ctzll(ovr)) < j)
                    break;
#ifdef RAMCRC_WALK_DEBUG
                fast = false;
#endif
                const uint32_t kj = k0 + uint32_t(j);
                const uint32_t pe = j == 0 ? pos : uint32_t(__builtin_amdgcn_readlane(int(ex), j - 1));
                const uint32_t st = uint32_t(__builtin_amdgcn_readlane(int(gst), j));
                const uint32_t fl = uint32_t(__builtin_amdgcn_readlane(int(r.flags), j));
                const uint64_t Ej64 = (uint64_t(kj) << w.pshift) + (1ull << w.pshift);
                const uint32_t Ej = uint32_t(Ej64 < w.capacity ? Ej64 : w.capacity);
                const uint32_t stop = Ej < limit ? Ej : limit;
                const uint32_t budget = rewalk < kRewalkBudget ? kRewalkBudget - rewalk : 0u;
                bool jemit = true;
                uint32_t jex = pe;
                if (uint64_t(pe) >= Ej64) {
                    jemit = false;   // the chain jumps over this part
                } else if (fl & kPartWalked) {
                    // Walk from pe until the chain meets the guessed one at any
                    // of the offsets A recorded for it (lane e holds its e-th
                    // entry; the first is the guess); its entries from there on
                    // are the true chain's.  Without a meeting the walk covers
                    // the part (a full re-walk).
                    const uint32_t gc = uint32_t(__builtin_amdgcn_readlane(int(r.count), j));
                    const uint32_t gn = (fl & kPartHuge) ? 0u : (gc < kPartRec ? gc : kPartRec);
                    const uint64_t pidx = uint64_t(seg) * w.nparts + kj;
                    uint2 g = make_uint2(0xFFFFFFFFu, 0u);
                    if (uint32_t(lane) < gn)
                        g = w.recs[pidx * kPartRec + uint32_t(lane)];
                    uint32_t p = pe, wc = 0, wnn = 0, wrr = 0, wflags = kPartWalked;
                    int cut = -1;
                    // the walk's records and header + length bytes, 64 at a time:
                    // record wc in lane wc % 64; each full block's metadata CRC is
                    // summed in parallel off the chase, and blocks 1.. go to pool
                    // blocks (unattached until the walk proves to be a re-walk)
                    uint2 mine = make_uint2(0u, 0u), mine0 = make_uint2(0u, 0u);
                    uint64_t mq = 0;
                    uint32_t myblk = 0xFFFFFFFFu;   // lane b: pool block of block b
                    bool huge = false, pool_ok = true;
                    auto fold_block = [&](uint32_t n) {   // lanes < n hold metadata
                        const bool inr = uint32_t(lane) < n;
                        const uint32_t mb = inr ? uint32_t((mq >> 6) & 3) + 2 : 0u;
                        const uint32_t re = inr ? meta_update(tab, 0u, mq, mb) : 0u;
                        uint32_t incl = mb;
#pragma unroll
                        for (int s2 = 1; s2 < kWaveSize; s2 <<= 1) {
                            const uint32_t y = __shfl_down(incl, s2, kWaveSize);
                            if (lane + s2 < kWaveSize)
                                incl += y;
                        }
                        const uint32_t hn = __shfl(incl, 0, kWaveSize);
                        uint32_t hr = inr ? mulmod_horner(re, xpow8_dev(incl - mb)) : 0u;
#pragma unroll
                        for (int s2 = 1; s2 < kWaveSize; s2 <<= 1)
                            hr ^= __shfl_xor(hr, s2, kWaveSize);
                        // raw(0, A||B) = X^|B|(raw(0, A)) ^ raw(0, B)
                        wrr = mulmod_horner(wrr, xpow8_dev(hn)) ^ hr;
                        wnn += hn;
                    };
                    auto store_block = [&](uint32_t b, uint32_t n) {   // lanes < n hold records
                        if (b == 0) {
                            mine0 = mine;
                            return;
                        }
                        if (!pool_ok || b > kMaxBlocks) {
                            pool_ok = false;
                            return;
                        }
                        unsigned long long k = 0;
                        if (lane == 0)
                            k = atomicAdd(w.pool_used, 1ull);
                        k = __shfl(k, 0, kWaveSize);
                        if (k >= w.pool_cap) {
                            pool_ok = false;
                            return;
                        }
                        if (uint32_t(lane) < n)
                            w.pool[k * kPartRec + uint32_t(lane)] = mine;
                        if (lane == 0)
                            w.pool_owner[k] = 0xFFFFFFFFu;   // unattached
                        if (uint32_t(lane) == b)
                            myblk = uint32_t(k);
                    };
                    while (true) {
                        const uint64_t hit = __ballot(uint32_t(lane) < gn && g.x == p);
                        if (hit || (!(fl & kPartWrap) && p == st)) {
                            cut = hit ? int(__builtin_ctzll(hit)) : 0;
                            break;
                        }
                        if (p >= stop)
                            break;
                        if (wc >= budget) {
                            wflags |= kPartWrap;   // out of budget: the serial walker
                            break;
                        }
                        const uint64_t q = wpeek(p);
                        const Hop h = hop_of(q, p);
                        if (uint32_t(lane) == (wc & (kWaveSize - 1)))
                            mq = q;
                        if (h.next > 0xFFFFFFFFull) {
                            wflags |= kPartWrap;
                            break;
                        }
                        if (h.next > w.capacity) {
                            wflags |= kPartOverrun;
                            break;
                        }
                        if (uint32_t(lane) == (wc & (kWaveSize - 1)))
                            mine = make_uint2(p, (h.len << 8) | (uint32_t(q) & 0xFF));
                        huge = huge || h.len >= (1u << 24);
                        wc++;
                        p = uint32_t(h.next);
                        if ((wc & (kWaveSize - 1)) == 0) {
                            fold_block(kWaveSize);
                            store_block(wc / kWaveSize - 1, kWaveSize);
                        }
                    }
                    rewalk += wc + 1;
                    {
                        // the last partial block's header + length bytes (with an
                        // entry that overran or wrapped: the reference checksums its
                        // header too)
                        const uint32_t rem = (wc & (kWaveSize - 1)) +
                                             ((wflags & (kPartWrap | kPartOverrun)) ? 1u : 0u);
                        if (rem)
                            fold_block(rem);
                    }
                    if (cut >= 0 && (fl & kPartWrap)) {
                        wflags |= kPartWrap;   // met a chain that wraps: the serial walker
                    } else if (cut >= 0) {
#ifdef RAMCRC_WALK_DEBUG
                        dbg_meet++;
                        dbg_meet_hops += wc;
#endif
                        // the guess's totals minus its first `cut` entries, whose
                        // header + length bytes are folded from the records:
                        // raw(0, A||S) = X^|S|(raw(0, A)) ^ raw(0, S)
                        const bool inp = lane < cut;
                        const uint32_t mb = inp ? ((g.y >> 6) & 3) + 2 : 0u;
                        const uint64_t qe = uint64_t(g.y & 0xFF) | (uint64_t(g.y >> 8) << 8);
                        const uint32_t re = inp ? meta_update(tab, 0u, qe, mb) : 0u;
                        uint32_t incl = mb;   // suffix sums of the prefix's bytes
#pragma unroll
                        for (int s = 1; s < kWaveSize; s <<= 1) {
                            const uint32_t y = __shfl_down(incl, s, kWaveSize);
                            if (lane + s < kWaveSize)
                                incl += y;
                        }
                        const uint32_t pn = __shfl(incl, 0, kWaveSize);
                        uint32_t pr = inp ? mulmod_horner(re, xpow8_dev(incl - mb)) : 0u;
#pragma unroll
                        for (int s = 1; s < kWaveSize; s <<= 1)
                            pr ^= __shfl_xor(pr, s, kWaveSize);
                        const uint32_t tn = uint32_t(__builtin_amdgcn_readlane(int(r.nmeta), j));
                        const uint32_t tr = uint32_t(__builtin_amdgcn_readlane(int(r.raw), j));
                        const uint32_t sn = tn - pn;   // suffix metadata bytes
                        const uint32_t sr = tr ^ mulmod_horner(pr, xpow8_dev(sn));
                        jex = uint32_t(__builtin_amdgcn_readlane(int(r.exit), j));
                        const uint32_t nn = wnn + sn;
                        const uint32_t rr = mulmod_horner(wrr, xpow8_dev(sn)) ^ sr;
                        if (lane == j) {
                            r.start = pe;
                            r.count = wc + gc - uint32_t(cut);
                            r.nmeta = nn;
                            r.raw = rr;
                            r.pre = wc;
                            r.cut = uint32_t(cut);
                            mt = kResolved;
                        }
                    } else {
#ifdef RAMCRC_WALK_DEBUG
                        dbg_chase++;
                        {
                            const uint32_t g0 = uint32_t(__builtin_amdgcn_readlane(int(g.x), 0));
                            const uint32_t g1 = uint32_t(__builtin_amdgcn_readlane(int(g.x), 1));
                            const uint32_t g2 = uint32_t(__builtin_amdgcn_readlane(int(g.x), 2));
                            const uint32_t l0 = uint32_t(__builtin_amdgcn_readlane(int(g.y), 0));
                            const uint64_t q0 = seg_peek(sb, pe, w.capacity);
                            const Hop h0 = hop_of(q0, pe);
                            const uint64_t qg = seg_peek(sb, st, w.capacity);
                            if (lane == 0)
                                printf("chasedbg seg=%u part=%u B=%u pe=%u st=%u g=%u,%u,%u ghdr=%08x glen=%u "
                                       "true_hdr=%02x true_len=%u true_next=%u qg=%016llx q0=%016llx\n",
                                       uint32_t(seg), kj, kj << w.pshift, pe, st, g0, g1, g2, l0 & 0xFF,
                                       l0 >> 8, uint32_t(q0 & 0xFF), h0.len, uint32_t(h0.next),
                                       (unsigned long long)qg, (unsigned long long)q0);
                        }
#endif
                        // walked the whole part: its records go to the scratch and
                        // pool blocks (C copies them), or, when they do not fit, C
                        // walks it again
                        jex = p;
                        if (wc > kPartRec && (wc & (kPartRec - 1)))
                            store_block(wc / kPartRec, wc & (kPartRec - 1));
                        const bool keep = !huge && pool_ok && wc <= kPartRec * (1 + kMaxBlocks);
                        if (keep) {
                            const uint2 first = wc <= kPartRec ? mine : mine0;
                            if (uint32_t(lane) < (wc < kPartRec ? wc : kPartRec))
                                w.recs[pidx * kPartRec + uint32_t(lane)] = first;
                            // replace A's blocks of this part by the walk's
                            const uint32_t nb = (wc + kPartRec - 1) / kPartRec;   // blocks incl. 0
                            if (lane >= 1 && uint32_t(lane) <= kMaxBlocks) {
                                const uint32_t own = uint32_t(pidx * 16 + uint32_t(lane));
                                const uint32_t old = w.blocks[pidx * kMaxBlocks + uint32_t(lane) - 1];
                                if (old < w.pool_cap && w.pool_owner[old] == own)
                                    w.pool_owner[old] = 0xFFFFFFFFu;
                                if (uint32_t(lane) < nb) {
                                    w.blocks[pidx * kMaxBlocks + uint32_t(lane) - 1] = myblk;
                                    w.pool_owner[myblk] = own;
                                }
                            }
                        }
                        if (lane == j) {
                            r.start = pe;
                            r.exit = p;
                            r.count = wc;
                            r.nmeta = wnn;
                            r.raw = wrr;
                            r.flags = keep ? wflags : (wflags | kPartChase);
                            r.pre = r.cut = 0;
                            mt = kResolved;
                        }
                    }
                    if (wflags & kPartWrap)
                        fallback = true;
                } else {
#ifdef RAMCRC_WALK_DEBUG
                    dbg_miss++;
#endif
                    // no guess: walk this part from the true offset, its
                    // records to the scratch as above
                    PartRes x;
                    uint2 mine = make_uint2(0u, 0u);
                    bool huge = false;
                    walk_lane(w, tab, pe, stop, x,
                              [&](uint32_t idx, uint32_t rp, uint32_t len, uint32_t hdr) {
                                  if (uint32_t(lane) == idx)
                                      mine = make_uint2(rp, (len << 8) | hdr);
                                  huge = huge || len >= (1u << 24);
                              },
                              budget, wpeek);
                    rewalk += x.count + 1;
                    jex = x.exit;
                    const bool keep = x.count <= kPartRec && !huge;
                    if (keep && uint32_t(lane) < x.count)
                        w.recs[(uint64_t(seg) * w.nparts + kj) * kPartRec + uint32_t(lane)] = mine;
                    if (lane == j) {
                        r.start = pe;
                        r.exit = x.exit;
                        r.count = x.count;
                        r.nmeta = x.nmeta;
                        r.raw = x.raw;
                        r.flags = keep ? x.flags : (x.flags | kPartChase);
                        r.pre = r.cut = 0;
                        mt = kResolved;
                    }
                    if (x.flags & kPartWrap)
                        fallback = true;
                }
                if (fallback)
                    break;
                if (lane == j) {
                    ok = true;
                    emit = jemit;
                    ex = jex;
                    mt = kResolved;
                }
                // the part after j: its arrival offset is now known
                if (lane == j + 1 && in) {
                    mt = meet_at(k, gst, r.flags, r.count, jex, wr, wn);
                    r.start = mt > 0 ? jex : gst;
                    ok = mt >= 0;
                    emit = ok;
                }
            }
            if (fallback)
                break;
            // the chain ends at the first accepted part that overran
            const uint64_t ovr = __ballot(emit && (r.flags & kPartOverrun));
            const int olane = ovr ? int(__builtin_ctzll(ovr)) : kWaveSize;
            if (lane > olane)
                emit = false;
            if (emit && mt > 0) {
                // drop the guess's first `cut` entries (junk), whose header +
                // length bytes are rebuilt from the records, and put the
                // `hops` entries walked from the arrival offset in front
#ifdef RAMCRC_WALK_DEBUG
                dbg_meet++;
#endif
                const uint32_t hops = uint32_t(mt) >> 8, cut = uint32_t(mt) & 0xFF;
                const uint64_t base = (uint64_t(seg) * w.nparts + k) * kPartRec;
                uint32_t jr = 0, jn = 0;
                for (uint32_t e = 0; e < cut; e++) {
                    const uint2 g = w.recs[base + e];
                    const uint32_t mb = ((g.y >> 6) & 3) + 2;
                    const uint64_t qe = uint64_t(g.y & 0xFF) | (uint64_t(g.y >> 8) << 8);
                    jr = meta_update(tab, jr, qe, mb);
                    jn += mb;
                }
                const uint32_t tn = r.nmeta - jn;
                const uint32_t tr = r.raw ^ mulmod_horner(jr, xpow8_dev(tn));
                r.raw = mulmod_horner(wr, xpow8_dev(tn)) ^ tr;
                r.nmeta = wn + tn;
                r.count = hops + r.count - cut;
                r.pre = hops;   // walked again (and emitted) by C
                r.cut = cut;
            } else if (emit && mt == 0) {
                r.pre = r.cut = 0;   // accepted as walked
            }
            const uint32_t c = emit ? r.count : 0u;
            uint32_t incl = c;   // inclusive prefix of the record counts
#pragma unroll
            for (int s = 1; s < kWaveSize; s <<= 1) {
                const uint32_t y = __shfl_up(incl, s, kWaveSize);
                if (lane >= s)
                    incl += y;
            }
            fold(emit, r.nmeta, r.raw);
            if (emit) {
                r.rec = count + incl - c;
                r.flags |= kPartEmit;
                parts[k] = r;
            }
            count += uint32_t(__builtin_amdgcn_readlane(int(incl), kWaveSize - 1));
            // the chain's position after the chunk: the overrun part's exit,
            // else the last live part's
            const int last = olane < kWaveSize ? olane
                                               : int(nlive - 1 - k0 < uint32_t(kWaveSize - 1)
                                                         ? nlive - 1 - k0 : uint32_t(kWaveSize - 1));
            pos = uint32_t(__builtin_amdgcn_readlane(int(ex), last));
            overrun = olane < kWaveSize;
        }
#ifdef RAMCRC_WALK_DEBUG
        const uint64_t dbg_t1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            const unsigned long long dt = dbg_t1 - dbg_t0;
            atomicMax(&g_fixdbg[fast ? 0 : 1], dt);
            atomicAdd(&g_fixdbg[fast ? 2 : 3], 1ull);
            atomicAdd(&g_fixdbg[fast ? 4 : 5], dt);
            if (!fast)
                printf("fixdbg seg=%u meet=%u meet_hops=%u chase=%u miss=%u rewalk=%u us=%.1f\n",
                       uint32_t(seg), dbg_meet, dbg_meet_hops, dbg_chase, dbg_miss, rewalk,
                       double(dt) / 100.0);
            if (atomicAdd(&g_fixdbg[7], 1ull) == w.nseg - 1) {
                printf("fixsum fast n=%llu max=%.1fus avg=%.1fus slow n=%llu max=%.1fus avg=%.1fus\n",
                       g_fixdbg[2], g_fixdbg[0] / 100.0, g_fixdbg[4] / 100.0 / (g_fixdbg[2] + 1e-9),
                       g_fixdbg[3], g_fixdbg[1] / 100.0, g_fixdbg[5] / 100.0 / (g_fixdbg[3] + 1e-9));
                for (int t = 0; t < 8; t++)
                    g_fixdbg[t] = 0;
            }
        }
#endif
        if (fallback) {
            if (lane == 0)
                w.fallback[seg] = 1;
            continue;
        }
        uint32_t flags = 0;
        const uint32_t fin = ~crc_small(tab, crc, cert.segment_length, 4);
        if (overrun)
            flags |= RAMCRC_SEG_PAST_CAPACITY;
        else if (pos > cert.segment_length)
            flags |= RAMCRC_SEG_PAST_LENGTH;
        else if (fin != cert.checksum)
            flags |= RAMCRC_SEG_BAD_CHECKSUM;
        unsigned long long b = 0;
        if (lane == 0 && count)
            b = atomicAdd(w.n_entries, (unsigned long long)count);
        b = __shfl(b, 0, kWaveSize);
        if (b + count > w.cap)
            flags |= RAMCRC_SEG_TABLE_FULL;
        if (!(flags & (RAMCRC_SEG_PAST_CAPACITY | RAMCRC_SEG_PAST_LENGTH | RAMCRC_SEG_BAD_CHECKSUM |
                       RAMCRC_SEG_TABLE_FULL)))
            flags |= RAMCRC_SEG_OK;   // records dropped (TABLE_FULL): not verified, never OK
        if (lane == 0) {
            w.fallback[seg] = 0;
            w.seg_base[seg] = b;
            ramcrc_seg_status st;
            st.flags = flags;
            st.checksum = fin;
            st.entries = count;
            st.bad_objects = 0;
            w.status[seg] = st;
        }
    }
}

// C: the records of every accepted part at their final slots.  A part
// accepted as walked (the common case) already has its records in the
// scratch A wrote: the wave copies them, part after part, 64 records per
// instruction.  Entries walked by k_walk_fix before it met the guessed chain
// are walked once more here; parts walked again in full, or with more
// records than the scratch holds, are walked again here in full.
__global__ __launch_bounds__(256) void k_walk_emit(PWalk w0)
{
    const PWalk w = walk_geo(w0);
    __shared__ uint32_t tab[4 * 256];
    walk_tab_fill(tab);
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const bool valid = i < w.nseg * w.nparts;
    const uint64_t seg = valid ? i / w.nparts : 0;
    PartRes r{};
    bool emit = false;
    uint64_t slot = 0;
    if (valid) {
        r = w.parts[i];
        emit = (r.flags & kPartEmit) && !w.fallback[seg];
        if (emit)
            slot = w.seg_base[seg] + r.rec;
    }
    const bool chase = emit && (r.flags & (kPartChase | kPartSpill));
    const uint32_t pre = emit && !chase ? r.pre : 0u;
    uint32_t hard = 0;
    if (chase || pre) {
        const uint32_t k = uint32_t(i - seg * w.nparts);
        const uint32_t B = k << w.pshift;
        const uint32_t limit = walk_limit(w, seg);
        const uint32_t pend = uint32_t(uint64_t(B) + (1ull << w.pshift) < w.capacity ? uint64_t(B) + (1ull << w.pshift)
                                                                             : w.capacity);
        const uint64_t sb = reinterpret_cast<uint64_t>(w.base) + seg * w.stride;
        PartRes x;
        walk_lane(w, tab, seg, sb, r.start, pend < limit ? pend : limit, x,
                  TableSink{w.entries + slot, slot < w.cap ? w.cap - slot : 0, uint32_t(seg),
                            w.sum ? &hard : nullptr},
                  chase ? (1u << w.pshift) : pre);
    }
    if (w.sum) {
        const uint32_t hw = (__ballot(hard & 1u) ? 1u : 0u) | (__ballot(hard & 2u) ? 2u : 0u) |
                           (__ballot(hard & 4u) ? 4u : 0u);
        if (hw && (threadIdx.x & (kWaveSize - 1)) == 0 && (hw & ~walk_sum_seen(w.sum)))
            atomicOr(w.sum, hw);
    }
}

// C': the scratch records of the parts accepted without a second walk.  One
// wave per block of kPartRec (= 64) records -- a part's first block in the
// scratch, then the pool blocks in use -- lane j copying record j.  The copy
// is a chain of dependent loads (block owner and records, the part's result,
// the segment's base), so a wave takes kCopyU blocks at a time and issues
// each level's loads for all of them together.
static_assert(kPartRec == kWaveSize, "k_walk_copy: one lane per record of a block");

#ifndef RAMCRC_COPY_NT
#define RAMCRC_COPY_NT 1   // k_walk_copy: nontemporal record stores (replay 64 B +1.7 %)
#endif
#ifndef RAMCRC_COPY_U
#define RAMCRC_COPY_U 4
#endif
constexpr int kCopyU = RAMCRC_COPY_U;
__global__ __launch_bounds__(256) void k_walk_copy(PWalk w0)
{
    const PWalk w = walk_geo(w0);
    const uint64_t nfirst = w.nseg * w.nparts;
    const uint64_t used = *w.pool_used;
    const uint64_t nblk = nfirst + (used < w.pool_cap ? used : w.pool_cap);
    const uint64_t nwave = uint64_t(gridDim.x) * (blockDim.x / kWaveSize);
    const uint32_t lane = threadIdx.x & (kWaveSize - 1);
    // the fused replay's summary (w.sum) over every record copied; the
    // records C walks again set it in k_walk_emit.  (Taking it in A and the
    // fix-up instead -- the last hard index per part, counted from each
    // accepted part's cut -- measured 1 % slower: profiles/r05/replayfix.)
    const uint32_t seen = walk_sum_seen(w.sum);
    uint32_t hard = 0;
    for (uint64_t b0 = (uint64_t(blockIdx.x) * (blockDim.x / kWaveSize) +
                        __builtin_amdgcn_readfirstlane(threadIdx.x / kWaveSize)) * kCopyU;
         b0 < nblk; b0 += nwave * kCopyU) {
        uint64_t part[kCopyU];
        uint32_t blk[kCopyU];   // block number within the part; ~0u: nothing to copy
        uint2 v[kCopyU];
#pragma unroll
        for (int u = 0; u < kCopyU; u++) {
            const uint64_t bi = b0 + u;
            blk[u] = ~0u;
            part[u] = 0;
            if (bi < nfirst) {
                part[u] = bi;
                blk[u] = 0;
                v[u] = w.recs[bi * kPartRec + lane];
            } else if (bi < nblk) {
                const uint32_t own = w.pool_owner[bi - nfirst];
                v[u] = w.pool[(bi - nfirst) * kPartRec + lane];
                if (own != 0xFFFFFFFFu) {   // else a block the fix-up wrote for a walk that met the guess
                    part[u] = own / 16;
                    blk[u] = own % 16;
                }
            }
        }
        PartRes r[kCopyU];
#pragma unroll
        for (int u = 0; u < kCopyU; u++)
            if (blk[u] != ~0u)
                r[u] = w.parts[part[u]];
        uint32_t fb[kCopyU];
        uint64_t sbase[kCopyU];
#pragma unroll
        for (int u = 0; u < kCopyU; u++) {
            const uint32_t fl = r[u].flags;
            if (blk[u] != ~0u && (!(fl & kPartEmit) || (fl & (kPartChase | kPartSpill))))
                blk[u] = ~0u;
            if (blk[u] != ~0u) {
                const uint64_t seg = part[u] / w.nparts;
                fb[u] = w.fallback[seg];
                sbase[u] = w.seg_base[seg];
            }
        }
#pragma unroll
        for (int u = 0; u < kCopyU; u++) {
            if (blk[u] == ~0u || fb[u])
                continue;
            const uint32_t n = r[u].count - r[u].pre;   // records ri = cut .. cut + n - 1
            const uint32_t ri = blk[u] * kPartRec + lane;
            if (ri < r[u].cut || ri - r[u].cut >= n)
                continue;
            const uint64_t dst = sbase[u] + r[u].rec + r[u].pre + (ri - r[u].cut);
            if (dst < w.cap) {
                const u32x4 rec = {uint32_t(part[u] / w.nparts), v[u].x, v[u].y >> 8, v[u].y & 0xFF};
#if RAMCRC_COPY_NT
                // streamed: not read back by this kernel.  (The same for the
                // part walk's scratch stores was 8 % slower: k_walk_copy reads
                // that scratch back while it is still in the caches.)
                __builtin_nontemporal_store(rec, &w.entries[dst]);
#else
                w.entries[dst] = rec;
#endif
                hard |= (seen & kHardAll) != kHardAll ? replay_hard(v[u].x, v[u].y >> 8, v[u].y & 0xFF) : 0u;
            }
        }
    }
    {
        const uint32_t hw = (__ballot(hard & 1u) ? 1u : 0u) | (__ballot(hard & 2u) ? 2u : 0u) |
                           (__ballot(hard & 4u) ? 4u : 0u);
        if ((hw & ~seen) && lane == 0)
            atomicOr(w.sum, hw);
    }
}

// ObjectManager::replaySegment's checksum checks on the walk records of the
// segments that passed the metadata check:
//   OBJ          computed object CRC (left in d.out[i] by the scan kernels) vs.
//                Object::Header::checksum, the payload's first 4 B
//                (src/ObjectManager.cc:659-669);
//   OBJTOMB      ObjectTombstone::checkIntegrity (src/ObjectManager.cc:752-758,
//                src/Object.cc:1014-1057): CRC of header bytes [0, 28) and the
//                key [32, len) vs. the checksum at [28, 32);
//   SAFEVERSION  ObjectSafeVersion::checkIntegrity (src/ObjectManager.cc:873-880,
//                src/Object.cc:1107-1143): CRC of [0, 8) vs. the checksum at [8, 12);
//   PREP         PreparedOp::checkIntegrity (src/ObjectManager.cc:956,
//                src/PreparedOp.cc:177-190): its 32-byte header up to the
//                checksum, [0, 28), then Object::applyChecksum of the object at
//                32, i.e. [36, len); checksum at [28, 32);
//   PREPTOMB     PreparedOpTombstone::checkIntegrity (src/ObjectManager.cc:1013,
//                src/PreparedOp.cc:271-282): [0, 40) vs. [40, 44);
//   TXDECISION   TxDecisionRecord::checkIntegrity (src/ObjectManager.cc:1060,
//                src/TxDecisionRecord.cc:209-223): [0, 44) and the uint32
//                24 * participantCount (at [36, 40)) bytes from 48, clipped to
//                the entry as Buffer::Iterator clips; checksum at [44, 48);
//   TXPLIST      ParticipantList::checkIntegrity (src/ObjectManager.cc:1084,
//                src/ParticipantList.cc:96-110): [0, 20) and 24 * count (at
//                [16, 20)) bytes from 24; checksum at [20, 24).  A list longer
//                than the entry fails: the reference's getRange returns NULL.
// All but OBJ are rare, and short apart from a prepared op's object, so one
// thread runs the byte-table CRC over each and writes it to d.out[i].
// Records shorter than their type's header, or unreadable, count as failures.
__device__ __forceinline__ uint32_t crc_bytes_g(const uint32_t* t1, uint32_t c, const gu8* p,
                                                uint32_t n)
{
    for (uint32_t k = 0; k < n; k++)
        c = t1[(c ^ p[k]) & 0xFF] ^ (c >> 8);
    return c;
}

__device__ __forceinline__ uint32_t le32_g(const gu8* p)
{
    return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}


// nother (nullable): the binning count of records this kernel has work for
// (replay_other); 0 ends the launch at once.  Grid-stride over the records.
__device__ __forceinline__ void obj_compare_one(const BatchDesc& d, ramcrc_seg_status* status,
                                                uint64_t i);

__global__ __launch_bounds__(256) void k_obj_compare(BatchDesc d, ramcrc_seg_status* status,
                                                     const uint32_t* nother)
{
    if (nother && *nother == 0)
        return;
    const uint64_t n = entry_count<kRecords>(d);
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += uint64_t(gridDim.x) * blockDim.x)
        obj_compare_one(d, status, i);
}

__device__ __forceinline__ void obj_compare_one(const BatchDesc& d, ramcrc_seg_status* status,
                                                uint64_t i)
{
    const u32x4 r = d.rec[i];
    const uint32_t type = r.w & 0x3f;
    const uint32_t hdr = replay_header_bytes(type);
    if (hdr == 0)
        return;
    const bool readable = r.z >= hdr && !(r.w & kRecOverlong);
    if (d.vstat && type == RAMCRC_LOG_ENTRY_TYPE_OBJ && readable && !is_large(uint64_t(r.z) - 4))
        return;   // compared beside the scan (k_entries, below the 64 KiB split)
    const uint64_t payload = reinterpret_cast<uint64_t>(d.base) + uint64_t(r.x) * d.seg_bytes +
                             r.y + 1 + ((r.w >> 6) & 3) + 1;
    const gu8* p = reinterpret_cast<const gu8*>(payload);
    // The segment's status, the stored object checksum and the computed CRC
    // are independent loads: issue them together (one memory round trip, not
    // two).  Readable records lie inside their segment, so the object header
    // read is in bounds.
    const uint32_t seg_flags = d.seg_status[r.x].x;
    uint32_t stored = 0, computed = 0;
    if (type == RAMCRC_LOG_ENTRY_TYPE_OBJ && readable) {
        stored = le32_g(p);
        computed = d.out[i];
    }
    if (!(seg_flags & RAMCRC_SEG_OK))
        return;
    bool ok = false;
    if (readable) {
        if (type == RAMCRC_LOG_ENTRY_TYPE_OBJ) {
            ok = computed == stored;
        } else {
            // CRC of [0, at) then of [from, from + tail); stored checksum at [at, at + 4)
            uint32_t at = hdr - 4, from = hdr, tail = 0;
            bool fits = true;
            switch (type) {
            case RAMCRC_LOG_ENTRY_TYPE_OBJTOMB: tail = r.z - hdr; break;
            case RAMCRC_LOG_ENTRY_TYPE_PREP:
                at = kPrepHeaderBytes - 4;
                from = kPrepHeaderBytes + 4;
                tail = r.z - from;
                break;
            case RAMCRC_LOG_ENTRY_TYPE_TXDECISION:
                tail = min(24u * le32_g(p + 36), r.z - hdr);
                break;
            case RAMCRC_LOG_ENTRY_TYPE_TXPLIST:
                tail = 24u * le32_g(p + 16);
                fits = tail <= r.z - hdr;
                break;
            default: break;
            }
            if (fits) {
                const uint32_t* t1 = &g_tab.pos[1 + kTinyRow0][0];   // X^1(b): the byte step
                const uint32_t c = ~crc_bytes_g(t1, crc_bytes_g(t1, 0xFFFFFFFFu, p, at), p + from, tail);
                d.out[i] = c;
                ok = c == le32_g(p + at);
            }
        }
    }
    if (!ok)
        atomicAdd(&status[r.x].bad_objects, 1u);
}

// Object::assembleForLog (src/Object.cc:213-238): header.checksum =
// computeChecksum(), i.e. the finalized CRC of bytes [4, len) the scan
// kernels left in d.out[i], stored little-endian into the object's first 4
// bytes (which no object's checksum range covers).  Byte stores: objects are
// packed back to back in a log, so headers are unaligned.
__global__ __launch_bounds__(256) void k_obj_stamp(BatchDesc d)
{
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= d.n)
        return;
    if (d.len[i] < kObjHeaderBytes) {
        d.out[i] = 0;
        return;
    }
    const uint32_t c = d.out[i];
    uint8_t* p = const_cast<uint8_t*>(d.base) + d.off[i];
    p[0] = uint8_t(c);
    p[1] = uint8_t(c >> 8);
    p[2] = uint8_t(c >> 16);
    p[3] = uint8_t(c >> 24);
}

// ramcrc_segments_certify_device: the walk's certificates are {head, 0}, so
// the walk stops at each segment's head and its status carries the running
// metadata checksum finished over the 4 head bytes -- exactly
// Segment::getAppendedLength's certificate (src/Segment.cc:672-684) when the
// entries end at the head.
__global__ __launch_bounds__(256) void k_cert_prep(const uint32_t* heads, ramcrc_seg_cert* certs,
                                                   uint64_t n)
{
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n)
        certs[i] = ramcrc_seg_cert{heads[i], 0u};
}

__global__ __launch_bounds__(256) void k_cert_emit(const ramcrc_seg_cert* tmp,
                                                   const ramcrc_seg_status* st,
                                                   ramcrc_seg_cert* certs, uint32_t* flags, uint64_t n)
{
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const ramcrc_seg_status s = st[i];
    certs[i] = ramcrc_seg_cert{tmp[i].segment_length, s.checksum};
    if (flags) {
        // the walk's checksum test is against the placeholder 0: only its
        // structural findings matter here
        const uint32_t bad = s.flags & (RAMCRC_SEG_PAST_CAPACITY | RAMCRC_SEG_PAST_LENGTH |
                                        RAMCRC_SEG_CYCLE);
        flags[i] = bad ? bad : RAMCRC_SEG_OK;
    }
}

}  // namespace

extern "C" {

int ramcrc_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n;
}

int ramcrc_last_hip_error(void) { return t_last_hip; }

const char* ramcrc_strerror(int code)
{
    switch (code) {
    case RAMCRC_OK: return "ok";
    case RAMCRC_EINVAL: return "invalid argument";
    case RAMCRC_ENOMEM: return "out of memory";
    case RAMCRC_EHIP: return hipGetErrorString(hipError_t(t_last_hip));
    case RAMCRC_ENODEV: return "no usable device";
    case RAMCRC_ERCCL: return "rccl failure";
    case RAMCRC_EREFUSED: return "launch refused: chunk scratch too small (ramcrc_ctx_reserve)";
    case RAMCRC_EINTERNAL: return "launch refused: inconsistent small-entry bin layout";
    case RAMCRC_EPEER: return "another rank of the shard failed this step";
    default: return "unknown error";
    }
}

#ifndef RAMCRC_SRC_SHA
#define RAMCRC_SRC_SHA "unknown"
#endif
#define RAMCRC_STR2(x) #x
#define RAMCRC_STR(x) RAMCRC_STR2(x)

// Probe builds only: copies k_entries' phase stamps (RAMCRC_STAMPS) to host
// memory; RAMCRC_EINVAL in product builds.  Not part of the C ABI header.
int ramcrc_debug_stamps(void* out, uint64_t bytes)
{
#if RAMCRC_STAMPS
    if (bytes > sizeof(g_stamps))
        bytes = sizeof(g_stamps);
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), bytes) == hipSuccess ? RAMCRC_OK : RAMCRC_EHIP;
#else
    (void)out;
    (void)bytes;
    return RAMCRC_EINVAL;
#endif
}

const char* ramcrc_build_info(void)
{
    // src_sha: sha256 of the sources the library was built from (build.py),
    // the same marker build.py reads back to decide staleness
    return "ramcrc gfx950 src_sha=" RAMCRC_SRC_SHA
           " chunk=" RAMCRC_STR(RAMCRC_CHUNK_SHIFT) "..20 (adaptive: largest giving every wave two chunks)"
           " block=1KiB waves/WG=16 unroll=" RAMCRC_STR(RAMCRC_UNROLL)
           " lds_chunks=" RAMCRC_STR(RAMCRC_LDS_CHUNKS) " lds_entries=" RAMCRC_STR(RAMCRC_LDS_ENTRIES)
           " entries: waves=" RAMCRC_STR(RAMCRC_ENT_WAVES) " smallk=" RAMCRC_STR(RAMCRC_SMALLK)
           " pu=" RAMCRC_STR(RAMCRC_PU) " tiny_cf=" RAMCRC_STR(RAMCRC_TINY_CF)
           " large_min=64KiB part_shift=" RAMCRC_STR(RAMCRC_PART_SHIFT);
}

int ramcrc_ctx_create(int device, ramcrc_ctx** out)
{
    if (!out)
        return RAMCRC_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return RAMCRC_ENODEV;
    DeviceGuard g(device);
    if (!g.ok)
        return RAMCRC_ENODEV;
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        fprintf(stderr, "ramcrc: device %d is %s, this build targets gfx950 only\n", device,
                prop.gcnArchName);
        return RAMCRC_ENODEV;
    }
    ramcrc_ctx* c = new (std::nothrow) ramcrc_ctx();
    if (!c)
        return RAMCRC_ENOMEM;
    c->device = device;
    c->ncu = prop.multiProcessorCount;
    c->ncu_all = c->ncu;
    if (hipMalloc(reinterpret_cast<void**>(&c->status), 16) != hipSuccess) {
        delete c;
        return RAMCRC_ENOMEM;
    }
    (void)hipMemset(c->status, 0, 16);
    if (hipMalloc(reinterpret_cast<void**>(&c->bins), sizeof(BinTable)) != hipSuccess) {
        ramcrc_ctx_destroy(c);
        return RAMCRC_ENOMEM;
    }
    (void)hipMemset(c->bins, 0, sizeof(BinTable));   // hist must start at zero
    *out = c;
    return RAMCRC_OK;
}

int ramcrc_ctx_destroy(ramcrc_ctx* c)
{
    if (!c)
        return RAMCRC_OK;
    DeviceGuard g(c->device);
    (void)hipDeviceSynchronize();
    if (c->partials) (void)hipFree(c->partials);
    if (c->plan_local) (void)hipFree(c->plan_local);
    if (c->group_pref) (void)hipFree(c->group_pref);
    if (c->status) (void)hipFree(c->status);
    if (c->bins) (void)hipFree(c->bins);
    if (c->sdesc) (void)hipFree(c->sdesc);
    if (c->sidx) (void)hipFree(c->sidx);
    if (c->sinit) (void)hipFree(c->sinit);
    if (c->obj_out) (void)hipFree(c->obj_out);
    if (c->cert_scratch) (void)hipFree(c->cert_scratch);
    if (c->walk_parts) (void)hipFree(c->walk_parts);
    if (c->walk_fallback) (void)hipFree(c->walk_fallback);
    if (c->walk_base) (void)hipFree(c->walk_base);
    if (c->walk_recs) (void)hipFree(c->walk_recs);
    if (c->walk_pool) (void)hipFree(c->walk_pool);
    if (c->walk_pool_owner) (void)hipFree(c->walk_pool_owner);
    if (c->walk_blocks) (void)hipFree(c->walk_blocks);
    if (c->walk_pool_used) (void)hipFree(c->walk_pool_used);
    if (c->walk_sum) (void)hipFree(c->walk_sum);
    if (c->d_stage) (void)hipFree(c->d_stage);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    if (c->compute_stream) (void)hipStreamDestroy(c->compute_stream);
    for (auto& ev : c->ev_used) {
        (void)hipEventDestroy(ev.first);
        (void)hipEventDestroy(ev.second);
    }
    for (auto& ev : c->ev_free) {
        (void)hipEventDestroy(ev.first);
        (void)hipEventDestroy(ev.second);
    }
    delete c;
    return RAMCRC_OK;
}

int ramcrc_ctx_reserve(ramcrc_ctx* c, uint64_t max_chunks, uint64_t max_entries)
{
    if (!c)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    return reserve_locked(c, max_chunks, max_entries);
}

int ramcrc_ctx_set_option(ramcrc_ctx* c, int option, int64_t value)
{
    if (!c)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    switch (option) {
    case RAMCRC_OPT_SERIAL_WALK: c->serial_walk = value != 0; return RAMCRC_OK;
    case RAMCRC_OPT_TEST_FAIL_AFTER_COUNT:
        if (value < 0 || value > 1000)
            return RAMCRC_EINVAL;
        c->fail_after_count = int(value);
        return RAMCRC_OK;
    case RAMCRC_OPT_TEST_DIRTY_BINS:
        if (value < 0 || value > 0xFFFFFFFFll)
            return RAMCRC_EINVAL;
        c->dirty_bins = uint32_t(value);
        return RAMCRC_OK;
    case RAMCRC_OPT_TEST_BIN_STRAGGLER:
        c->bin_straggler = value != 0;
        return RAMCRC_OK;
    case RAMCRC_OPT_WALK_PART_SHIFT:
        if (value != 0 && (value < kPartShiftMin || value > 20))
            return RAMCRC_EINVAL;
        c->walk_pshift = uint32_t(value);
        return RAMCRC_OK;
    default: return RAMCRC_EINVAL;
    }
}

int ramcrc_ctx_set_timing(ramcrc_ctx* c, int enable)
{
    if (!c)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    c->timing = enable != 0;
    return RAMCRC_OK;
}

int ramcrc_stream_create_cu_mask(int device, const uint32_t* cu_mask, uint32_t mask_words,
                                 void** out_stream)
{
    if (!cu_mask || !out_stream || mask_words == 0 || mask_words > 8)
        return RAMCRC_EINVAL;
    DeviceGuard g(device);
    if (!g.ok)
        return RAMCRC_ENODEV;
    hipStream_t st = nullptr;
    HIPCHK(hipExtStreamCreateWithCUMask(&st, mask_words, cu_mask));
    *out_stream = st;
    return RAMCRC_OK;
}

int ramcrc_stream_destroy(void* stream)
{
    if (!stream)
        return RAMCRC_EINVAL;
    HIPCHK(hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)));
    return RAMCRC_OK;
}

int ramcrc_ctx_set_cus(ramcrc_ctx* c, int ncu)
{
    if (!c || ncu < 0)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if (ncu == 0 || ncu > c->ncu_all)
        ncu = c->ncu_all;
    c->ncu = ncu;
    return RAMCRC_OK;
}

int ramcrc_ctx_scan_time(ramcrc_ctx* c, double* total_ms, uint64_t* launches)
{
    if (!c)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    double sum = 0;
    uint64_t cnt = 0;
    for (auto& ev : c->ev_used) {
        HIPCHK(hipEventSynchronize(ev.second));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ev.first, ev.second));
        sum += ms;
        cnt++;
        c->ev_free.push_back(ev);
    }
    c->ev_used.clear();
    if (total_ms)
        *total_ms = sum;
    if (launches)
        *launches = cnt;
    return RAMCRC_OK;
}

int ramcrc_ctx_debug_bins(ramcrc_ctx* c, uint64_t* host, uint64_t nwords, uint32_t* par_next)
{
    if (!c || !host)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    HIPCHK(hipDeviceSynchronize());
    // count[kNB], then cursor[0][kNB], cursor[1][kNB], then hist[0], hist[1] (as uint64)
    std::vector<uint64_t> v;
    BinTable h;
    HIPCHK(hipMemcpy(&h, c->bins, sizeof(BinTable), hipMemcpyDeviceToHost));
    for (int b = 0; b < kNB; b++) v.push_back(h.count[b]);
    for (int p = 0; p < 2; p++)
        for (int b = 0; b < kNB; b++) v.push_back(h.ctr[p].cursor[b]);
    for (int p = 0; p < 2; p++)
        for (int b = 0; b < kNB; b++) v.push_back(h.ctr[p].hist[b]);
    v.push_back(h.rescues);
    for (uint64_t i = 0; i < nwords && i < v.size(); i++)
        host[i] = v[i];
    if (par_next)
        *par_next = c->bin_par;
    return RAMCRC_OK;
}

int ramcrc_ctx_status(ramcrc_ctx* c, uint32_t* status)
{
    if (!c || !status)
        return RAMCRC_EINVAL;
    DeviceGuard g(c->device);
    HIPCHK(hipMemcpy(status, c->status, sizeof(uint32_t), hipMemcpyDeviceToHost));
    return RAMCRC_OK;
}

int ramcrc_ctx_check(ramcrc_ctx* c, void* stream)
{
    if (!c)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    HIPCHK(hipStreamSynchronize(s));
    uint32_t st = 0;
    HIPCHK(hipMemcpy(&st, c->status, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (!(st & kStatusSticky))
        return RAMCRC_OK;
    // take the sticky bits with one device atomic: a bit another stream's
    // launch sets meanwhile is either taken here or stays for the next check
    hipLaunchKernelGGL(k_status_take, dim3(1), dim3(1), 0, s, c->status);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipMemcpy(&st, c->status + 1, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (st & kStatusBins)
        return RAMCRC_EINTERNAL;
    return (st & kStatusSticky) ? RAMCRC_EREFUSED : RAMCRC_OK;
}

int ramcrc_segments_device(ramcrc_ctx* c, const void* d_base, uint64_t seg_bytes, uint64_t nseg,
                           const uint32_t* d_init, uint32_t* d_out, uint32_t flags, void* stream)
{
    if (!c || !d_out || (!d_base && nseg && seg_bytes))
        return RAMCRC_EINVAL;
    if (nseg == 0)
        return RAMCRC_OK;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    BatchDesc d{};
    d.cshift = kChunkShift;
    d.base = static_cast<const uint8_t*>(d_base);
    d.seg_bytes = seg_bytes;
    d.n = nseg;
    d.init = d_init;
    d.out = d_out;
    d.flags = flags;
    if (seg_bytes < kLargeMin) {
        return launch_binned<kSegUniform>(c, d, s, 0);
    }
    const uint64_t B = reinterpret_cast<uint64_t>(d_base);
    if ((B % kChunk) == 0 && (seg_bytes % kChunk) == 0) {
        // The recovery-scan fast path: no plan, chunk g -> (g / per, g % per).
        // Largest chunk (256 KiB .. 1 MiB) that still gives every wave two
        // chunks: fewer per-chunk pipeline drains and folds.
        const uint64_t waves = uint64_t(c->ncu) * kWavesPerGroup;
        uint32_t shift = kChunkShift;
        while (shift < 20 && (B % (2ull << shift)) == 0 && (seg_bytes % (2ull << shift)) == 0 &&
               (seg_bytes >> (shift + 1)) * nseg >= 2 * waves)
            shift++;
        d.cshift = shift;
        const uint64_t per = seg_bytes >> shift;
        int rc = reserve_locked(c, per * nseg, 1);
        if (rc)
            return rc;
        Plan pl = make_plan(c, 0);
        {
            ScanTimer t(c, s);
            t.launch(k_chunks<kSegAligned>, dim3(c->ncu), dim3(kThreads), d, pl, per);
        }
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL((k_combine<kSegAligned, false>), dim3((nseg + 3) / 4), dim3(256), 0, s,
                           d, pl, per);
        HIPCHK(hipGetLastError());
        return RAMCRC_OK;
    }
    int rc = reserve_locked(c, nseg * (seg_bytes / kChunk + 2) + 16, nseg);
    if (rc)
        return rc;
    return launch_planned<kSegUniform>(c, d, s);
}

int ramcrc_batch_device(ramcrc_ctx* c, const void* d_base, const uint64_t* d_off,
                        const uint64_t* d_len, const uint32_t* d_init, uint32_t* d_out, uint64_t n,
                        uint32_t flags, void* stream)
{
    if (n == 0)
        return c ? RAMCRC_OK : RAMCRC_EINVAL;
    if (!c || !d_out || !d_off || !d_len || !d_base)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    int rc = reserve_locked(c, default_chunk_bound(n), n);
    if (rc)
        return rc;
    BatchDesc d{};
    d.cshift = kChunkShift;
    d.base = static_cast<const uint8_t*>(d_base);
    d.off = d_off;
    d.len = d_len;
    d.n = n;
    d.init = d_init;
    d.out = d_out;
    d.flags = flags;
    return launch_planned<kTable>(c, d, reinterpret_cast<hipStream_t>(stream));
}

int ramcrc_entries_device(ramcrc_ctx* c, const void* d_base, const uint64_t* d_off,
                          const uint64_t* d_len, const uint32_t* d_init, uint32_t* d_out, uint64_t n,
                          uint32_t flags, void* stream)
{
    if (n == 0)
        return c ? RAMCRC_OK : RAMCRC_EINVAL;
    if (!c || !d_out || !d_off || !d_len || !d_base)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    BatchDesc d{};
    d.cshift = kChunkShift;
    d.base = static_cast<const uint8_t*>(d_base);
    d.off = d_off;
    d.len = d_len;
    d.n = n;
    d.init = d_init;
    d.out = d_out;
    d.flags = flags;
    return launch_binned<kTable>(c, d, s, 0);
}

int ramcrc_batch_host(ramcrc_ctx* c, const void* const* ptrs, const uint64_t* lens,
                      const uint32_t* init, uint32_t* out, uint64_t n, uint32_t flags)
{
    if (!c || (n && (!ptrs || !lens || !out)))
        return RAMCRC_EINVAL;
    if (n == 0)
        return RAMCRC_OK;
    // The context lock is held from sizing the staging buffers to the final
    // synchronize: another thread on this context must not free or refill
    // them while they are being copied from.
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    // Pack every buffer 16-byte aligned into one pinned staging area, then one
    // H2D copy, one batch launch, one D2H copy.
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (lens[i] && !ptrs[i])
            return RAMCRC_EINVAL;
        total += (lens[i] + 15) & ~uint64_t(15);
    }
    const uint64_t meta = n * (2 * sizeof(uint64_t) + 2 * sizeof(uint32_t));
    const uint64_t need = total + meta + 64;
    if (c->h_stage_cap < need) {
        if (c->h_stage) (void)hipHostFree(c->h_stage);
        c->h_stage = nullptr;
        c->h_stage_cap = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&c->h_stage), need, hipHostMallocDefault) !=
            hipSuccess)
            return RAMCRC_ENOMEM;
        c->h_stage_cap = need;
    }
    if (c->d_stage_cap < need) {
        if (c->d_stage) (void)hipFree(c->d_stage);
        c->d_stage = nullptr;
        c->d_stage_cap = 0;
        if (hipMalloc(reinterpret_cast<void**>(&c->d_stage), need) != hipSuccess)
            return RAMCRC_ENOMEM;
        c->d_stage_cap = need;
    }
    if (!c->copy_stream)
        HIPCHK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    uint8_t* h = c->h_stage;
    uint64_t* h_off = reinterpret_cast<uint64_t*>(h + total);
    uint64_t* h_len = h_off + n;
    uint32_t* h_init = reinterpret_cast<uint32_t*>(h_len + n);
    uint32_t* h_out = h_init + n;
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (lens[i])
            memcpy(h + pos, ptrs[i], lens[i]);
        h_off[i] = pos;
        h_len[i] = lens[i];
        h_init[i] = init ? init[i] : 0xFFFFFFFFu;
        pos += (lens[i] + 15) & ~uint64_t(15);
    }
    uint8_t* d = c->d_stage;
    hipStream_t s = c->copy_stream;
    const uint64_t in_bytes = total + n * (2 * sizeof(uint64_t) + sizeof(uint32_t));
    HIPCHK(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, s));
    uint64_t* d_off = reinterpret_cast<uint64_t*>(d + total);
    uint64_t* d_len = d_off + n;
    uint32_t* d_init = reinterpret_cast<uint32_t*>(d_len + n);
    uint32_t* d_out = d_init + n;
    int rc = ramcrc_batch_device(c, d, d_off, d_len, d_init, d_out, n, flags, s);
    if (rc) {
        (void)hipStreamSynchronize(s);   // the H2D copy reads h_stage
        return rc;
    }
    HIPCHK(hipMemcpyAsync(h_out, d_out, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    rc = ramcrc_ctx_check(c, s);   // synchronizes s; a refused launch wrote nothing
    if (rc)
        return rc;
    memcpy(out, h_out, n * sizeof(uint32_t));
    return RAMCRC_OK;
}

int ramcrc_stream_host(ramcrc_ctx* c, const void* h_base, uint64_t seg_bytes, uint64_t nseg,
                       uint32_t* h_out, uint32_t flags, int batch, int depth)
{
    if (!c || !h_base || !h_out || batch < 1 || depth < 1 || seg_bytes == 0)
        return RAMCRC_EINVAL;
    if (nseg == 0)
        return RAMCRC_OK;
    std::lock_guard<std::recursive_mutex> lk(c->mu);   // held until both streams drained
    DeviceGuard g(c->device);
    if (depth > 8)
        depth = 8;
    const uint64_t slot_bytes = uint64_t(batch) * seg_bytes;
    // Each slot: batch*seg_bytes of data + batch CRCs.
    const uint64_t slot_stride = (slot_bytes + 4 * uint64_t(batch) + 4095) & ~uint64_t(4095);
    const uint64_t need = slot_stride * uint64_t(depth);
    if (c->d_stage_cap < need) {
        if (c->d_stage) (void)hipFree(c->d_stage);
        c->d_stage = nullptr;
        c->d_stage_cap = 0;
        if (hipMalloc(reinterpret_cast<void**>(&c->d_stage), need) != hipSuccess)
            return RAMCRC_ENOMEM;
        c->d_stage_cap = need;
    }
    if (!c->copy_stream)
        HIPCHK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    if (!c->compute_stream)
        HIPCHK(hipStreamCreateWithFlags(&c->compute_stream, hipStreamNonBlocking));
    hipEvent_t copied[8] = {}, done[8] = {};
    int rc = RAMCRC_OK;
    auto hip = [&](hipError_t e) {
        if (e != hipSuccess && rc == RAMCRC_OK) {
            t_last_hip = int(e);
            rc = RAMCRC_EHIP;
        }
        return rc == RAMCRC_OK;
    };
    for (int k = 0; k < depth && rc == RAMCRC_OK; k++) {
        hip(hipEventCreateWithFlags(&copied[k], hipEventDisableTiming));
        hip(hipEventCreateWithFlags(&done[k], hipEventDisableTiming));
    }
    const uint8_t* src = static_cast<const uint8_t*>(h_base);
    const uint64_t nb = (nseg + batch - 1) / batch;
    // On any failure the loop stops issuing; the streams are drained below
    // before the events are destroyed and before returning, so no copy into
    // h_out or out of h_base is still in flight when the call returns.
    for (uint64_t b = 0; b < nb && rc == RAMCRC_OK; b++) {
        const int k = int(b % depth);
        const uint64_t first = b * batch;
        const uint64_t cnt = (nseg - first) < uint64_t(batch) ? (nseg - first) : uint64_t(batch);
        uint8_t* slot = c->d_stage + uint64_t(k) * slot_stride;
        uint32_t* slot_out = reinterpret_cast<uint32_t*>(slot + slot_bytes);
        if (b >= uint64_t(depth) && !hip(hipStreamWaitEvent(c->copy_stream, done[k], 0)))
            break;
        if (!hip(hipMemcpyAsync(slot, src + first * seg_bytes, cnt * seg_bytes,
                                hipMemcpyHostToDevice, c->copy_stream)) ||
            !hip(hipEventRecord(copied[k], c->copy_stream)) ||
            !hip(hipStreamWaitEvent(c->compute_stream, copied[k], 0)))
            break;
        rc = ramcrc_segments_device(c, slot, seg_bytes, cnt, nullptr, slot_out, flags,
                                    c->compute_stream);
        if (rc)
            break;
        if (!hip(hipMemcpyAsync(h_out + first, slot_out, cnt * sizeof(uint32_t),
                                hipMemcpyDeviceToHost, c->compute_stream)) ||
            !hip(hipEventRecord(done[k], c->compute_stream)))
            break;
    }
    hip(hipStreamSynchronize(c->compute_stream));
    hip(hipStreamSynchronize(c->copy_stream));
    for (int k = 0; k < depth; k++) {
        if (copied[k]) (void)hipEventDestroy(copied[k]);
        if (done[k]) (void)hipEventDestroy(done[k]);
    }
    return rc;
}


namespace {
int walk_impl(ramcrc_ctx* c, const void* d_base, uint64_t seg_stride, uint32_t seg_capacity,
              uint64_t n_seg, const ramcrc_seg_cert* d_certs, ramcrc_seg_status* d_status,
              ramcrc_seg_entry* d_entries, uint64_t entries_cap, uint64_t* d_n_entries,
              hipStream_t s, uint32_t* sum);
int verify_impl(ramcrc_ctx* c, const void* d_base, uint64_t seg_stride,
                const ramcrc_seg_entry* d_entries, uint64_t entries_cap, const uint64_t* d_n_entries,
                uint32_t* d_obj_crc, ramcrc_seg_status* d_status, hipStream_t s, const uint32_t* sum);
}  // namespace

int ramcrc_segment_walk_device(ramcrc_ctx* c, const void* d_base, uint64_t seg_stride,
                               uint32_t seg_capacity, uint64_t n_seg,
                               const ramcrc_seg_cert* d_certs, ramcrc_seg_status* d_status,
                               ramcrc_seg_entry* d_entries, uint64_t entries_cap,
                               uint64_t* d_n_entries, void* stream)
{
    if (!c)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    return walk_impl(c, d_base, seg_stride, seg_capacity, n_seg, d_certs, d_status, d_entries,
                     entries_cap, d_n_entries, reinterpret_cast<hipStream_t>(stream), nullptr);
}

int ramcrc_replay_verify_device(ramcrc_ctx* c, const void* d_base, uint64_t seg_stride,
                                uint32_t seg_capacity, uint64_t n_seg, const ramcrc_seg_cert* d_certs,
                                ramcrc_seg_status* d_status, ramcrc_seg_entry* d_entries,
                                uint64_t entries_cap, uint64_t* d_n_entries, uint32_t* d_obj_crc,
                                void* stream)
{
    if (!c)
        return RAMCRC_EINVAL;
    if (entries_cap && !d_obj_crc)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc = grow_device(reinterpret_cast<void**>(&c->walk_sum), &c->walk_sum_cap, 4, sizeof(uint32_t));
    if (rc)
        return rc;
    rc = walk_impl(c, d_base, seg_stride, seg_capacity, n_seg, d_certs, d_status, d_entries,
                   entries_cap, d_n_entries, s, c->walk_sum);
    if (rc || n_seg == 0)
        return rc;
    return verify_impl(c, d_base, seg_stride, d_entries, entries_cap, d_n_entries, d_obj_crc,
                       d_status, s, c->walk_sum);
}

namespace {
int walk_impl(ramcrc_ctx* c, const void* d_base, uint64_t seg_stride, uint32_t seg_capacity,
              uint64_t n_seg, const ramcrc_seg_cert* d_certs, ramcrc_seg_status* d_status,
              ramcrc_seg_entry* d_entries, uint64_t entries_cap, uint64_t* d_n_entries,
              hipStream_t s, uint32_t* sum)
{
    if (!d_n_entries || (entries_cap && !d_entries))
        return RAMCRC_EINVAL;
    if (n_seg && (!d_base || !d_certs || !d_status))
        return RAMCRC_EINVAL;
    if ((reinterpret_cast<uintptr_t>(d_base) & 15) || (seg_stride & 15) || (seg_capacity & 15) ||
        n_seg > 0xFFFFFFFFull || (n_seg > 1 && seg_stride < seg_capacity))
        return RAMCRC_EINVAL;
    if (n_seg == 0 || c->serial_walk) {
        // (the parallel walk's k_walk_probe zeroes these)
        HIPCHK(hipMemsetAsync(d_n_entries, 0, sizeof(uint64_t), s));
        if (sum)
            HIPCHK(hipMemsetAsync(sum, 0, sizeof(uint32_t), s));
    }
    if (n_seg == 0)
        return RAMCRC_OK;
    WalkDesc w{};
    w.base = static_cast<const uint8_t*>(d_base);
    w.stride = seg_stride;
    w.capacity = seg_capacity;
    w.nseg = n_seg;
    w.certs = d_certs;
    w.status = d_status;
    w.entries = reinterpret_cast<u32x4*>(d_entries);
    w.cap = entries_cap;
    w.n_entries = reinterpret_cast<unsigned long long*>(d_n_entries);
    w.only = nullptr;
    w.sum = sum;
    {
        int rc0 = grow_device(reinterpret_cast<void**>(&c->walk_base), &c->walk_base_cap, n_seg,
                              sizeof(uint64_t));
        if (rc0)
            return rc0;
    }
    w.seg_base = c->walk_base;   // every segment's first record slot (both walkers)
    uint64_t grid = n_seg;
    if (grid > uint64_t(64) * c->ncu)
        grid = uint64_t(64) * c->ncu;
    if (!c->serial_walk) {
        // parallel walk: sync search, part walks, per-segment fix-up, record
        // emission; the serial walker then takes only the segments the fix-up
        // handed back (uint32_t wraps, exhausted re-walk budget)
        // part size: chosen per batch on the device by k_walk_probe from the
        // entry density (or forced, RAMCRC_OPT_WALK_PART_SHIFT); grids and
        // scratch are sized for the smallest part it may choose
        const uint32_t pshift = c->walk_pshift ? c->walk_pshift : kPartShift;
        const uint32_t nparts = uint32_t((uint64_t(seg_capacity) + (1ull << pshift) - 1) >> pshift);
        const uint64_t total = n_seg * uint64_t(nparts);
        int rc = grow_device(&c->walk_parts, &c->walk_parts_cap, total, sizeof(PartRes));
        if (!rc)
            rc = grow_device(reinterpret_cast<void**>(&c->walk_fallback), &c->walk_fallback_cap,
                             n_seg, sizeof(uint32_t));
        if (!rc)
            rc = grow_device(&c->walk_recs, &c->walk_recs_cap, total * kPartRec, sizeof(uint2));
        // the pool holds A's records past each part's first block: sized for
        // entries of 96 B on average (denser parts than that, and records past
        // entries_cap, fall back to C's second walk of the part)
        uint64_t pool_blocks = (n_seg * uint64_t(seg_capacity) / 96) / kPartRec + 1;
        const uint64_t cap_blocks = entries_cap / kPartRec + 1;
        pool_blocks = pool_blocks < cap_blocks ? pool_blocks : cap_blocks;
        if (!rc)
            rc = grow_device(&c->walk_pool, &c->walk_pool_cap, pool_blocks * kPartRec, sizeof(uint2));
        if (!rc)
            rc = grow_device(reinterpret_cast<void**>(&c->walk_pool_owner), &c->walk_pool_owner_cap,
                             pool_blocks, sizeof(uint32_t));
        if (!rc)
            rc = grow_device(reinterpret_cast<void**>(&c->walk_blocks), &c->walk_blocks_cap,
                             total * kMaxBlocks, sizeof(uint32_t));
        if (!rc)
            rc = grow_device(reinterpret_cast<void**>(&c->walk_pool_used), &c->walk_pool_used_cap, 2,
                             sizeof(unsigned long long));   // [1]: the part shift word
        if (rc)
            return rc;
        PWalk pw{};
        pw.base = w.base;
        pw.stride = seg_stride;
        pw.capacity = seg_capacity;
        pw.nparts = nparts;
        pw.nseg = n_seg;
        pw.certs = d_certs;
        pw.status = d_status;
        pw.entries = w.entries;
        pw.cap = entries_cap;
        pw.n_entries = w.n_entries;
        pw.parts = static_cast<PartRes*>(c->walk_parts);
        pw.fallback = c->walk_fallback;
        pw.seg_base = c->walk_base;
        pw.recs = static_cast<uint2*>(c->walk_recs);
        pw.pshift = pshift;
        uint32_t* geo = reinterpret_cast<uint32_t*>(c->walk_pool_used + 1);
        pw.geo = geo;
        pw.pool = static_cast<uint2*>(c->walk_pool);
        pw.pool_owner = c->walk_pool_owner;
        pw.blocks = c->walk_blocks;
        pw.pool_used = c->walk_pool_used;
        pw.pool_cap = pool_blocks;
        pw.sum = sum;
        hipLaunchKernelGGL(k_walk_probe, dim3(1), dim3(kWaveSize), 0, s, pw, c->walk_pshift, geo);
        HIPCHK(hipGetLastError());
        if (nparts > 1) {
            uint64_t g0 = (total + kSyncWaves - 1) / kSyncWaves;
            if (g0 > uint64_t(8) * c->ncu)
                g0 = uint64_t(8) * c->ncu;
            hipLaunchKernelGGL(k_walk_sync, dim3(g0), dim3(kSyncWaves * kWaveSize), 0, s, pw);
            HIPCHK(hipGetLastError());
        }
        hipLaunchKernelGGL(k_walk_parts, dim3((total + 255) / 256), dim3(256), 0, s, pw);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_walk_fix, dim3(grid), dim3(kWaveSize), 0, s, pw);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_walk_emit, dim3((total + 255) / 256), dim3(256), 0, s, pw);
        HIPCHK(hipGetLastError());
        uint64_t gc = (total + pool_blocks + 4 * kCopyU - 1) / (4 * kCopyU);   // kCopyU blocks per wave
        if (gc > uint64_t(32) * c->ncu)
            gc = uint64_t(32) * c->ncu;
        hipLaunchKernelGGL(k_walk_copy, dim3(gc), dim3(256), 0, s, pw);
        HIPCHK(hipGetLastError());
        w.only = c->walk_fallback;
    }
    hipLaunchKernelGGL(k_seg_walk, dim3(grid), dim3(kWaveSize), 0, s, w);
    HIPCHK(hipGetLastError());
    return RAMCRC_OK;
}
}  // namespace

int ramcrc_segments_certify_device(ramcrc_ctx* c, const void* d_base, uint64_t seg_stride,
                                   uint32_t seg_capacity, uint64_t n_seg, const uint32_t* d_heads,
                                   ramcrc_seg_cert* d_certs, uint32_t* d_flags, void* stream)
{
    if (!c)
        return RAMCRC_EINVAL;
    if (n_seg == 0)
        return RAMCRC_OK;
    if (!d_base || !d_heads || !d_certs || n_seg > 0xFFFFFFFFull)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // scratch: placeholder certificates, walk status, the walk's entry count
    const uint64_t need = n_seg * (sizeof(ramcrc_seg_cert) + sizeof(ramcrc_seg_status)) / 4 + 2;
    int rc = grow_device(reinterpret_cast<void**>(&c->cert_scratch), &c->cert_scratch_cap, need,
                         sizeof(uint32_t));
    if (rc)
        return rc;
    uint64_t* d_n = reinterpret_cast<uint64_t*>(c->cert_scratch);
    ramcrc_seg_cert* tmp = reinterpret_cast<ramcrc_seg_cert*>(c->cert_scratch + 2);
    ramcrc_seg_status* st = reinterpret_cast<ramcrc_seg_status*>(tmp + n_seg);
    const dim3 grid(uint32_t((n_seg + 255) / 256));
    hipLaunchKernelGGL(k_cert_prep, grid, dim3(256), 0, s, d_heads, tmp, n_seg);
    HIPCHK(hipGetLastError());
    rc = ramcrc_segment_walk_device(c, d_base, seg_stride, seg_capacity, n_seg, tmp, st, nullptr, 0,
                                    d_n, stream);
    if (rc)
        return rc;
    hipLaunchKernelGGL(k_cert_emit, grid, dim3(256), 0, s, tmp, st, d_certs, d_flags, n_seg);
    HIPCHK(hipGetLastError());
    return RAMCRC_OK;
}

int ramcrc_verify_objects_device(ramcrc_ctx* c, const void* d_base, uint64_t seg_stride,
                                 const ramcrc_seg_entry* d_entries, uint64_t entries_cap,
                                 const uint64_t* d_n_entries, uint32_t* d_obj_crc,
                                 ramcrc_seg_status* d_status, void* stream)
{
    if (!c)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    return verify_impl(c, d_base, seg_stride, d_entries, entries_cap, d_n_entries, d_obj_crc,
                       d_status, reinterpret_cast<hipStream_t>(stream), nullptr);
}

namespace {
int verify_impl(ramcrc_ctx* c, const void* d_base, uint64_t seg_stride,
                const ramcrc_seg_entry* d_entries, uint64_t entries_cap, const uint64_t* d_n_entries,
                uint32_t* d_obj_crc, ramcrc_seg_status* d_status, hipStream_t s, const uint32_t* sum)
{
    if (entries_cap == 0)
        return RAMCRC_OK;
    if (!d_base || !d_entries || !d_n_entries || !d_obj_crc || !d_status)
        return RAMCRC_EINVAL;
    int rc = reserve_locked(c, default_chunk_bound(entries_cap), entries_cap);
    if (rc)
        return rc;
    BatchDesc d{};
    d.cshift = kChunkShift;
    d.base = static_cast<const uint8_t*>(d_base);
    d.seg_bytes = seg_stride;
    d.n = entries_cap;
#ifndef RAMCRC_NO_CAPTURE
    d.vstat = d_status;
#endif
    d.rec = reinterpret_cast<const u32x4*>(d_entries);
    d.n_dev = d_n_entries;
    d.seg_status = reinterpret_cast<const u32x4*>(d_status);
    d.out = d_obj_crc;
    d.flags = RAMCRC_FINALIZE;
    const uint32_t* nother = nullptr;
    rc = launch_planned<kRecords>(c, d, s, &nother, sum);
    if (rc)
        return rc;
    uint64_t grid = (entries_cap + 255) / 256;
    grid = grid < uint64_t(16) * c->ncu ? grid : uint64_t(16) * c->ncu;
    hipLaunchKernelGGL(k_obj_compare, dim3(grid), dim3(256), 0, s, d, d_status, nother);
    HIPCHK(hipGetLastError());
    return RAMCRC_OK;
}
}  // namespace

int ramcrc_assemble_objects_device(ramcrc_ctx* c, void* d_base, const uint64_t* d_off,
                                   const uint64_t* d_len, uint32_t* d_out, uint64_t n,
                                   void* stream)
{
    if (n == 0)
        return c ? RAMCRC_OK : RAMCRC_EINVAL;
    if (!c || !d_base || !d_off || !d_len)
        return RAMCRC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc = reserve_locked(c, default_chunk_bound(n), n);
    if (rc)
        return rc;
    if (!d_out) {
        rc = grow_device(reinterpret_cast<void**>(&c->obj_out), &c->obj_out_cap, n,
                         sizeof(uint32_t));
        if (rc)
            return rc;
        d_out = c->obj_out;
    }
    BatchDesc d{};
    d.cshift = kChunkShift;
    d.base = static_cast<const uint8_t*>(d_base);
    d.off = d_off;
    d.len = d_len;
    d.n = n;
    d.out = d_out;
    d.flags = RAMCRC_FINALIZE;
    rc = launch_planned<kObjects>(c, d, s);
    if (rc)
        return rc;
    hipLaunchKernelGGL(k_obj_stamp, dim3((n + 255) / 256), dim3(256), 0, s, d);
    HIPCHK(hipGetLastError());
    return RAMCRC_OK;
}

int ramcrc_assemble_objects_host(ramcrc_ctx* c, void* const* objs, const uint64_t* lens,
                                 uint64_t n)
{
    if (!c || (n && (!objs || !lens)))
        return RAMCRC_EINVAL;
    // CRC of bytes [4, len) of every object with a full header through the
    // pinned-staging batch path, then header.checksum stamped on the host.
    std::vector<const void*> ptrs;
    std::vector<uint64_t> ls;
    std::vector<uint64_t> which;
    for (uint64_t i = 0; i < n; i++) {
        if (lens[i] < kObjHeaderBytes)
            continue;
        if (!objs[i])
            return RAMCRC_EINVAL;
        ptrs.push_back(static_cast<const uint8_t*>(objs[i]) + 4);
        ls.push_back(lens[i] - 4);
        which.push_back(i);
    }
    if (ptrs.empty())
        return RAMCRC_OK;
    std::vector<uint32_t> out(ptrs.size());
    int rc = ramcrc_batch_host(c, ptrs.data(), ls.data(), nullptr, out.data(), ptrs.size(),
                               RAMCRC_FINALIZE);
    if (rc)
        return rc;
    for (size_t k = 0; k < which.size(); k++) {
        uint8_t* p = static_cast<uint8_t*>(objs[which[k]]);
        for (int b = 0; b < 4; b++)
            p[b] = uint8_t(out[k] >> (8 * b));
    }
    return RAMCRC_OK;
}

}  // extern "C"
