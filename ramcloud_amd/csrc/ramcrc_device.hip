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

#include <mutex>
#include <new>
#include <utility>
#include <vector>
#include <stdio.h>
#include <string.h>

#include "gf2.h"
#include "ramcrc.h"

namespace {

using ramcrc::OpTable;

constexpr int kWaveSize = 64;
constexpr int kWavesPerGroup = 16;                 // 1024-thread workgroups, 1 per CU
constexpr int kThreads = kWaveSize * kWavesPerGroup;
constexpr uint32_t kBlock = 1024;                  // bytes per wave step
constexpr int kChunkShift = 18;
constexpr uint64_t kChunk = 1ull << kChunkShift;   // 256 KiB per wave work item
constexpr uint64_t kLargeMin = 64 * 1024;          // batch API threshold
constexpr int kUnroll = 8;                         // blocks in flight per wave

// ------------------------------------------------------------------ tables
struct DeviceTables {
    OpTable stride_large;   // X^1024: Horner step of k_chunks
    OpTable stride_small;   // X^16:   Horner step of k_entries
    OpTable comb[7];        // X^4, X^16, X^32, X^64, X^128, X^256, X^512
    ramcrc::ByteTable t0;   // X^1 byte step
    uint32_t xblk[4][256];  // x^(8 * 1024 * b * 256^j)
    uint32_t xinv[1024];    // x^(-8 p)
};

constexpr DeviceTables make_device_tables()
{
    DeviceTables t{};
    t.stride_large = ramcrc::make_op(kBlock);
    t.stride_small = ramcrc::make_op(16);
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
constexpr uint32_t kX4Off = kRepBytes;                    // k_entries: X^4 (4 KiB)
constexpr uint32_t kT0Off = kRepBytes + 4096;             // k_entries: X^1 (1 KiB)
constexpr uint32_t kLdsEntries = kT0Off + 1024;           // 136192 B
static_assert(kLdsChunks <= 160 * 1024, "LDS budget");

__device__ __forceinline__ void fill_replicated(uint8_t* lds, const OpTable& op)
{
    // 4 tables x 256 entries x 32 replicas; each thread writes 4 replicas
    // (16 contiguous bytes) per iteration.
    for (uint32_t idx = threadIdx.x; idx < 4 * 256 * 8; idx += blockDim.x) {
        const uint32_t k = idx >> 11;
        const uint32_t b = (idx >> 3) & 255;
        const uint32_t q = idx & 7;
        const uint32_t v = op.t[k][b];
        const uint32_t off = (k >> 1) * 65536 + b * 256 + (k & 1) * 128 + q * 16;
        *reinterpret_cast<uint4*>(lds + off) = make_uint4(v, v, v, v);
    }
}

__device__ __forceinline__ void fill_plain(uint8_t* lds, uint32_t off, const uint32_t* src,
                                           uint32_t words)
{
    uint32_t* dst = reinterpret_cast<uint32_t*>(lds + off);
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x)
        dst[i] = src[i];
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

struct RepOp {
    uint32_t lr0, lr1, lr2, lr3;
    __device__ explicit RepOp(int lane)
        : lr0(lane_reg(0, lane)), lr1(lane_reg(1, lane)), lr2(lane_reg(2, lane)),
          lr3(lane_reg(3, lane))
    {
    }
    // X^stride(u) ^ w through the replicated tables.
    __device__ __forceinline__ uint32_t apply(const uint8_t* lds, uint32_t u, uint32_t w) const
    {
        const uint32_t a = *reinterpret_cast<const uint32_t*>(lds + rep_addr<0>(u, lr0));
        const uint32_t b = *reinterpret_cast<const uint32_t*>(lds + rep_addr<1>(u, lr1));
        const uint32_t c = *reinterpret_cast<const uint32_t*>(lds + rep_addr<2>(u, lr2));
        const uint32_t d = *reinterpret_cast<const uint32_t*>(lds + rep_addr<3>(u, lr3));
        return (a ^ b ^ w) ^ (c ^ d);
    }
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
    const int64_t dlo = int64_t(S) - int64_t(a);
    const int64_t dhi = int64_t(E) - int64_t(a);
    const int lo = dlo <= 0 ? 0 : (dlo >= 4 ? 4 : int(dlo));
    const int hi = dhi <= 0 ? 0 : (dhi >= 4 ? 4 : int(dhi));
    const uint32_t mhi = hi >= 4 ? 0xFFFFFFFFu : ((1u << (8 * hi)) - 1u);
    const uint32_t mlo = lo >= 4 ? 0xFFFFFFFFu : ((1u << (8 * lo)) - 1u);
    w &= (hi > lo) ? (mhi & ~mlo) : 0u;
    const int64_t d = -dlo;  // a - S
    if (d > -4 && d < 4)
        w ^= d >= 0 ? (init >> (8 * int(d))) : (init << (8 * int(-d)));
    return w;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Explicit global address space: generic (flat_*) loads would also count in
// lgkmcnt and serialise against the LDS table lookups.
typedef const __attribute__((address_space(1))) u32x4 gu32x4;
typedef const __attribute__((address_space(1))) uint8_t gu8;

__device__ __forceinline__ const gu32x4* gptr16(uint64_t addr)
{
    return (const gu32x4*)addr;
}

__device__ __forceinline__ u32x4 load16(uint64_t addr) { return *gptr16(addr); }

// ------------------------------------------------------------ descriptors
struct BatchDesc {
    const uint8_t* base;     // d_base
    const uint64_t* off;     // general mode
    const uint64_t* len;     // general mode
    uint64_t seg_bytes;      // uniform mode
    uint64_t n;              // buffers
    const uint32_t* init;    // nullable
    uint32_t* out;
    uint32_t flags;
};

// Buffer addressing modes.
//   kSegAligned: segment i = base + i*seg_bytes, base and seg_bytes multiples
//                of the chunk size -> chunk g maps to (g / per, g % per).
//   kSegUniform: same geometry, any alignment -> goes through the plan.
//   kTable:      buffer i = base + off[i], len[i] -> goes through the plan.
enum Mode { kSegAligned = 0, kSegUniform = 1, kTable = 2 };

template <int kMode>
__device__ __forceinline__ void buffer_range(const BatchDesc& d, uint64_t i, uint64_t& S,
                                             uint64_t& E)
{
    if (kMode != kTable) {
        S = reinterpret_cast<uint64_t>(d.base) + i * d.seg_bytes;
        E = S + d.seg_bytes;
    } else {
        S = reinterpret_cast<uint64_t>(d.base) + d.off[i];
        E = S + d.len[i];
    }
}

__device__ __forceinline__ uint64_t chunk_count(uint64_t S, uint64_t E)
{
    return ((E - 1) >> kChunkShift) - (S >> kChunkShift) + 1;
}

struct Plan {
    uint64_t* local;       // per entry: exclusive prefix of chunk counts within its group
    uint64_t* group_pref;  // per group of kThreads entries, exclusive prefix; [ngroups] = total
    uint64_t ngroups;
    uint32_t* partials;
    uint64_t partials_cap;
    uint32_t* status;      // bit 0: partials overflow
};

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
            atomicOr(pl.status, 1u);
        return;
    }
    for (uint64_t g = wave; g < total; g += nwaves) {
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
        const uint64_t cs = S >> kChunkShift;
        const uint64_t c_lo = (cs + k) << kChunkShift;
        const uint64_t lo = c_lo > S ? c_lo : S;
        const uint64_t c_hi = c_lo + kChunk;
        const uint64_t hi = c_hi < E ? c_hi : E;
        const uint32_t r = scan_chunk(lds, op, lane, S, E, init, lo, hi);
        if (lane == 0)
            pl.partials[g] = r;
    }
}

// ------------------------------------------------------------ k_combine
template <int kMode>
__global__ __launch_bounds__(256) void k_combine(BatchDesc d, Plan pl, uint64_t per_seg)
{
    const int lane = threadIdx.x & (kWaveSize - 1);
    const uint64_t i = uint64_t(blockIdx.x) * (256 / kWaveSize) + threadIdx.x / kWaveSize;
    if (i >= d.n)
        return;
    uint64_t S, E;
    buffer_range<kMode>(d, i, S, E);
    if (!is_large(E - S))
        return;   // handled by k_entries
    if (kMode != kSegAligned && ((*pl.status) & 1u))
        return;   // k_chunks refused the launch (partials overflow)
    const uint64_t g0 = kMode == kSegAligned ? i * per_seg
                                             : pl.group_pref[i / kThreads] + pl.local[i];
    const uint64_t cnt = chunk_count(S, E);
    const uint64_t cs = S >> kChunkShift;
    const uint64_t pend = (E + kBlock - 1) & ~uint64_t(kBlock - 1);
    uint32_t R = 0;
    for (uint64_t k = lane; k < cnt; k += kWaveSize) {
        const uint32_t r = pl.partials[g0 + k];
        const uint64_t ek = (k + 1 == cnt) ? pend : ((cs + k + 1) << kChunkShift);
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

// ------------------------------------------------------------ k_entries
template <int kMode>
__global__ __launch_bounds__(kThreads, 1) void k_entries(BatchDesc d, int skip_large)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsEntries];
    fill_replicated(lds, g_tab.stride_small);
    fill_plain(lds, kX4Off, &g_tab.comb[0].t[0][0], 1024);
    fill_plain(lds, kT0Off, g_tab.t0.t, 256);
    __syncthreads();

    const int lane = threadIdx.x & (kWaveSize - 1);
    const RepOp op(lane);
    const uint32_t* t0 = reinterpret_cast<const uint32_t*>(lds + kT0Off);
    const uint64_t nthreads = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < d.n; i += nthreads) {
        uint64_t S, E;
        buffer_range<kMode>(d, i, S, E);
        const uint64_t n = E - S;
        if (skip_large && is_large(n))
            continue;
        const uint32_t init = d.init ? d.init[i] : 0xFFFFFFFFu;
        uint32_t R;
        if (n < 4) {
            R = init;
            const gu8* p = (const gu8*)S;
            for (uint64_t b = 0; b < n; b++)
                R = t0[(R ^ p[b]) & 0xFF] ^ (R >> 8);
        } else {
            const uint64_t A = S & ~uint64_t(15);
            const uint64_t B = (E + 15) & ~uint64_t(15);
            uint32_t u0 = 0, u1 = 0, u2 = 0, u3 = 0;
            for (uint64_t a = A; a < B; a += 16) {
                u32x4 w = load16(a);
                if (a < S + 4 || a + 16 > E) {
                    w.x = fix_word(w.x, a + 0, S, E, init);
                    w.y = fix_word(w.y, a + 4, S, E, init);
                    w.z = fix_word(w.z, a + 8, S, E, init);
                    w.w = fix_word(w.w, a + 12, S, E, init);
                }
                u0 = op.apply(lds, u0, w.x);
                u1 = op.apply(lds, u1, w.y);
                u2 = op.apply(lds, u2, w.z);
                u3 = op.apply(lds, u3, w.w);
            }
            uint32_t y = plain_apply(lds, kX4Off, u0) ^ u1;
            y = plain_apply(lds, kX4Off, y) ^ u2;
            y = plain_apply(lds, kX4Off, y) ^ u3;
            y = plain_apply(lds, kX4Off, y);
            const uint32_t pad = uint32_t(B - E);
            R = pad ? mulmod_dev(y, g_tab.xinv[pad]) : y;
        }
        d.out[i] = (d.flags & RAMCRC_FINALIZE) ? ~R : R;
    }
}

// ------------------------------------------------------------ k_plan
template <int kMode>
__global__ __launch_bounds__(kThreads) void k_plan_count(BatchDesc d, Plan pl)
{
    __shared__ uint64_t wsum[kWavesPerGroup];
    const uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    uint64_t c = 0;
    if (i < d.n) {
        uint64_t S, E;
        buffer_range<kMode>(d, i, S, E);
        c = is_large(E - S) ? chunk_count(S, E) : 0;
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
        pl.group_pref[blockIdx.x] = before + x;   // group total, scanned by k_plan_scan
}

__global__ __launch_bounds__(kThreads) void k_plan_scan(Plan pl)
{
    // single workgroup: exclusive scan of ngroups totals in place, [ngroups] = total
    __shared__ uint64_t wsum[kWavesPerGroup];
    __shared__ uint64_t carry_s;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        carry_s = 0;
        *pl.status = 0;   // stream-ordered before this launch's k_chunks
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
    int ncu = 256;
    std::mutex mu;
    uint32_t* partials = nullptr;
    uint64_t partials_cap = 0;
    uint64_t* plan_local = nullptr;
    uint64_t plan_cap = 0;
    uint64_t* group_pref = nullptr;
    uint64_t group_cap = 0;
    uint32_t* status = nullptr;
    // host staging for ramcrc_batch_host / ramcrc_stream_host
    uint8_t* h_stage = nullptr;
    uint64_t h_stage_cap = 0;
    uint8_t* d_stage = nullptr;
    uint64_t d_stage_cap = 0;
    hipStream_t copy_stream = nullptr;
    hipStream_t compute_stream = nullptr;
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
    return pl;
}

// Bracket the byte-scan kernel with events when benchmark timing is on.
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
        } else if (hipEventCreate(&ev.first) != hipSuccess ||
                   hipEventCreate(&ev.second) != hipSuccess) {
            ev = {nullptr, nullptr};
            return;
        }
        (void)hipEventRecord(ev.first, s);
    }
    ~ScanTimer()
    {
        if (!ev.first)
            return;
        (void)hipEventRecord(ev.second, s);
        c->ev_used.push_back(ev);
    }
};

template <int kMode>
int launch_planned(ramcrc_ctx* c, const BatchDesc& d, hipStream_t s)
{
    Plan pl = make_plan(c, d.n);
    hipLaunchKernelGGL(k_plan_count<kMode>, dim3(pl.ngroups), dim3(kThreads), 0, s, d, pl);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_plan_scan, dim3(1), dim3(kThreads), 0, s, pl);
    HIPCHK(hipGetLastError());
    {
        ScanTimer t(c, s);
        hipLaunchKernelGGL(k_chunks<kMode>, dim3(c->ncu), dim3(kThreads), 0, s, d, pl,
                           uint64_t(0));
    }
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_combine<kMode>, dim3((d.n + 3) / 4), dim3(256), 0, s, d, pl, uint64_t(0));
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_entries<kMode>, dim3(c->ncu), dim3(kThreads), 0, s, d, 1);
    HIPCHK(hipGetLastError());
    return RAMCRC_OK;
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
    default: return "unknown error";
    }
}

const char* ramcrc_build_info(void)
{
    return "ramcrc gfx950: chunk=256KiB block=1KiB waves/WG=16 unroll=8 lds_chunks=159744 "
           "lds_entries=136192 large_min=64KiB";
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
    if (hipMalloc(reinterpret_cast<void**>(&c->status), 16) != hipSuccess) {
        delete c;
        return RAMCRC_ENOMEM;
    }
    (void)hipMemset(c->status, 0, 16);
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
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    return reserve_locked(c, max_chunks, max_entries);
}

int ramcrc_ctx_set_timing(ramcrc_ctx* c, int enable)
{
    if (!c)
        return RAMCRC_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    c->timing = enable != 0;
    return RAMCRC_OK;
}

int ramcrc_ctx_scan_time(ramcrc_ctx* c, double* total_ms, uint64_t* launches)
{
    if (!c)
        return RAMCRC_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
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

int ramcrc_ctx_status(ramcrc_ctx* c, uint32_t* status)
{
    if (!c || !status)
        return RAMCRC_EINVAL;
    DeviceGuard g(c->device);
    HIPCHK(hipMemcpy(status, c->status, sizeof(uint32_t), hipMemcpyDeviceToHost));
    return RAMCRC_OK;
}

int ramcrc_segments_device(ramcrc_ctx* c, const void* d_base, uint64_t seg_bytes, uint64_t nseg,
                           const uint32_t* d_init, uint32_t* d_out, uint32_t flags, void* stream)
{
    if (!c || !d_out || (!d_base && nseg && seg_bytes))
        return RAMCRC_EINVAL;
    if (nseg == 0)
        return RAMCRC_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    BatchDesc d{};
    d.base = static_cast<const uint8_t*>(d_base);
    d.seg_bytes = seg_bytes;
    d.n = nseg;
    d.init = d_init;
    d.out = d_out;
    d.flags = flags;
    if (seg_bytes < kLargeMin) {
        {
            ScanTimer t(c, s);
            hipLaunchKernelGGL(k_entries<kSegUniform>, dim3(c->ncu), dim3(kThreads), 0, s, d, 0);
        }
        HIPCHK(hipGetLastError());
        return RAMCRC_OK;
    }
    const uint64_t B = reinterpret_cast<uint64_t>(d_base);
    if ((B % kChunk) == 0 && (seg_bytes % kChunk) == 0) {
        // The recovery-scan fast path: no plan, chunk g -> (g / per, g % per).
        const uint64_t per = seg_bytes / kChunk;
        int rc = reserve_locked(c, per * nseg, 1);
        if (rc)
            return rc;
        Plan pl = make_plan(c, 0);
        {
            ScanTimer t(c, s);
            hipLaunchKernelGGL(k_chunks<kSegAligned>, dim3(c->ncu), dim3(kThreads), 0, s, d, pl,
                               per);
        }
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_combine<kSegAligned>, dim3((nseg + 3) / 4), dim3(256), 0, s, d, pl,
                           per);
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
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    int rc = reserve_locked(c, default_chunk_bound(n), n);
    if (rc)
        return rc;
    BatchDesc d{};
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
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    BatchDesc d{};
    d.base = static_cast<const uint8_t*>(d_base);
    d.off = d_off;
    d.len = d_len;
    d.n = n;
    d.init = d_init;
    d.out = d_out;
    d.flags = flags;
    {
        ScanTimer t(c, s);
        hipLaunchKernelGGL(k_entries<kTable>, dim3(c->ncu), dim3(kThreads), 0, s, d, 0);
    }
    HIPCHK(hipGetLastError());
    return RAMCRC_OK;
}

int ramcrc_batch_host(ramcrc_ctx* c, const void* const* ptrs, const uint64_t* lens,
                      const uint32_t* init, uint32_t* out, uint64_t n, uint32_t flags)
{
    if (!c || (n && (!ptrs || !lens || !out)))
        return RAMCRC_EINVAL;
    if (n == 0)
        return RAMCRC_OK;
    DeviceGuard g(c->device);
    // Pack every buffer 16-byte aligned into one pinned staging area, then one
    // H2D copy, one batch launch, one D2H copy.
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++)
        total += (lens[i] + 15) & ~uint64_t(15);
    const uint64_t meta = n * (2 * sizeof(uint64_t) + 2 * sizeof(uint32_t));
    const uint64_t need = total + meta + 64;
    {
        std::lock_guard<std::mutex> lk(c->mu);
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
    }
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
    if (rc)
        return rc;
    HIPCHK(hipMemcpyAsync(h_out, d_out, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
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
    DeviceGuard g(c->device);
    if (depth > 8)
        depth = 8;
    const uint64_t slot_bytes = uint64_t(batch) * seg_bytes;
    // Each slot: batch*seg_bytes of data + batch CRCs.
    const uint64_t slot_stride = (slot_bytes + 4 * uint64_t(batch) + 4095) & ~uint64_t(4095);
    const uint64_t need = slot_stride * uint64_t(depth);
    {
        std::lock_guard<std::mutex> lk(c->mu);
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
    }
    hipEvent_t copied[8], done[8];
    for (int k = 0; k < depth; k++) {
        HIPCHK(hipEventCreateWithFlags(&copied[k], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&done[k], hipEventDisableTiming));
    }
    const uint8_t* src = static_cast<const uint8_t*>(h_base);
    int rc = RAMCRC_OK;
    uint64_t nb = (nseg + batch - 1) / batch;
    for (uint64_t b = 0; b < nb && rc == RAMCRC_OK; b++) {
        const int k = int(b % depth);
        const uint64_t first = b * batch;
        const uint64_t cnt = (nseg - first) < uint64_t(batch) ? (nseg - first) : uint64_t(batch);
        uint8_t* slot = c->d_stage + uint64_t(k) * slot_stride;
        uint32_t* slot_out = reinterpret_cast<uint32_t*>(slot + slot_bytes);
        if (b >= uint64_t(depth))
            HIPCHK(hipStreamWaitEvent(c->copy_stream, done[k], 0));
        HIPCHK(hipMemcpyAsync(slot, src + first * seg_bytes, cnt * seg_bytes,
                              hipMemcpyHostToDevice, c->copy_stream));
        HIPCHK(hipEventRecord(copied[k], c->copy_stream));
        HIPCHK(hipStreamWaitEvent(c->compute_stream, copied[k], 0));
        rc = ramcrc_segments_device(c, slot, seg_bytes, cnt, nullptr, slot_out, flags,
                                    c->compute_stream);
        if (rc)
            break;
        HIPCHK(hipMemcpyAsync(h_out + first, slot_out, cnt * sizeof(uint32_t),
                              hipMemcpyDeviceToHost, c->compute_stream));
        HIPCHK(hipEventRecord(done[k], c->compute_stream));
    }
    HIPCHK(hipStreamSynchronize(c->compute_stream));
    HIPCHK(hipStreamSynchronize(c->copy_stream));
    for (int k = 0; k < depth; k++) {
        (void)hipEventDestroy(copied[k]);
        (void)hipEventDestroy(done[k]);
    }
    return rc;
}

}  // extern "C"
