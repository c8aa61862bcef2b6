// Ordered small-entry batches as one byte stream (RAMCRC_ORDERED; included
// by ramcrc_device.hip inside its anonymous namespace).
//
// RAMCloud hands the checksum path log entries in log order: the entries of a
// segment lie back to back (src/Segment.cc:197-228), the objects a recovery
// master replays come out of a segment walk in offset order
// (src/ObjectManager.cc:585-700), and a write batch is appended in order
// (src/ObjectManager.cc:1274-1297).  For such a batch -- entries sorted by
// offset, never overlapping, neighbours less than a page apart -- the CRCs
// follow from one pass over the covered bytes instead of one pass per entry:
//
//   raw(0, [S, E)) = P(E) ^ X^(E-S)(P(S)),   P(x) = raw(0, stream bytes before x)
//
// (the state-algebra identity of gf2.h), with the state reset to zero at every
// entry start, so the value at an entry's end *is* its CRC.  The stream is cut
// into equal spans of 128-byte steps, one per group of 8 lanes.  Per step the
// group reads its 128 bytes (lane u: dwords u, u + 8, u + 16, u + 24) and
// looks every byte up once in a position table: byte b at step position q
// contributes X^(128-q)(b) to the state at the step end, so the step's sum is
// an XOR of 16 lookups per lane and three shuffles, and the carry from the
// previous step is the previous state injected into the step's first four
// bytes.  Each group takes its dwords' bytes in a rotated order (byte
// (k + g4) & 3 at lookup k, g4 the group's index in its half-wave), so the 32
// lanes of a ds_read half-wave hit 32 banks for any data: the table's bank is
// the byte's step position mod 32 (table layout below).
//
// An entry boundary inside a step (an "event") costs one masked sum over the
// positions before it: whole dwords from the step's dword sums, the 1-3
// remaining bytes by four more lookups in the lane that holds them.  At an
// entry start the running state is re-based (C); at an entry end the value,
// taken relative to the step end, is moved back to the boundary with
// X^(-128) and X^(p) (8 lookups) and stored.  Entries whose start lies in an
// earlier span leave their partial value for k_stream_fix, which chains the
// span-end states (one GF(2) multiply per span crossed).  All arithmetic is
// exact; the kernels reproduce Crc32C::update / getResult bit for bit.
//
// Launch sequence: k_stream_prep (validation, first entry per span),
// k_stream (the pass), k_stream_fix (entries crossing spans).  A batch that
// is not ordered and dense is refused: nothing is written, RAMCRC_EORDER
// from ramcrc_ctx_check.

constexpr uint32_t kStatusOrder = 8u;      // an ORDERED batch was not: nothing written
#ifndef RAMCRC_STREAM_WAVES
#define RAMCRC_STREAM_WAVES 16
#endif
constexpr int kStreamWaves = RAMCRC_STREAM_WAVES;   // waves per workgroup (one workgroup per CU)
constexpr int kStreamGroups = kStreamWaves * 8;   // spans per workgroup
constexpr int kStreamWin = 8;              // entry slots per lane: 64 entries per group window
constexpr uint64_t kStreamGap = 4096;      // largest gap between neighbours (page safety)
#ifndef RAMCRC_STREAM_U
#define RAMCRC_STREAM_U 4
#endif
constexpr int kStreamU = RAMCRC_STREAM_U;  // steps of prefetch per group
constexpr int32_t kBig = 0x7FFFFFFF;       // "no boundary"
constexpr uint32_t kStreamMaxPass = 1u << 22;   // event passes per step: a hard stop
// LDS: position table (v_perm layout) | X^-128 tables | X^d(0xFFFFFFFF)
//   word (q & 63) of row [q >> 6][b] = X^(128 - q)(b), q = step position 0..127:
//   byte address = (q >> 6) * 65536 + b * 256 + 4 * (q & 63)  ->  bank q mod 32
constexpr uint32_t kStrInvOff = 131072;                   // X^-128: 4 x 256 words
constexpr uint32_t kStrFfOff = kStrInvOff + 4096;         // X^d(0xFFFFFFFF), d = 0..128
constexpr uint32_t kLdsStream = kStrFfOff + 132 * 4;      // 135696 B
static_assert(kLdsStream <= 160 * 1024, "LDS budget");

struct StreamDesc {
    const uint8_t* base;
    const uint64_t* off;
    const uint64_t* len;
    uint64_t n;
    uint32_t* out;
    uint32_t flags;
    uint32_t obj;          // kObjects: entry i is bytes [4, len) of the object at off[i]
                           // (Object::computeChecksum); objects under 24 B are empty
    uint32_t nspan;        // groups of the launch: one span each
    uint32_t seq;          // launch sequence number (refusal word)
    uint32_t* first_ev;    // per span: first entry whose end lies past the span start
    uint32_t* span_t;      // per span: the group's state at the span end
    uint32_t* xe_val;      // per span: raw(0, [span start, E)) of an entry from an earlier span
    uint32_t* xe_idx;      // per span: that entry, or kNoIdx
    uint32_t* bad_seq;     // == seq: this launch's batch was refused by k_stream_prep
    uint32_t* status;
    // records mode (k_stream<true>): the object records of a segment walk
    const u32x4* rec;      // ramcrc_seg_entry {segment, offset, length, header}
    const uint64_t* n_dev; // live records (device), <= n
    ramcrc_seg_status* vstat;   // the walk's status per segment; bad_objects counted here
    uint64_t stride;       // segment i at base + i * stride
    uint64_t nseg;
    uint32_t spr;          // spans per segment (a multiple of 8: a wave stays in one segment)
    unsigned long long* seg_first;   // per segment: seq << 32 | its first record (k_stream_rprep)
};

// One segment of a records-mode launch: its records are rec[first, first +
// count), contiguous and in offset order (both walkers write them so), and its
// stream covers [0, rlen) -- the end of its last entry -- cut into spr spans
// of L bytes.  ok: the walk passed it (RAMCRC_SEG_OK) and this launch indexed it.
struct SegInfo {
    bool ok;
    uint64_t first, count, rlen, L, sps, addr;
};

// Object bytes of a walk record relative to its segment: [S, E) of
// Object::computeChecksum (payload bytes [4, length)), or an empty range at
// the payload for records that are not checked here (other types, objects
// shorter than their header or running past the segment).
__device__ __forceinline__ bool rec_range(const u32x4& r, uint64_t& S, uint64_t& E)
{
    const uint64_t payload = uint64_t(r.y) + 1 + ((r.w >> 6) & 3) + 1;
    const bool obj = (r.w & (0x3f | kRecOverlong)) == RAMCRC_LOG_ENTRY_TYPE_OBJ &&
                     r.z >= kObjHeaderBytes;
    S = obj ? payload + 4 : payload;
    E = obj ? payload + r.z : payload;
    return obj;
}

__device__ __forceinline__ SegInfo seg_info(const StreamDesc& d, uint64_t s)
{
    SegInfo g{};
    const u32x4 st = *reinterpret_cast<const u32x4*>(&d.vstat[s]);   // flags, checksum, entries
    const unsigned long long f = d.seg_first[s];
    g.count = st.z;
    g.first = uint32_t(f);
    g.ok = (st.x & RAMCRC_SEG_OK) && g.count > 0 && uint32_t(f >> 32) == d.seq;
    if (!g.ok)
        return g;
    uint64_t S, E;
    rec_range(d.rec[g.first + g.count - 1], S, E);
    g.rlen = E;
    const uint64_t steps = (g.rlen + 127) / 128;
    g.sps = (steps + d.spr - 1) / d.spr;
    if (g.sps == 0)
        g.sps = 1;
    g.L = 128 * g.sps;
    g.addr = reinterpret_cast<uint64_t>(d.base) + s * d.stride;
    return g;
}

struct StreamGeo {
    uint64_t A0;    // start of step 0: the first entry's 128-byte line
    uint64_t R1;    // end of the last entry (the end of the batch when ordered)
    uint64_t ns;    // steps
    uint64_t sps;   // steps per span
    uint64_t L;     // span bytes
};

// [S, E) of entry i.
__device__ __forceinline__ void stream_range(const StreamDesc& d, uint64_t i, uint64_t& S,
                                             uint64_t& E)
{
    const uint64_t o = reinterpret_cast<uint64_t>(d.base) + d.off[i], L = d.len[i];
    if (d.obj) {
        const bool live = L >= kObjHeaderBytes;
        S = live ? o + 4 : o;
        E = live ? o + L : o;
    } else {
        S = o;
        E = o + L;
    }
}

__device__ __forceinline__ StreamGeo stream_geo(const StreamDesc& d)
{
    uint64_t R0, R1, S1;
    stream_range(d, 0, R0, S1);
    stream_range(d, d.n - 1, S1, R1);
    StreamGeo g;
    g.A0 = R0 & ~uint64_t(127);
    g.R1 = R1 > g.A0 ? R1 : g.A0;
    g.ns = (g.R1 - g.A0 + 127) / 128;
    if (g.ns == 0)
        g.ns = 1;
    g.sps = (g.ns + d.nspan - 1) / d.nspan;
    g.L = 128 * g.sps;
    return g;
}

// x^(8 d) for any 32-bit d: four table factors.
__device__ __forceinline__ uint32_t xpow8_any(uint64_t d)
{
    uint32_t r = ramcrc::kOne;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t b = uint32_t(d >> (8 * j)) & 0xFF;
        if (b)
            r = mulmod_dev(r, g_tab.xbyte[j][b]);
    }
    return r;
}

// Validation and the first entry of every span.  Entry i owns the spans whose
// start lies in [E(i-1), E(i)); the last entry also the empty spans after it.
__global__ __launch_bounds__(256) void k_stream_prep(StreamDesc d)
{
    const StreamGeo g = stream_geo(d);
    const uint64_t nsp = (g.ns + g.sps - 1) / g.sps;   // spans holding steps
    bool bad = false;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < d.n;
         i += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t S, E;
        stream_range(d, i, S, E);
        uint64_t lo = 0;
        bad |= E < S;
        if (i > 0) {
            uint64_t Sp, Ep;
            stream_range(d, i - 1, Sp, Ep);
            bad |= S < Ep || S - Ep >= kStreamGap || Ep < Sp;
            lo = Ep > g.A0 ? (Ep - g.A0 + g.L - 1) / g.L : 0;
        }
        uint64_t hi = E > g.A0 ? (E - g.A0 + g.L - 1) / g.L : 0;
        if (i == d.n - 1)
            hi = nsp;
        if (hi > nsp)
            hi = nsp;
        for (uint64_t s = lo; s < hi; s++)
            d.first_ev[s] = (i == d.n - 1 && s * g.L + g.A0 >= E) ? uint32_t(d.n) : uint32_t(i);
    }
    if (bad) {
        *d.bad_seq = d.seq;
        atomicOr(d.status, kStatusSticky | kStatusOrder);
    }
}

// Records mode, pass 1: every segment's first record, tagged with the launch
// sequence number.  A segment whose records form two runs, or whose offsets do
// not increase, is refused (it cannot come from the walk).
__global__ __launch_bounds__(256) void k_stream_rprep(StreamDesc d)
{
    const uint64_t live = *d.n_dev < d.n ? *d.n_dev : d.n;
    bool bad = false;
    for (uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < live;
         r += uint64_t(gridDim.x) * blockDim.x) {
        const u32x4 x = d.rec[r];
        if (x.x >= d.nseg) {
            bad = true;
            continue;
        }
        // only segments that passed the walk are checked (the records of a
        // failed one -- e.g. an offset wrap walked backwards -- are skipped)
        if (!(reinterpret_cast<const u32x4*>(d.vstat)[x.x].x & RAMCRC_SEG_OK))
            continue;
        const u32x4 y = r ? d.rec[r - 1] : u32x4{0xFFFFFFFFu, 0u, 0u, 0u};
        if (y.x != x.x) {
            const unsigned long long old =
                atomicExch(&d.seg_first[x.x], (static_cast<unsigned long long>(d.seq) << 32) | r);
            bad |= uint32_t(old >> 32) == d.seq;   // a second run of the segment
        } else {
            bad |= y.y >= x.y;
        }
    }
    if (bad) {
        *d.bad_seq = d.seq;
        atomicOr(d.status, kStatusSticky | kStatusOrder);
    }
}

// Records mode, pass 2: the first record of every span (as k_stream_prep,
// per segment).
__global__ __launch_bounds__(256) void k_stream_rprep2(StreamDesc d)
{
    if (*d.bad_seq == d.seq)
        return;
    const uint64_t live = *d.n_dev < d.n ? *d.n_dev : d.n;
    bool bad = false;
    for (uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < live;
         r += uint64_t(gridDim.x) * blockDim.x) {
        const u32x4 x = d.rec[r];
        const SegInfo g = seg_info(d, x.x);
        if (!g.ok)
            continue;
        if (r < g.first || r >= g.first + g.count) {
            bad = true;   // the table does not hold exactly the segment's walked entries
            continue;
        }
        uint64_t S, E, lo = 0;
        rec_range(x, S, E);
        if (r > g.first) {
            uint64_t Sp, Ep;
            rec_range(d.rec[r - 1], Sp, Ep);
            bad |= S < Ep;
            lo = (Ep + g.L - 1) / g.L;
        }
        uint64_t hi = (E + g.L - 1) / g.L;
        const bool last = r == g.first + g.count - 1;
        if (last || hi > d.spr)
            hi = d.spr;
        for (uint64_t k = lo; k < hi; k++)
            d.first_ev[uint64_t(x.x) * d.spr + k] =
                (last && k * g.L >= E) ? uint32_t(g.first + g.count) : uint32_t(r);
    }
    // a segment that passed the walk but has no records in this table
    for (uint64_t sg = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; sg < d.nseg;
         sg += uint64_t(gridDim.x) * blockDim.x) {
        const u32x4 st = *reinterpret_cast<const u32x4*>(&d.vstat[sg]);
        bad |= (st.x & RAMCRC_SEG_OK) && st.z > 0 && uint32_t(d.seg_first[sg] >> 32) != d.seq;
    }
    if (bad) {
        *d.bad_seq = d.seq;
        atomicOr(d.status, kStatusSticky | kStatusOrder);
    }
}

// XOR / min over the 8 lanes of a group: quad swaps, then the half-row mirror.
__device__ __forceinline__ uint32_t grp_xor(uint32_t v)
{
    v ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0xB1, 0xF, 0xF, false));    // lane ^ 1
    v ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x4E, 0xF, 0xF, false));    // lane ^ 2
    v ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x141, 0xF, 0xF, false));   // 7 - lane
    return v;
}
__device__ __forceinline__ uint32_t quad_xor(uint32_t v)
{
    v ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0xB1, 0xF, 0xF, false));
    v ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x4E, 0xF, 0xF, false));
    return v;
}
__device__ __forceinline__ int32_t grp_min(int32_t v)
{
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false));
    return v;
}
__device__ __forceinline__ uint32_t grp_or(uint32_t v)
{
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0xB1, 0xF, 0xF, false));
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x4E, 0xF, 0xF, false));
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x141, 0xF, 0xF, false));
    return v;
}

__device__ __forceinline__ uint32_t lds_u32(const uint8_t* lds, uint32_t a)
{
    return *reinterpret_cast<const uint32_t*>(lds + a);
}

// LDS address of X^(128 - q)(b) for a step position q.
__device__ __forceinline__ uint32_t str_addr(uint32_t q, uint32_t b)
{
    return ((q >> 6) << 16) | (b << 8) | ((q & 63) << 2);
}

__device__ __forceinline__ void stream_fill(uint8_t* lds)
{
    // position table: 8192 chunks of 16 B; chunk (h, b, c) = post[128 (255 - b) + 64 h + 4 c ..]
    constexpr uint32_t kPos = 8192, kInv = 256, kFf = 132 / 4;
    constexpr uint32_t kAll = kPos + kInv + kFf;
    constexpr uint32_t kPer = (kAll + kStreamWaves * kWaveSize - 1) / (kStreamWaves * kWaveSize);
    const uint4* post = reinterpret_cast<const uint4*>(g_tab.post);
    const uint4* inv = reinterpret_cast<const uint4*>(&g_tab.xinv128);
    const uint4* ff = reinterpret_cast<const uint4*>(g_tab.xff);
    uint4 v[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t i = threadIdx.x + j * (kStreamWaves * kWaveSize);
        if (i < kPos) {
            const uint32_t h = i >> 12, b = (i >> 4) & 255, c = i & 15;
            v[j] = post[(128 * (255 - b) + 64 * h) / 4 + c];
        } else if (i < kPos + kInv) {
            v[j] = inv[i - kPos];
        } else if (i < kAll) {
            v[j] = ff[i - kPos - kInv];
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t i = threadIdx.x + j * (kStreamWaves * kWaveSize);
        if (i < kAll)
            *reinterpret_cast<uint4*>(lds + 16 * i) = v[j];
    }
}

// One span per group of 8 lanes.  kRec: records mode (object checks of a
// segment walk; spans per segment, the stored Object::Header::checksum compared
// at each object's end).
template <bool kRec>
__global__ __launch_bounds__(kStreamWaves * kWaveSize, 1) void k_stream(StreamDesc d)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsStream];
    const int lane = threadIdx.x & (kWaveSize - 1);
    const uint32_t u = uint32_t(lane) & 7, grp = uint32_t(lane) >> 3, g4 = grp & 3;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWaveSize);
    const uint64_t wspan = (uint64_t(blockIdx.x) * kStreamWaves + wave) * 8;   // first span of the wave
    const uint64_t span = wspan + grp;
    const bool refused = *d.bad_seq == d.seq;
    // geometry: this group's span [sg, sg + L), the wave's bytes [wbase, wbase + wlen),
    // entries [e_lo, e_hi)
    uint64_t sg, L, sps, wbase, wlen, e0, e_hi, seg = 0;
    bool idle_wave, idle;
    if (kRec) {
        seg = wspan / d.spr;   // uniform: the wave's 8 spans are in one segment
        const SegInfo gi = seg < d.nseg ? seg_info(d, seg) : SegInfo{};
        const uint64_t k = span - seg * d.spr, k0 = wspan - seg * d.spr;
        idle_wave = refused || !gi.ok;
        L = gi.L;
        sps = gi.sps;
        sg = gi.addr + k * L;
        wbase = gi.addr + k0 * L;
        // whole dwords: a dword load partly past the limit would read as 0
        const uint64_t rl4 = (gi.rlen + 3) & ~uint64_t(3);
        wlen = rl4 > k0 * L ? min(rl4 - k0 * L, 8 * L) : 0;
        idle = idle_wave;
        e_hi = gi.first + gi.count;
        e0 = idle ? e_hi : d.first_ev[span];
    } else {
        const StreamGeo geo = stream_geo(d);
        idle_wave = refused || wspan * geo.sps >= geo.ns;
        L = geo.L;
        sps = geo.sps;
        sg = geo.A0 + span * L;
        wbase = geo.A0 + wspan * L;
        // whole dwords (the last one may pass R1 by up to 3 bytes, inside its
        // page): a dword load partly past the limit would read as 0
        const uint64_t r4 = (geo.R1 + 3) & ~uint64_t(3);
        wlen = r4 > wbase ? min(r4 - wbase, 8 * L) : 0;
        idle = span * geo.sps >= geo.ns;
        e_hi = d.n;
        e0 = idle ? d.n : 0;
    }
    stream_fill(lds);
    if (!kRec && !idle_wave && !idle)
        e0 = d.first_ev[span];
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(idle_wave ? 1 : 0))
        return;   // uniform per wave
    const int32_t Li = int32_t(L);
    const bool finalize = d.flags & RAMCRC_FINALIZE;

    // the wave's 8 spans through one buffer descriptor per step (base advanced
    // by the step, records shrunk by it): the range check covers voffset + the
    // immediate, not soffset, so the step offset lives in the descriptor and
    // every byte past the batch reads 0
    const uint32_t voff = grp * uint32_t(L) + 4 * u;
    auto load_step = [&](uint64_t t) -> u32x4 {
        const uint64_t tb = __builtin_amdgcn_readfirstlane(uint32_t(t)) * uint64_t(128);
        const uint64_t b = wbase + tb;
        const uint32_t nrec = wlen > tb ? uint32_t(wlen - tb) : 0u;
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<void*>((uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(b >> 32))) << 32) |
                                    uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(b)))),
            (short)0, int(__builtin_amdgcn_readfirstlane(nrec)), 0x00020000);
        u32x4 w;
        w.x = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, 0, 0);
        w.y = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff + 32, 0, 0);
        w.z = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff + 64, 0, 0);
        w.w = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff + 96, 0, 0);
        return w;
    };

    // lookup address constants: byte k of the rotated dword (position (k + g4) & 3 of the
    // dword) of dword j: half j >> 1 in lr[j >> 1][k], +128 for odd j
    uint32_t lr[2][4];
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int k = 0; k < 4; k++)
            lr[h][k] = (uint32_t(h) << 16) | (16 * u + 4 * ((uint32_t(k) + g4) & 3));
    auto addr = [&](uint32_t xr, int h, int k) -> uint32_t {
        return __builtin_amdgcn_perm(xr, lr[h][k], 0x0C020000u | ((4u + uint32_t(k)) << 8));
    };

    // entry window: lane u holds entries e0 + u + 8 m, m = 0..7, relative to the span start
    int32_t Sr[kStreamWin], Er[kStreamWin];
    uint32_t cnt = 0;   // slots this lane has finished
    auto rel = [&](uint64_t x) -> int32_t {
        const int64_t r = int64_t(x - sg);
        return r < 0 ? -1 : (r > int64_t(Li) + 1 ? Li + 1 : int32_t(r));
    };
    auto load_window = [&]() {
#pragma unroll
        for (int m = 0; m < kStreamWin; m++) {
            const uint64_t e = e0 + u + 8 * uint64_t(m);
            if (e < e_hi) {
                uint64_t S, E;
                if (kRec) {
                    rec_range(d.rec[e], S, E);
                    const uint64_t a = sg - (span - seg * d.spr) * L;   // the segment's address
                    S += a;
                    E += a;
                } else {
                    stream_range(d, e, S, E);
                }
                Sr[m] = rel(S);
                Er[m] = rel(E);
            } else {
                Sr[m] = kBig;
                Er[m] = kBig;
            }
        }
        cnt = 0;
    };
    load_window();
    // empty entries exactly at the start of step 0 belong to no span's boundaries
    // (a span owns (start, start + L]): span 0 writes them (no record mode entry
    // starts at a segment's offset 0)
    if (!kRec && span == 0)
        for (uint64_t i = u; i < e0; i += 8)
            d.out[i] = finalize ? 0u : 0xFFFFFFFFu;
    // the group's first entry may have started before the span: its start is done
    bool Sd = u == 0 && Sr[0] <= 0, Ed = false;
    bool cross = u == 0 && Sr[0] < 0;   // started in an earlier span: k_stream_fix finishes it
    bool xe_done = false;               // lane 0: the cross-span entry ended here
    // state at the end of the previous step: an entry starting exactly at the
    // span start gets its initial state injected into the first four bytes
    uint32_t G = grp_or(u == 0 && Sr[0] == 0 ? 1u : 0u) ? 0xFFFFFFFFu : 0u;
    bool overrun = false;
    uint32_t stored = 0;   // records mode: Object::Header::checksum of this lane's open object
    // records mode: the previous step's dword 24 + u (lane 7: step bytes 124..127);
    // before step 0 the bytes ahead of the span (none ahead of a segment's first span)
    uint32_t prev3 = 0;
    if (kRec && span != seg * d.spr)
        prev3 = *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(sg - 32 + 4 * u);
    // an object starting exactly at the span start never sees its start event:
    // its stored checksum is the previous span's last dword (no object starts at
    // a segment's offset 0)
    if (kRec && u == 0 && Sr[0] == 0 && span != seg * d.spr)
        stored = *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(sg - 4);

    u32x4 buf[kStreamU];
#pragma unroll
    for (int i = 0; i < kStreamU; i++)
        buf[i] = load_step(uint64_t(i) < sps ? uint64_t(i) : sps - 1);

    for (uint64_t t0 = 0; t0 < sps; t0 += kStreamU) {
#pragma unroll
        for (int ii = 0; ii < kStreamU; ii++) {
            const uint64_t t = t0 + ii;
            if (t >= sps)
                break;   // uniform
            u32x4 w = buf[ii];
            const uint64_t tn = t + kStreamU;
            buf[ii] = load_step(tn < sps ? tn : sps - 1);
            const uint32_t wr0 = w.x;   // dword 0 before the carry
            if (u == 0)
                w.x ^= G;   // carry: the previous state injected into bytes 0..3
            const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
            uint32_t D[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t xr = __builtin_amdgcn_alignbyte(ws[j], ws[j], g4);
                const uint32_t a0 = lds_u32(lds, addr(xr, j >> 1, 0) + 128 * (j & 1));
                const uint32_t a1 = lds_u32(lds, addr(xr, j >> 1, 1) + 128 * (j & 1));
                const uint32_t a2 = lds_u32(lds, addr(xr, j >> 1, 2) + 128 * (j & 1));
                const uint32_t a3 = lds_u32(lds, addr(xr, j >> 1, 3) + 128 * (j & 1));
                D[j] = xor3(a0, a1, a2) ^ a3;
            }
            const uint32_t F = xor3(D[0], D[1], D[2]) ^ D[3];
            const int32_t T0 = int32_t(t) * 128;
            uint32_t C = 0;
            // boundaries in (T0, T0 + 128], in order; every pass resolves at least one
            uint32_t guard = 0;
            while (true) {
                if (++guard > kStreamMaxPass) {   // cannot happen; never spin the GPU
                    overrun = true;
                    break;
                }
                int32_t nb = !Sd ? Sr[0] : (!Ed ? Er[0] : kBig);
                int32_t P = grp_min(nb);
                if (P == kBig && e0 + 64 < e_hi && cnt == kStreamWin) {
                    // window used up (cnt is equal in the group then): next 64 entries
                    e0 += 64;
                    load_window();
                    Sd = false;
                    Ed = false;
                    nb = Sr[0];
                    P = grp_min(nb);
                }
                const bool has = P <= T0 + 128;
                if (!__builtin_amdgcn_ballot_w64(has))
                    break;
                if (has) {
                    const uint32_t p = uint32_t(P - T0);   // 1..128
                    const uint32_t Pd = p >> 2, r = p & 3;
                    // positions < p: whole dwords from D, then the r bytes of dword Pd
                    uint32_t acc = 0;
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        acc ^= (u + 8 * uint32_t(j) < Pd) ? D[j] : 0u;
                    if (r) {
                        const uint32_t js = Pd >> 3, us = Pd & 7;
                        uint32_t wsel = js == 0 ? ws[0] : (js == 1 ? ws[1] : (js == 2 ? ws[2] : ws[3]));
                        const uint32_t m = (1u << (8 * r)) - 1u;
                        // bytes r..3 of dword 0 hold the injected carry only
                        wsel = (wsel & m) | (Pd == 0 ? (G & ~m) : 0u);
                        wsel = u == us ? wsel : 0u;
                        const uint32_t xr = __builtin_amdgcn_alignbyte(wsel, wsel, g4);
                        const uint32_t hj = js >> 1, oj = (js & 1) * 128;
#pragma unroll
                        for (int k = 0; k < 4; k++) {
                            const uint32_t a = __builtin_amdgcn_perm(
                                xr, lr[0][k] | (hj << 16), 0x0C020000u | ((4u + uint32_t(k)) << 8));
                            acc ^= lds_u32(lds, a + oj);
                        }
                    }
                    const uint32_t V = grp_xor(acc);
                    const uint32_t d8 = 128 - p;   // distance of the boundary to the step end
                    const bool isS = !Sd && Sr[0] == P;
                    const bool isE = (Sd || isS) && !Ed && Er[0] == P;
                    const bool empty = isS && isE;
                    const uint32_t idx = uint32_t(e0) + u + 8 * cnt;
                    // the entry (at most one) that ends here and began before
                    const bool realE = isE && !empty;
                    if (grp_or(realE ? 1u : 0u)) {
                        const uint32_t Y = V ^ C;
                        uint32_t raw = Y;
                        if (d8) {
                            const uint32_t k = u & 3;
                            const uint32_t Z = quad_xor(
                                lds_u32(lds, kStrInvOff + 4 * (256 * k + ((Y >> (8 * k)) & 0xFF))));
                            if (p >= 4) {
                                raw = quad_xor(lds_u32(lds, str_addr(128 - p + k, (Z >> (8 * k)) & 0xFF)));
                            } else {
                                raw = mulmod_dev(Z, p == 1 ? ramcrc::xpow8(1)
                                                           : (p == 2 ? ramcrc::xpow8(2) : ramcrc::xpow8(3)));
                            }
                        }
                        if (realE) {
                            if (cross) {
                                d.xe_val[span] = raw;
                                d.xe_idx[span] = idx;
                                xe_done = true;
                            } else {
                                const uint32_t res = finalize ? ~raw : raw;
                                d.out[idx] = res;
                                if (kRec && res != stored)   // src/ObjectManager.cc:659-663
                                    atomicAdd(&d.vstat[seg].bad_objects, 1u);
                            }
                        }
                    }
                    if (!kRec && empty)   // Crc32C of no bytes: the initial state
                        d.out[idx] = finalize ? 0u : 0xFFFFFFFFu;
                    if (grp_or(isS ? 1u : 0u)) {
                        // re-base at the entry start, initial state injected
                        C = V ^ lds_u32(lds, kStrFfOff + 4 * d8);
                        if (kRec) {
                            // the object's stored checksum: the 4 bytes before S (step
                            // positions p - 4 .. p - 1; below 0 they are the previous
                            // step's bytes 124..127, held by lane 7)
                            const int32_t q0 = int32_t(p) - 4;
                            const int32_t d0 = q0 >> 2, d1 = (q0 + 3) >> 2;
                            auto own = [&](int32_t dd) -> uint32_t {   // this lane's dword dd >> 3
                                const int32_t j = dd >> 3;
                                return j < 0 ? prev3 : (j == 0 ? wr0 : (j == 1 ? ws[1] : (j == 2 ? ws[2] : ws[3])));
                            };
                            const uint32_t gbase = uint32_t(lane) & ~7u;
                            const uint32_t v0 = uint32_t(__builtin_amdgcn_ds_bpermute(
                                int((gbase + (uint32_t(d0) & 7)) * 4), int(own(d0))));
                            const uint32_t v1 = uint32_t(__builtin_amdgcn_ds_bpermute(
                                int((gbase + (uint32_t(d1) & 7)) * 4), int(own(d1))));
                            const uint32_t hdr = __builtin_amdgcn_alignbyte(v1, v0, uint32_t(q0) & 3);
                            if (isS)
                                stored = hdr;
                        }
                    }
                    Sd = Sd || isS;
                    Ed = Ed || isE;
                    if (Ed) {   // next slot
#pragma unroll
                        for (int m = 0; m < kStreamWin - 1; m++) {
                            Sr[m] = Sr[m + 1];
                            Er[m] = Er[m + 1];
                        }
                        Sr[kStreamWin - 1] = kBig;
                        Er[kStreamWin - 1] = kBig;
                        cnt++;
                        Sd = false;
                        Ed = false;
                        cross = false;
                    }
                }
            }
            G = grp_xor(F) ^ C;
            prev3 = ws[3];
        }
    }
    // span end: the state (of an entry still open, or of the whole span) and the
    // cross-span marker (lane 0 owns the group's first entry)
    if (overrun)   // refuse: RAMCRC_EINTERNAL from ramcrc_ctx_check
        atomicOr(d.status, kStatusSticky | kStatusBins);
    if (u == 0) {
        d.span_t[span] = G;
        if (!xe_done)
            d.xe_idx[span] = kNoIdx;   // no entry of an earlier span ended here
    }
}

// Entries that began in an earlier span: the state at their start span's end,
// carried through the spans they cover, then the partial value of the span
// where they end.  Records mode: spans of the object's segment, and the
// stored checksum compared (its header was in an earlier span).
template <bool kRec>
__global__ __launch_bounds__(256) void k_stream_fix(StreamDesc d)
{
    const uint64_t g = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (g >= d.nspan || *d.bad_seq == d.seq)
        return;
    uint64_t S, E, sg, L, h, kg;
    const uint32_t* span_t = d.span_t;
    uint32_t i;
    uint64_t seg = 0;
    if (kRec) {
        seg = g / d.spr;
        if (seg >= d.nseg)
            return;
        const SegInfo gi = seg_info(d, seg);
        if (!gi.ok)
            return;
        i = d.xe_idx[g];
        if (i == kNoIdx)
            return;
        rec_range(d.rec[i], S, E);   // relative to the segment
        L = gi.L;
        kg = g - seg * d.spr;
        sg = kg * L;
        h = S / L;
        span_t += seg * d.spr;
    } else {
        const StreamGeo geo = stream_geo(d);
        if (g * geo.sps >= geo.ns)
            return;
        i = d.xe_idx[g];
        if (i == kNoIdx)
            return;
        stream_range(d, i, S, E);
        // the span holding S: its group re-based there (an entry starting exactly
        // at a span start had its initial state injected by that span's group)
        L = geo.L;
        kg = g;
        sg = geo.A0 + g * L;
        h = (S - geo.A0) / L;
    }
    uint32_t st = span_t[h];
    if (h + 1 < kg) {
        const uint32_t cL = xpow8_any(L);
        for (uint64_t m = h + 1; m < kg; m++)
            st = mulmod_dev(st, cL) ^ span_t[m];
    }
    const uint32_t raw = mulmod_dev(st, xpow8_any(E - sg)) ^ d.xe_val[g];
    const uint32_t res = (d.flags & RAMCRC_FINALIZE) ? ~raw : raw;
    d.out[i] = res;
    if (kRec) {
        const uint64_t a = reinterpret_cast<uint64_t>(d.base) + seg * d.stride + S - 4;
        const gu8* q = reinterpret_cast<const gu8*>(a);
        const uint32_t stored = uint32_t(q[0]) | (uint32_t(q[1]) << 8) | (uint32_t(q[2]) << 16) |
                                (uint32_t(q[3]) << 24);
        if (res != stored)
            atomicAdd(&d.vstat[seg].bad_objects, 1u);
    }
}
