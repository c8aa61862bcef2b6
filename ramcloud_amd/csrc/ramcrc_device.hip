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
//  * k_bin_* / k_entries -- small buffers (log entries, objects): binned by
//    128-byte step count, then a group of 8 lanes per entry; entries of one
//    window take the tiny phase (one position-table lookup per byte), longer
//    ones Horner with X^128.
//  * k_plan_* -- for the general offset/length table: per-entry chunk counts
//    and their exclusive prefix so waves can map a global chunk index to
//    (entry, chunk) with two binary searches.
//  * k_seg_walk / k_walk_* -- Segment::checkMetadataIntegrity over whole
//    segments, and the records the replay checks read.
//
// The kernels live in per-family parts included below, in this order, into
// this one translation unit (shared __device__ tables and LDS layouts, no
// relocatable device code):
//   dev_common.inc   geometry, tables, LDS layouts, operators, descriptors
//   dev_chunks.inc   k_chunks, k_combine
//   dev_bins.inc     small-entry configuration, k_bin_count/_scatter/_one
//   dev_entries.inc  k_entries (tiny, multi-window and long phases)
//   dev_plan.inc     k_plan_count, k_plan_scan, status kernels
//   dev_host.inc     ramcrc_ctx and the host launch helpers
//   dev_walk.inc     k_seg_walk and the parallel walk (k_walk_*)
//   dev_checks.inc   k_obj_compare, k_obj_stamp, certificate kernels
// This file keeps the extern "C" entry points of include/ramcrc.h.
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

}  // namespace

#include "dev_common.inc"
#include "dev_chunks.inc"
#include "dev_bins.inc"
#include "dev_entries.inc"
#include "dev_plan.inc"
#include "dev_host.inc"
#include "dev_walk.inc"
#include "dev_checks.inc"

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
#ifndef RAMCRC_DEFINES
#define RAMCRC_DEFINES "none"   // build.py: the -D knobs of a variant build (variants.py)
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
           " large_min=64KiB part_shift=" RAMCRC_STR(RAMCRC_PART_SHIFT)
           " defines=" RAMCRC_DEFINES;
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
    if (c->walk_left) (void)hipFree(c->walk_left);
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
    case RAMCRC_OPT_BIN_ONE:
        c->bin_one = value != 0;
        return RAMCRC_OK;
    case RAMCRC_OPT_VERIFY_IN_WALK:
        if (value < 0 || value > 2)
            return RAMCRC_EINVAL;
        c->verify_in_walk = int(value);
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
    // count[kNB], then cursor[0][kNB], cursor[1][kNB], then hist[0], hist[1] (as uint64),
    // the k_bin_one rescues
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
    if (!c || !d_out || (!d_base && nseg && seg_bytes) || (flags & ~RAMCRC_FINALIZE))
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
    if (flags & ~RAMCRC_FINALIZE)
        return RAMCRC_EINVAL;   // unknown flag bits (2 was the removed RAMCRC_ORDERED)
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
    if (flags & ~RAMCRC_FINALIZE)
        return RAMCRC_EINVAL;   // unknown flag bits (2 was the removed RAMCRC_ORDERED)
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
    if (!c || (n && (!ptrs || !lens || !out)) || (flags & ~RAMCRC_FINALIZE))
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
    if (!c || !h_base || !h_out || batch < 1 || depth < 1 || seg_bytes == 0 ||
        (flags & ~RAMCRC_FINALIZE))
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
              hipStream_t s, uint32_t* sum, uint32_t* d_obj_crc = nullptr);
int verify_impl(ramcrc_ctx* c, const void* d_base, uint64_t seg_stride,
                const ramcrc_seg_entry* d_entries, uint64_t entries_cap, const uint64_t* d_n_entries,
                uint32_t* d_obj_crc, ramcrc_seg_status* d_status, hipStream_t s, const uint32_t* sum,
                uint64_t n_seg = 0);
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
                   entries_cap, d_n_entries, s, c->walk_sum,
                   entries_cap && c->verify_in_walk ? d_obj_crc : nullptr);
    if (rc || n_seg == 0)
        return rc;
    return verify_impl(c, d_base, seg_stride, d_entries, entries_cap, d_n_entries, d_obj_crc,
                       d_status, s, c->walk_sum, n_seg);
}

namespace {
int walk_impl(ramcrc_ctx* c, const void* d_base, uint64_t seg_stride, uint32_t seg_capacity,
              uint64_t n_seg, const ramcrc_seg_cert* d_certs, ramcrc_seg_status* d_status,
              ramcrc_seg_entry* d_entries, uint64_t entries_cap, uint64_t* d_n_entries,
              hipStream_t s, uint32_t* sum, uint32_t* d_obj_crc)
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
        const uint32_t pshift = c->walk_pshift ? c->walk_pshift : kPartShiftLow;
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
            rc = grow_device(reinterpret_cast<void**>(&c->walk_pool_used), &c->walk_pool_used_cap, 3,
                             sizeof(unsigned long long));   // [1]: the part shift word, [2]: k_left's count
        // verify-in-walk mode (fused call): the list of records k_left checks
        const uint64_t left_cap = entries_cap / 8 + 65536 < entries_cap ? entries_cap / 8 + 65536 : entries_cap;
        if (!rc && d_obj_crc && sum)
            rc = grow_device(reinterpret_cast<void**>(&c->walk_left), &c->walk_left_cap, left_cap,
                             sizeof(uint32_t));
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
        if (d_obj_crc && sum) {
            pw.obj_crc = d_obj_crc;
            pw.left = c->walk_left;
            pw.nleft = c->walk_pool_used + 2;
            pw.left_cap = left_cap;
            pw.vmode = uint32_t(c->verify_in_walk);
        }
        // The pool block map starts empty on every call: the part -> block
        // table (blocks) and the block -> part table (pool_owner) of the
        // previous call on this context are stale, and the fix-up's block
        // replacement reads them.  Carried over, they gave wrong records on a
        // repeated call when the fix-up re-walked parts with pool blocks
        // (replay of 2 and 3 KiB values, 256 KiB parts: records of one part's
        // pool block replaced by another's, found in round 6 by the bench's
        // object-CRC check, tests/test_gpu_replay_fused.py::
        // test_repeated_calls_pool_blocks).
        HIPCHK(hipMemsetAsync(c->walk_blocks, 0xFF, total * kMaxBlocks * sizeof(uint32_t), s));
        HIPCHK(hipMemsetAsync(c->walk_pool_owner, 0xFF, pool_blocks * sizeof(uint32_t), s));
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
        if (pw.obj_crc) {   // verify-in-walk mode, decided by k_walk_probe (else it exits)
            uint64_t gv = (total + kVWaves - 1) / kVWaves;   // a wave per part
            if (gv > uint64_t(16) * c->ncu)
                gv = uint64_t(16) * c->ncu;
            // (the probe picks the stage size; the other instantiation exits).
            // Timed with the scan kernels: in this mode they do the object
            // checks k_entries does otherwise.
            {
                ScanTimer t(c, s);
                t.launch(k_walk_copyv<kVStageS>, dim3(gv), dim3(kVWaves * kWaveSize), pw);
            }
            HIPCHK(hipGetLastError());
            {
                ScanTimer t(c, s);
                t.launch(k_walk_copyv<kVStageL>, dim3(gv), dim3(kVWaves * kWaveSize), pw);
            }
            HIPCHK(hipGetLastError());
        }
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
                uint32_t* d_obj_crc, ramcrc_seg_status* d_status, hipStream_t s, const uint32_t* sum,
                uint64_t n_seg)
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
    d.vstat = d_status;
    d.rec = reinterpret_cast<const u32x4*>(d_entries);
    d.n_dev = d_n_entries;
    d.seg_status = reinterpret_cast<const u32x4*>(d_status);
    d.out = d_obj_crc;
    d.flags = RAMCRC_FINALIZE;
    if (sum && c->walk_left && !c->serial_walk) {
        // the fused call's verify-in-walk leftovers (exits unless k_walk_probe chose that mode)
        uint64_t gl = uint64_t(4) * c->ncu;
        hipLaunchKernelGGL(k_left, dim3(gl), dim3(256), 0, s, d, d_status, sum, c->walk_left,
                           reinterpret_cast<const unsigned long long*>(c->walk_pool_used + 2),
                           c->walk_left_cap, n_seg);
        HIPCHK(hipGetLastError());
    }
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
