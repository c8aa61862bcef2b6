// RecoverSegmentBenchmark-shaped segments built on the device
// (ramcrc_segment_fill_objects_device, include/ramcrc.h).
//
// nanobenchmarks/RecoverSegmentBenchmark.cc:123-146 fills every segment with
// objects {tableId 0, 8-byte counter key, version 0, timestamp 0, value}
// until the next one does not fit.  Every entry of a segment has the same
// size, so entry j of segment i sits at j * entryBytes and the layout is a
// pure function of (i, j): one thread writes one entry's EntryHeader, length
// bytes and object header + key (src/Segment.h:99-112, src/Object.h:137-182,
// src/Object.cc:107-141, 213-218), the batch kernels compute every
// Object::Header::checksum (ramcrc_assemble_objects_device), and the
// certificate -- which covers only entry headers, lengths and the segment
// length, identical for every segment -- comes from the host append path
// (ramcrc_segment_fill_objects) run once on a scratch segment, so both
// paths agree byte for byte by construction.
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include "ramcrc.h"

namespace {

struct FillDesc {
    uint8_t* base;
    uint64_t stride;
    uint64_t per;         // objects per segment
    uint64_t nobj;        // per * nseg
    uint32_t entry;       // bytes per entry
    uint32_t objlen;      // bytes per object
    uint32_t lb;          // length bytes
    uint64_t first_key;
    uint64_t* off;        // object offsets from base (for the checksum batch)
    uint64_t* len;
};

__global__ __launch_bounds__(256) void k_fill_headers(FillDesc f)
{
    const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= f.nobj)
        return;
    const uint64_t seg = t / f.per, j = t - seg * f.per;
    uint8_t* e = f.base + seg * f.stride + j * f.entry;
    e[0] = uint8_t(RAMCRC_LOG_ENTRY_TYPE_OBJ | ((f.lb - 1) << 6));
    for (uint32_t k = 0; k < f.lb; k++)
        e[1 + k] = uint8_t(f.objlen >> (8 * k));
    uint8_t* o = e + 1 + f.lb;
    for (int k = 0; k < 24; k++)    // checksum (stamped later), timestamp, version, tableId
        o[k] = 0;
    o[24] = 1;                      // KeyCount
    o[25] = 8;                      // CumulativeKeyLength, little-endian
    o[26] = 0;
    const uint64_t key = f.first_key + t;   // keys continue across segments
    for (int k = 0; k < 8; k++)
        o[27 + k] = uint8_t(key >> (8 * k));
    f.off[t] = uint64_t(o - f.base);
    f.len[t] = f.objlen;
}

__global__ __launch_bounds__(256) void k_fill_tails(uint8_t* base, uint64_t stride, uint64_t head,
                                                    uint64_t capacity, uint64_t nseg)
{
    // zero [head, capacity) of every segment, one thread per 16 bytes where
    // aligned, bytes at the ragged ends
    const uint64_t tail = capacity - head;
    const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t per_seg = (tail + 15) / 16;
    if (t >= per_seg * nseg)
        return;
    const uint64_t seg = t / per_seg, q = t - seg * per_seg;
    uint8_t* p = base + seg * stride + head;
    const uint64_t a = q * 16, b = a + 16 < tail ? a + 16 : tail;
    for (uint64_t k = a; k < b; k++)
        p[k] = 0;
}

__global__ __launch_bounds__(256) void k_fill_certs(ramcrc_seg_cert* certs, ramcrc_seg_cert c,
                                                    uint64_t nseg)
{
    const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t < nseg)
        certs[t] = c;
}

int fill_on_device(ramcrc_ctx* ctx, uint8_t* base, uint64_t seg_stride, uint32_t capacity,
                   uint64_t n_seg, uint32_t value_len, uint64_t first_key, uint32_t per,
                   ramcrc_seg_cert* d_certs, ramcrc_seg_cert cert);

}  // namespace

extern "C" int ramcrc_segment_fill_objects_device(ramcrc_ctx* ctx, void* d_base,
                                                  uint64_t seg_stride, uint32_t capacity,
                                                  uint64_t n_seg, uint32_t value_len,
                                                  uint64_t first_key, ramcrc_seg_cert* d_certs,
                                                  ramcrc_seg_cert* h_cert, uint32_t* h_objects)
{
    if (!ctx || !h_cert || (n_seg && !d_base) || (n_seg > 1 && seg_stride < capacity))
        return RAMCRC_EINVAL;
    // The host append path on one scratch segment: certificate and count.
    uint8_t* scratch = static_cast<uint8_t*>(calloc(capacity ? capacity : 1, 1));
    if (!scratch)
        return RAMCRC_ENOMEM;
    uint32_t per = 0;
    int rc = ramcrc_segment_fill_objects(scratch, capacity, value_len, first_key, &per, h_cert);
    free(scratch);
    if (rc)
        return rc;
    if (h_objects)
        *h_objects = per;
    if (n_seg == 0)
        return RAMCRC_OK;
    // launch on the device that holds the segments
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, d_base) != hipSuccess || attr.type != hipMemoryTypeDevice)
        return RAMCRC_EINVAL;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(attr.device) != hipSuccess)
        return RAMCRC_ENODEV;
    rc = fill_on_device(ctx, static_cast<uint8_t*>(d_base), seg_stride, capacity, n_seg,
                        value_len, first_key, per, d_certs, *h_cert);
    (void)hipSetDevice(prev);
    return rc;
}

namespace {

int fill_on_device(ramcrc_ctx* ctx, uint8_t* base, uint64_t seg_stride, uint32_t capacity,
                   uint64_t n_seg, uint32_t value_len, uint64_t first_key, uint32_t per,
                   ramcrc_seg_cert* d_certs, ramcrc_seg_cert cert)
{
    const uint32_t objlen = 24 + 1 + 2 + 8 + value_len;
    const uint32_t lb = objlen < 0x100u ? 1 : objlen < 0x10000u ? 2 : objlen < 0x1000000u ? 3 : 4;
    const uint32_t entry = 1 + lb + objlen;
    const uint64_t nobj = uint64_t(per) * n_seg;
    uint64_t* d_tab = nullptr;
    if (nobj && hipMalloc(reinterpret_cast<void**>(&d_tab), 2 * nobj * sizeof(uint64_t)) != hipSuccess)
        return RAMCRC_ENOMEM;
    int rc = RAMCRC_OK;
    hipStream_t s = nullptr;
    if (nobj) {
        FillDesc f{base, seg_stride, per, nobj, entry, objlen, lb, first_key, d_tab, d_tab + nobj};
        hipLaunchKernelGGL(k_fill_headers, dim3((nobj + 255) / 256), dim3(256), 0, s, f);
        if (hipGetLastError() != hipSuccess)
            rc = RAMCRC_EHIP;
    }
    const uint64_t head = uint64_t(per) * entry;
    if (!rc && head < capacity) {
        const uint64_t items = (capacity - head + 15) / 16 * n_seg;
        hipLaunchKernelGGL(k_fill_tails, dim3((items + 255) / 256), dim3(256), 0, s, base,
                           seg_stride, head, uint64_t(capacity), n_seg);
        if (hipGetLastError() != hipSuccess)
            rc = RAMCRC_EHIP;
    }
    if (!rc && d_certs) {
        hipLaunchKernelGGL(k_fill_certs, dim3((n_seg + 255) / 256), dim3(256), 0, s, d_certs,
                           cert, n_seg);
        if (hipGetLastError() != hipSuccess)
            rc = RAMCRC_EHIP;
    }
    if (!rc && nobj)
        rc = ramcrc_assemble_objects_device(ctx, base, d_tab, d_tab + nobj, nullptr, nobj, s);
    if (!rc)
        rc = ramcrc_ctx_check(ctx, s);   // waits for the stamping; refused -> error
    if (hipDeviceSynchronize() != hipSuccess && !rc)
        rc = RAMCRC_EHIP;
    if (d_tab)
        (void)hipFree(d_tab);
    return rc;
}

}  // namespace
