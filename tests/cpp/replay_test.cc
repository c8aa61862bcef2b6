// Crc32CBatch::deviceReplayVerify as a recovery master would call it: two
// segments of object entries built with the drop-in Crc32C (the certificate
// of Segment::getAppendedLength, src/Segment.cc:672-684; the object checksum
// of Object::computeChecksum, src/Object.cc:805-819), one object damaged and
// the second segment's certificate wrong.  Built with hipcc for hipMalloc.
#include <stdio.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include <vector>

#include "Crc32C.h"
#include "Crc32CBatch.h"

using namespace RAMCloud;

static const uint32_t kCap = 64 * 1024;

// Fills `seg` with n objects of valueLen bytes; returns the certificate.
static ramcrc_seg_cert fill(uint8_t* seg, int n, uint32_t valueLen, uint32_t seed)
{
    Crc32C meta;
    uint32_t pos = 0;
    for (int k = 0; k < n; k++) {
        const uint32_t len = 24 + valueLen;           // Object::Header + keysAndValue
        const uint8_t hdr = 2 | (1 << 6);             // LOG_ENTRY_TYPE_OBJ, 2 length bytes
        seg[pos] = hdr;
        seg[pos + 1] = uint8_t(len);
        seg[pos + 2] = uint8_t(len >> 8);
        meta.update(&seg[pos], 3);
        uint8_t* obj = &seg[pos + 3];
        for (uint32_t i = 4; i < len; i++) {
            seed = seed * 1103515245u + 12345u;
            obj[i] = uint8_t(seed >> 16);
        }
        const uint32_t c = Crc32C().update(obj + 4, len - 4).getResult();
        memcpy(obj, &c, 4);
        pos += 3 + len;
    }
    ramcrc_seg_cert cert;
    cert.segment_length = pos;
    meta.update(&pos, 4);
    cert.checksum = meta.getResult();
    return cert;
}

int main()
{
    std::vector<uint8_t> host(2 * kCap, 0);
    ramcrc_seg_cert certs[2];
    certs[0] = fill(&host[0], 40, 1000, 7);
    certs[1] = fill(&host[kCap], 30, 700, 9);
    host[3 + 24 + 500] ^= 1;       // a value byte of segment 0's first object
    certs[1].checksum ^= 1;        // segment 1 fails its metadata check
    void *d_base, *d_certs, *d_status, *d_entries, *d_n, *d_crc;
    const uint64_t cap = 128;
    if (hipMalloc(&d_base, host.size()) || hipMalloc(&d_certs, sizeof certs) ||
        hipMalloc(&d_status, 2 * sizeof(ramcrc_seg_status)) ||
        hipMalloc(&d_entries, cap * sizeof(ramcrc_seg_entry)) || hipMalloc(&d_n, 8) ||
        hipMalloc(&d_crc, cap * 4)) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    if (hipMemcpy(d_base, &host[0], host.size(), hipMemcpyHostToDevice) ||
        hipMemcpy(d_certs, certs, sizeof certs, hipMemcpyHostToDevice)) {
        fprintf(stderr, "hipMemcpy failed\n");
        return 1;
    }
    Crc32CBatch batch(0);
    batch.deviceReplayVerify(d_base, kCap, kCap, 2, static_cast<ramcrc_seg_cert*>(d_certs),
                             static_cast<ramcrc_seg_status*>(d_status),
                             static_cast<ramcrc_seg_entry*>(d_entries), cap,
                             static_cast<uint64_t*>(d_n), static_cast<uint32_t*>(d_crc));
    ramcrc_seg_status st[2];
    if (hipMemcpy(st, d_status, sizeof st, hipMemcpyDeviceToHost)) {
        fprintf(stderr, "hipMemcpy failed\n");
        return 1;
    }
    int bad = 0;
    if (st[0].flags != RAMCRC_SEG_OK || st[0].checksum != certs[0].checksum ||
        st[0].entries != 40 || st[0].bad_objects != 1)
        bad++;
    if ((st[1].flags & RAMCRC_SEG_OK) || !(st[1].flags & RAMCRC_SEG_BAD_CHECKSUM) ||
        st[1].entries != 30 || st[1].bad_objects != 0)
        bad++;
    printf("replay verify: seg0 flags %u entries %u bad %u; seg1 flags %u entries %u bad %u; "
           "%d mismatches\n", st[0].flags, st[0].entries, st[0].bad_objects, st[1].flags,
           st[1].entries, st[1].bad_objects, bad);
    return bad ? 1 : 0;
}
