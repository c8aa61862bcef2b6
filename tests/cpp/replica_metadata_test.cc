// The drop-in Crc32C (include/ramcloud/Crc32C.h) under two of the reference's
// own caller structures:
//
//  * SegmentCertificate, taken from the reference's src/LogMetadata.h when
//    the build has its headers (-DREF_HEADERS -I/root/reference/src; the
//    include guard of that header's own `#include "Crc32C.h"` then resolves
//    to the drop-in, exactly as when the drop-in replaces src/Crc32C.h),
//    otherwise an 8-byte packed stand-in with the same layout;
//  * BackupReplicaMetadata (src/BackupMasterRecovery.h:517-628): a packed
//    42-byte record sealed with the CRC32C of its first 38 bytes.  Its header
//    pulls in the whole backup service, so the record is restated here with
//    the reference's field order, types and packing.
//
// With PROBE_BUFFER (compile-only, -fsyntax-only) the Buffer overloads of
// update() are instantiated against the reference's real src/Buffer.h.
//
// Output, one line per sealed record:  "meta <42 bytes hex> <checksum hex>",
// and per certificate: "cert <stream hex> <length> <checksum hex>"; the
// Python test recomputes every checksum with the oracle.
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "Crc32C.h"

#ifdef REF_HEADERS
#include "LogMetadata.h"
#else
namespace RAMCloud {
class SegmentCertificate {
  public:
    SegmentCertificate() : segmentLength(), checksum() {}
    uint32_t segmentLength;
    Crc32C::ResultType checksum;
} __attribute__((__packed__));
}  // namespace RAMCloud
#endif

namespace RAMCloud {

// Restated from src/BackupMasterRecovery.h:517-628 (fields, order, packing).
class BackupReplicaMetadata {
  public:
    BackupReplicaMetadata(const SegmentCertificate& certificate, uint64_t logId,
                          uint64_t segmentId, uint32_t segmentCapacity, uint64_t segmentEpoch,
                          bool closed, bool primary)
        : certificate(certificate), logId(logId), segmentId(segmentId),
          segmentCapacity(segmentCapacity), segmentEpoch(segmentEpoch), closed(closed),
          primary(primary), checksum()
    {
        checksum = seal();
    }

    bool checkIntegrity() const { return seal() == checksum; }

    Crc32C::ResultType seal() const
    {
        Crc32C c;
        c.update(this, static_cast<unsigned>(sizeof(*this) - sizeof(checksum)));
        return c.getResult();
    }

    SegmentCertificate certificate;
    uint64_t logId;
    uint64_t segmentId;
    uint32_t segmentCapacity;
    uint64_t segmentEpoch;
    bool closed;
    bool primary;
    Crc32C::ResultType checksum;
} __attribute__((packed));

static_assert(sizeof(SegmentCertificate) == 8, "SegmentCertificate layout");
static_assert(sizeof(BackupReplicaMetadata) == 42, "BackupReplicaMetadata layout");

#ifdef PROBE_BUFFER
// Buffer overloads of the drop-in against the reference's Buffer
// (src/Crc32C.h:219-242; Buffer::Iterator, src/Buffer.cc:838-975).
inline uint32_t
probeBuffer(Buffer& buffer)
{
    Crc32C a, b;
    a.update(buffer, 3, 100);
    b.update(buffer);
    Crc32C c(b);     // implicit copy (src/Segment.cc:677)
    c = a;           // operator= copies the running value only
#ifdef EXPOSE_PRIVATES
    c.result ^= 1;   // tests poke the running value (src/Crc32CTest.cc:120)
#endif
    return a.getResult() ^ b.getResult() ^ c.getResult();
}
#endif

}  // namespace RAMCloud

using namespace RAMCloud;

static void
hex(const void* p, size_t n)
{
    const uint8_t* b = static_cast<const uint8_t*>(p);
    for (size_t i = 0; i < n; i++)
        printf("%02x", b[i]);
}

int
main()
{
    int failures = 0;
    // Segment certificates as Segment::getAppendedLength builds them
    // (src/Segment.cc:672-684): the running metadata CRC of the entry
    // headers and lengths, extended by segmentLength.  Streams of the
    // SegmentTest goldens (src/SegmentTest.cc:159,369,373).
    // the entries: EntryHeader (LOG_ENTRY_TYPE_OBJ... as the test appends)
    // and a 1-byte length of the 2- and 3-byte payloads "hi" and "yo!"
    const char* streams[3] = {"", "\x02\x02", "\x02\x03"};
    const uint32_t lengths[3] = {0, 4, 5};
    for (int i = 0; i < 3; i++) {
        SegmentCertificate cert;
        cert.segmentLength = lengths[i];
        Crc32C meta;
        meta.update(streams[i], static_cast<uint32_t>(strlen(streams[i])));
        Crc32C copy(meta);   // fork-and-extend, src/Segment.cc:677-681
        copy.update(&cert.segmentLength, sizeof(cert.segmentLength));
        const uint32_t ck = copy.getResult();   // checksum is PRIVATE in the reference's class
        memcpy(reinterpret_cast<uint8_t*>(&cert) + 4, &ck, 4);
        printf("cert ");
        hex(streams[i], strlen(streams[i]));
        printf(" %u %08x\n", lengths[i], copy.getResult());
    }
    // Replica metadata records over a spread of field values.
    uint64_t x = 0x243F6A8885A308D3ull;
    for (int i = 0; i < 64; i++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        SegmentCertificate cert;
        cert.segmentLength = static_cast<uint32_t>(x >> 7);
        const uint32_t cck = static_cast<uint32_t>(x >> 29);
        memcpy(reinterpret_cast<uint8_t*>(&cert) + 4, &cck, 4);
        BackupReplicaMetadata m(cert, x >> 3, x ^ (x >> 17), 8u << 20, (x >> 40) + i, i & 1,
                                (i >> 1) & 1);
        if (!m.checkIntegrity())
            failures++;
        BackupReplicaMetadata damaged = m;
        reinterpret_cast<uint8_t*>(&damaged)[i % 38] ^= static_cast<uint8_t>(1u << (i % 8));
        if (damaged.checkIntegrity())
            failures++;   // any single-bit flip of a sealed field is caught
        printf("meta ");
        hex(&m, sizeof(m));
        printf(" %08x\n", m.checksum);
    }
    printf("failures=%d\n", failures);
    return failures ? 1 : 0;
}
