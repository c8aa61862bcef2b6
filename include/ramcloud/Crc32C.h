/* Drop-in replacement for RAMCloud's src/Crc32C.h.
 *
 * Same class, same members, same semantics as the reference
 * (src/Crc32C.h:167-260): callers such as src/Segment.cc:211,218,677-681,
 * src/Object.cc:770-819, src/BackupMasterRecovery.h:539-556 and
 * src/AbstractLog.cc (through Segment.h) compile against it unchanged, and
 * tests that read or poke `result` under EXPOSE_PRIVATES
 * (src/Crc32CTest.cc:120, src/ReplicatedSegmentTest.cc:760) keep working.
 *
 * update() stays synchronous on the caller's thread and never touches a GPU:
 * it calls the host path of libramcrc (include/ramcrc.h).  Batches of whole
 * segments / log entries opt into the MI355X kernels through
 * ramcloud/Crc32CBatch.h instead.
 *
 * No HIP or ROCm header is included here: this is an installed client header
 * in RAMCloud (GNUmakefile:443).
 */
#ifndef RAMCLOUD_CRC32C_H
#define RAMCLOUD_CRC32C_H

#include <stdint.h>

#include "Buffer.h"
#if defined(__has_include)
#if __has_include("Exception.h")
#include "Exception.h"   // as the reference header does (src/Crc32C.h:22)
#endif
#endif
#include "ramcrc.h"

#ifndef PRIVATE
#define PRIVATE private
#endif

/// The software path's lookup tables under the reference's names and types
/// (src/Crc32C.h:25-34): plain arrays, so objects compiled against the
/// reference header link against them too.  Defined (generated from the
/// polynomial at compile time, statically initialised) in
/// ramcloud_amd/dropin/Crc32C.cc; libramcrc's own copies
/// (ramcrc_slice8_tables) hold the same values.
namespace Crc32CSlicingBy8 {
extern const uint32_t crc_tableil8_o32[256];
extern const uint32_t crc_tableil8_o40[256];
extern const uint32_t crc_tableil8_o48[256];
extern const uint32_t crc_tableil8_o56[256];
extern const uint32_t crc_tableil8_o64[256];
extern const uint32_t crc_tableil8_o72[256];
extern const uint32_t crc_tableil8_o80[256];
extern const uint32_t crc_tableil8_o88[256];
}  // namespace Crc32CSlicingBy8

namespace RAMCloud {

/// The hardware CRC step of src/Crc32C.h:39-93: state in, state out, no
/// inversion (SSE4.2 crc32 with three interleaved chains in libramcrc).
static inline uint32_t
intelCrc32C(uint32_t crc, const void* buffer, uint64_t bytes)
{
    return ramcrc_update_hw(crc, buffer, bytes);
}

/// The table-driven CRC step of src/Crc32C.h:96-153 (slicing-by-8).
static inline uint32_t
softwareCrc32C(uint32_t crc, const void* data, uint64_t length)
{
    return ramcrc_update_sw(crc, data, length);
}

/**
 * CRC32C (Castagnoli polynomial, as used by iSCSI) accumulated over any
 * number of update() calls.  The running value starts at 0xFFFFFFFF and is
 * inverted only when read through getResult(), which leaves it untouched so
 * callers may keep updating (src/LogDigest.cc:75-80) or copy a running
 * checksum and extend the copy (src/Segment.cc:677-681).
 *
 * The hardware path uses the SSE4.2 crc32 instruction with three interleaved
 * chains; the software path is table-driven slicing-by-8.  Both produce the
 * same 32-bit values as the reference for every input.
 */
class Crc32C {
  public:
    /// Type of getResult(); swap-friendly alias kept from the reference.
    typedef uint32_t ResultType;

    /**
     * \param forceSoftware
     *      Use the table-driven path even when the CPU has a crc32
     *      instruction (the unit tests run both).
     */
    Crc32C(bool forceSoftware = false)
        : useHardware(!forceSoftware && haveHardware)
        , result(0xFFFFFFFFu)
    {
    }

    /// Copies only the accumulated value, like the reference's operator=.
    Crc32C&
    operator=(const Crc32C& other)
    {
        result = other.result;
        return *this;
    }

    /**
     * Fold `bytes` bytes at `buffer` into the checksum.
     * \return *this, so calls chain.
     */
    Crc32C&
    update(const void* buffer, uint32_t bytes)
    {
        result = useHardware ? ramcrc_update_hw(result, buffer, bytes)
                             : ramcrc_update_sw(result, buffer, bytes);
        return *this;
    }

    /**
     * Fold bytes [offset, offset+bytes) of a (possibly discontiguous)
     * Buffer into the checksum, one contiguous chunk at a time.
     */
    Crc32C&
    update(Buffer& buffer, uint32_t offset, uint32_t bytes)
    {
        for (Buffer::Iterator it(&buffer, offset, bytes); !it.isDone(); it.next())
            update(it.getData(), it.getLength());
        return *this;
    }

    /// Fold every byte of a Buffer into the checksum.
    Crc32C&
    update(Buffer& buffer)
    {
        return update(buffer, 0, buffer.size());
    }

    /// The checksum so far (the inverted running value); non-destructive.
    ResultType
    getResult() const
    {
        return ~result;
    }

  PRIVATE:
    /// Set once at static-initialisation time from ramcrc_cpu_has_hw().
    static bool haveHardware;

    /// Whether this instance uses the crc32 instruction.
    bool useHardware;

    /// The running checksum before the final inversion.
    uint32_t result;
};

} // namespace RAMCloud

#endif // RAMCLOUD_CRC32C_H
