/* Opt-in batch CRC32C on an MI355X for RAMCloud callers that hold many
 * independent buffers at once:
 *
 *   - the backup recovery scan: every loaded replica frame is a contiguous
 *     8 MiB buffer (BackupStorage::Frame::load, src/BackupStorage.h:227)
 *     verified independently in BackupMasterRecovery::CyclicReplicaBuffer::
 *     buildNext (src/BackupMasterRecovery.cc:743-809);
 *   - the recovery-master replay: one Object::computeChecksum per object of a
 *     recovery segment (src/ObjectManager.cc:659-663, src/Object.cc:805-819).
 *
 * Each call returns exactly what `Crc32C c; c.update(buf_i, len_i);
 * c.getResult()` returns for every buffer (or the raw running value, for
 * chaining), computed by libramcrc's gfx950 kernels.  Comparison against the
 * stored checksums stays with the caller, as in the reference
 * (src/Segment.cc:793-797, src/ObjectManager.cc:664-669).
 *
 * Errors from the C ABI (include/ramcrc.h) become RAMCRC_BATCH_THROW(msg),
 * which is `throw FatalError(HERE, msg)` inside RAMCloud (src/Exception.h:70)
 * and std::runtime_error elsewhere.  No HIP header is needed by callers.
 */
#ifndef RAMCLOUD_CRC32CBATCH_H
#define RAMCLOUD_CRC32CBATCH_H

#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

#include "ramcrc.h"

#ifndef RAMCRC_BATCH_THROW
#if defined(RAMCLOUD_EXCEPTION_H)
#define RAMCRC_BATCH_THROW(msg) throw RAMCloud::FatalError(HERE, msg)
#else
#include <stdexcept>
#define RAMCRC_BATCH_THROW(msg) throw std::runtime_error(msg)
#endif
#endif

namespace RAMCloud {

class Crc32CBatch {
  public:
    /// Binds to a GPU lazily on first use (never at static-init time).
    explicit Crc32CBatch(int device = 0)
        : device(device)
        , ctx(NULL)
    {
    }

    ~Crc32CBatch()
    {
        if (ctx)
            ramcrc_ctx_destroy(ctx);
    }

    /**
     * CRC32C of host buffers (e.g. loaded replica frames): staged through
     * pinned memory to the GPU and back.  Synchronous.
     * \param buffers
     *      (pointer, length) of every buffer.
     * \param finalize
     *      true: getResult() values; false: raw running values.
     */
    std::vector<uint32_t>
    hostBuffers(const std::vector<std::pair<const void*, uint64_t> >& buffers,
                bool finalize = true)
    {
        std::vector<const void*> ptrs;
        std::vector<uint64_t> lens;
        for (size_t i = 0; i < buffers.size(); i++) {
            ptrs.push_back(buffers[i].first);
            lens.push_back(buffers[i].second);
        }
        std::vector<uint32_t> out(buffers.size());
        if (!buffers.empty())
            check(ramcrc_batch_host(context(), &ptrs[0], &lens[0], NULL, &out[0],
                                    out.size(), finalize ? RAMCRC_FINALIZE : 0u),
                  "ramcrc_batch_host");
        return out;
    }

    /// Device-resident uniform segments (the recovery-scan batch): d_out[i]
    /// for segment i = d_base + i * segmentBytes.  With wait (the default)
    /// the call returns after the results are in d_out; wait = false leaves
    /// it asynchronous on `stream`, to be followed by sync(stream).
    void
    deviceSegments(const void* d_base, uint64_t segmentBytes, uint64_t count,
                   uint32_t* d_out, void* stream = NULL, bool finalize = true, bool wait = true)
    {
        check(ramcrc_segments_device(context(), d_base, segmentBytes, count, NULL, d_out,
                                     finalize ? RAMCRC_FINALIZE : 0u, stream),
              "ramcrc_segments_device");
        if (wait)
            sync(stream);
    }

    /// Device-resident (offset, length) table, e.g. the (off + 4, len - 4)
    /// object ranges of a recovery segment.  wait: as for deviceSegments.
    /// A batch the context's scratch cannot plan (overlapping buffers
    /// totalling more than the device holds) throws instead of leaving
    /// d_out unwritten.
    void
    deviceBatch(const void* d_base, const uint64_t* d_off, const uint64_t* d_len,
                const uint32_t* d_init, uint32_t* d_out, uint64_t count, void* stream = NULL,
                bool finalize = true, bool wait = true)
    {
        check(ramcrc_batch_device(context(), d_base, d_off, d_len, d_init, d_out, count,
                                  finalize ? RAMCRC_FINALIZE : 0u, stream),
              "ramcrc_batch_device");
        if (wait)
            sync(stream);
    }

    /// Waits for `stream` and throws if a launch of this object was refused
    /// since the last sync (ramcrc_ctx_check): the outputs of a refused
    /// launch are not written, and an integrity path must not read them.
    void
    sync(void* stream = NULL)
    {
        check(ramcrc_ctx_check(context(), stream), "ramcrc_ctx_check");
    }

    /**
     * The checks a recovery master makes on a batch of replicas resident in
     * HBM: Segment::checkMetadataIntegrity of every segment
     * (src/Segment.cc:758-800), then every checkIntegrity replaySegment makes
     * on the entries of the segments that passed (src/ObjectManager.cc:580-1100).
     * Segment i = d_base + i * stride, `capacity` bytes.  d_status[i] gets the
     * flags, metadata checksum, entry count and failed checks; d_entries /
     * d_objCrc the walked records and their computed CRCs.  Returns after
     * both kernels finished on `stream` (see ramcrc_segment_walk_device /
     * ramcrc_verify_objects_device).  A segment whose records did not fit
     * in entriesCap carries RAMCRC_SEG_TABLE_FULL and never RAMCRC_SEG_OK:
     * it was not verified; walk it again with a larger table.
     */
    void
    deviceReplayVerify(const void* d_base, uint64_t stride, uint32_t capacity, uint64_t count,
                       const ramcrc_seg_cert* d_certs, ramcrc_seg_status* d_status,
                       ramcrc_seg_entry* d_entries, uint64_t entriesCap, uint64_t* d_nEntries,
                       uint32_t* d_objCrc, void* stream = NULL)
    {
        // walk + checks in one call (ramcrc_replay_verify_device): the same as
        // ramcrc_segment_walk_device then ramcrc_verify_objects_device
        check(ramcrc_replay_verify_device(context(), d_base, stride, capacity, count, d_certs,
                                          d_status, d_entries, entriesCap, d_nEntries, d_objCrc,
                                          stream),
              "ramcrc_replay_verify_device");
        sync(stream);
    }

    /**
     * Object::assembleForLog's checksum for a batch of serialized objects
     * (the write path, src/ObjectManager.cc:1274): header.checksum of every
     * object (Object::Header + keysAndValue, src/Object.h:137-182) is set to
     * Object::computeChecksum() (src/Object.cc:770-819), computed on the GPU.
     * Objects shorter than the header are left unchanged.  Synchronous.
     */
    void
    assembleObjects(const std::vector<std::pair<void*, uint64_t> >& objects)
    {
        std::vector<void*> ptrs;
        std::vector<uint64_t> lens;
        for (size_t i = 0; i < objects.size(); i++) {
            ptrs.push_back(objects[i].first);
            lens.push_back(objects[i].second);
        }
        if (!objects.empty())
            check(ramcrc_assemble_objects_host(context(), &ptrs[0], &lens[0], ptrs.size()),
                  "ramcrc_assemble_objects_host");
    }

  private:
    ramcrc_ctx*
    context()
    {
        if (!ctx)
            check(ramcrc_ctx_create(device, &ctx), "ramcrc_ctx_create");
        return ctx;
    }

    static void
    check(int rc, const char* what)
    {
        if (rc != RAMCRC_OK)
            RAMCRC_BATCH_THROW(std::string(what) + ": " + ramcrc_strerror(rc));
    }

    int device;
    ramcrc_ctx* ctx;

    Crc32CBatch(const Crc32CBatch&);             // not copyable
    Crc32CBatch& operator=(const Crc32CBatch&);
};

/**
 * The recovery-scan batch sharded across the GPUs of a node (ramcrc_shard_*,
 * SURVEY.md 8(e)): every rank scans the contiguous range of replicas that
 * sits in its own HBM and one RCCL all-gather of the 4-byte results leaves
 * all CRCs, in segment order, with every rank -- what
 * BackupMasterRecovery::CyclicReplicaBuffer::buildNext
 * (src/BackupMasterRecovery.cc:743-809) checks per replica, for a whole
 * batch at once.  Errors throw like Crc32CBatch's.
 */
class Crc32CShard {
  public:
    /// One process driving several GPUs (ncclCommInitAll).
    explicit Crc32CShard(const std::vector<int>& devices)
        : shard(NULL)
    {
        check(ramcrc_shard_create_all(devices.empty() ? NULL : &devices[0],
                                      static_cast<int>(devices.size()), &shard),
              "ramcrc_shard_create_all");
    }

    /// One process per GPU (ncclCommInitRank); every process passes the same
    /// uniqueId() bytes, produced by one of them.
    Crc32CShard(const std::vector<uint8_t>& id, int nranks, int rank, int device)
        : shard(NULL)
    {
        if (id.size() != RAMCRC_SHARD_ID_BYTES)
            RAMCRC_BATCH_THROW(std::string("Crc32CShard: unique id must be 128 bytes"));
        check(ramcrc_shard_create_rank(&id[0], nranks, rank, device, &shard),
              "ramcrc_shard_create_rank");
    }

    ~Crc32CShard()
    {
        if (shard)
            ramcrc_shard_destroy(shard);
    }

    static std::vector<uint8_t>
    uniqueId()
    {
        std::vector<uint8_t> id(RAMCRC_SHARD_ID_BYTES);
        check(ramcrc_shard_unique_id(&id[0]), "ramcrc_shard_unique_id");
        return id;
    }

    /// [first, last) of the segments rank `rank` of `nranks` owns.
    static std::pair<uint64_t, uint64_t>
    range(uint64_t segments, int nranks, int rank)
    {
        uint64_t lo = 0, hi = 0;
        check(ramcrc_shard_range(segments, nranks, rank, &lo, &hi), "ramcrc_shard_range");
        return std::make_pair(lo, hi);
    }

    /**
     * One recovery-scan step: dShard[k] (device memory of local rank k)
     * holds that rank's range() of `segments` replicas of segmentBytes each.
     * Returns the finalized CRCs of all segments, in segment order, as
     * gathered on local rank 0.  Synchronous.
     */
    std::vector<uint32_t>
    deviceShard(const std::vector<const void*>& dShard, uint64_t segmentBytes,
                uint64_t segments)
    {
        if (static_cast<int>(dShard.size()) != ramcrc_shard_local_count(shard))
            RAMCRC_BATCH_THROW(std::string("Crc32CShard: one buffer per local rank"));
        std::vector<uint32_t> out(segments);
        check(ramcrc_shard_segments(shard, dShard.empty() ? NULL : &dShard[0], segmentBytes,
                                    segments, NULL, RAMCRC_FINALIZE),
              "ramcrc_shard_segments");
        check(ramcrc_shard_sync(shard), "ramcrc_shard_sync");
        if (segments)
            check(ramcrc_shard_results(shard, 0, &out[0], segments), "ramcrc_shard_results");
        return out;
    }

  private:
    static void
    check(int rc, const char* what)
    {
        if (rc != RAMCRC_OK)
            RAMCRC_BATCH_THROW(std::string(what) + ": " + ramcrc_strerror(rc));
    }

    ramcrc_shard* shard;

    Crc32CShard(const Crc32CShard&);             // not copyable
    Crc32CShard& operator=(const Crc32CShard&);
};

} // namespace RAMCloud

#endif // RAMCLOUD_CRC32CBATCH_H
