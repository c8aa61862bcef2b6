/*
 * ramcrc.h -- the C ABI of the MI355X-native CRC32C path (libramcrc.so).
 *
 * Plain C: no HIP, ROCm or torch types.  Device pointers are `const void*` /
 * `uint32_t*` into memory the caller allocated on the GPU; streams are passed
 * as `void*` (a hipStream_t; NULL = the legacy default stream).
 *
 * Semantics of every CRC entry point follow RAMCloud's Crc32C
 * (/root/reference/src/Crc32C.h):
 *   state 0xFFFFFFFF at construction            (src/Crc32C.h:175-179)
 *   update(p, n): state = CRC32C step, no ~      (src/Crc32C.h:200-206)
 *   getResult():  ~state, state unchanged        (src/Crc32C.h:247-249)
 * The batch entry points compute, for every buffer i,
 *   state_i = init ? init[i] : 0xFFFFFFFF;  state_i = update(buf_i, len_i)
 *   out[i]  = (flags & RAMCRC_FINALIZE) ? ~state_i : state_i
 * i.e. exactly `Crc32C c; c.result = init[i]; c.update(buf_i, len_i);`
 * followed by getResult() or a read of c.result.
 *
 * Errors: every int-returning function returns RAMCRC_OK (0) or a negative
 * code; nothing throws across this boundary.  The reference's update() cannot
 * fail (src/Crc32C.h:200-206); integrity failures stay with the caller, who
 * compares the returned per-buffer CRCs (src/Segment.cc:793-797).
 */
#ifndef RAMCRC_H
#define RAMCRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    RAMCRC_OK = 0,
    RAMCRC_EINVAL = -1,   /* bad argument (null pointer, size overflow) */
    RAMCRC_ENOMEM = -2,   /* device or pinned allocation failed */
    RAMCRC_EHIP = -3,     /* a HIP runtime call failed; see ramcrc_last_hip_error */
    RAMCRC_ENODEV = -4,   /* no usable gfx950 device */
    RAMCRC_ERCCL = -5,    /* RCCL failure or RCCL unavailable (multi-GPU shard) */
    RAMCRC_EREFUSED = -6, /* a launch found more chunks than the context's scratch holds and
                             wrote none of its outputs (see ramcrc_ctx_check) */
    RAMCRC_EINTERNAL = -7, /* a small-entry launch found its bin layout inconsistent with the
                             entries it binned and wrote none of its small-entry outputs.
                             Only a corrupted bin table produces it (the TEST_DIRTY_BINS
                             hook does so on purpose); scheduling cannot: a one-launch
                             binning whose grid is not all resident (other contexts'
                             kernels, preemption) falls back to the two-launch binning
                             inside the same call.  See ramcrc_ctx_check. */
    RAMCRC_EPEER = -8     /* multi-GPU shard: this rank's part of the step succeeded but
                             another rank's failed; that rank's segments read 0xFFFFFFFF */
    /* -9 was RAMCRC_EORDER of the ordered-stream batches, removed in round 5 */
};

/* Output flag: apply the final inversion (Crc32C::getResult, src/Crc32C.h:247).
 * Without it the raw running state (Crc32C::result, :259) is returned, which
 * callers use to keep chaining (src/LogDigest.cc:75-80, src/Segment.cc:677-681). */
#define RAMCRC_FINALIZE 1u
/* Any other flag bit is RAMCRC_EINVAL.  Round 4's RAMCRC_ORDERED (2) and its
 * ordered entry points were removed in round 5; a caller
 * built against that header gets EINVAL instead of a silently ignored flag.
 * RAMCRC_ABI_VERSION counts such removals. */
#define RAMCRC_ABI_VERSION 6

/* ---------------------------------------------------------------- host --- */

/* Replaces the body of Crc32C::update(const void*, uint32_t)
 * (src/Crc32C.h:200-206) when useHardware: SSE4.2 crc32 instruction,
 * three interleaved streams recombined with X^n operators.  Same result as
 * intelCrc32C (src/Crc32C.h:39-93) for every input.  64-bit length
 * (the reference takes uint32_t; see SURVEY.md section 7, hard part 6). */
uint32_t ramcrc_update_hw(uint32_t state, const void* data, uint64_t nbytes);

/* Replaces softwareCrc32C (src/Crc32C.h:96-153): slicing-by-8, tables
 * generated from the polynomial.  Used when forceSoftware or no SSE4.2. */
uint32_t ramcrc_update_sw(uint32_t state, const void* data, uint64_t nbytes);

/* Best available host path (what Crc32C::update uses by default). */
uint32_t ramcrc_update(uint32_t state, const void* data, uint64_t nbytes);

/* Replaces haveSse42()/Crc32C::haveHardware (src/Crc32C.cc:24-45):
 * 1 if this CPU and build support the crc32 instruction. */
int ramcrc_cpu_has_hw(void);

/* The eight slicing-by-8 tables ramcrc_update_sw uses, 8 x 256 words, table k
 * first: the values of the reference's Crc32CSlicingBy8::crc_tableil8_o32 ..
 * crc_tableil8_o88 (src/Crc32C.h:25-34, src/Crc32C.cc:108-537), generated from
 * the polynomial at compile time.  The drop-in header exposes them under the
 * reference's names. */
const uint32_t* ramcrc_slice8_tables(void);

/* State algebra.  ramcrc_shift(s, n) is the
 * state reached from s by updating with n zero bytes; ramcrc_combine(a, b, n)
 * = raw state of A||B given a = raw(0-based) state after A and b = raw(0, B)
 * with n = |B|.  Both are exact GF(2) identities. */
uint32_t ramcrc_shift(uint32_t state, uint64_t nbytes);
uint32_t ramcrc_combine(uint32_t raw_a, uint32_t raw_b, uint64_t len_b);

/* -------------------------------------------------------------- device --- */

typedef struct ramcrc_ctx ramcrc_ctx;

/* Creates a context bound to HIP device `device` (scratch buffers, pinned
 * staging, device properties).  No GPU work happens at static-init time;
 * contexts are created lazily by callers.  A context serialises its own
 * scratch: use one context per concurrently-launching thread/stream. */
int ramcrc_ctx_create(int device, ramcrc_ctx** out);
int ramcrc_ctx_destroy(ramcrc_ctx* ctx);

/* Pre-size device scratch so later launches never allocate (required before
 * capturing launches into a hipGraph).  max_chunks = number of 256 KiB chunks
 * a launch may cover; max_entries = entries of the largest batch call. */
int ramcrc_ctx_reserve(ramcrc_ctx* ctx, uint64_t max_chunks, uint64_t max_entries);

/* Uniform contiguous segments (the recovery-scan batch, src/BackupMasterRecovery.cc:743-809
 * per replica): segment i = d_base + i*seg_bytes, i < nseg.  d_init may be NULL.
 * Stream-ordered, asynchronous. */
int ramcrc_segments_device(ramcrc_ctx* ctx, const void* d_base, uint64_t seg_bytes,
                           uint64_t nseg, const uint32_t* d_init, uint32_t* d_out,
                           uint32_t flags, void* stream);

/* General batch: buffer i = d_base + d_off[i], length d_len[i] (64-bit, any
 * alignment, any length including 0).  Buffers of >= 64 KiB are split into
 * 256 KiB chunks scanned by all CUs; smaller ones go to the small-entry
 * kernel.  Stream-ordered, asynchronous. */
int ramcrc_batch_device(ramcrc_ctx* ctx, const void* d_base, const uint64_t* d_off,
                        const uint64_t* d_len, const uint32_t* d_init, uint32_t* d_out,
                        uint64_t n, uint32_t flags, void* stream);

/* Small-entry path only (log entries / objects, src/ObjectManager.cc:659-669):
 * every buffer through the per-entry kernel regardless of length. */
int ramcrc_entries_device(ramcrc_ctx* ctx, const void* d_base, const uint64_t* d_off,
                          const uint64_t* d_len, const uint32_t* d_init, uint32_t* d_out,
                          uint64_t n, uint32_t flags, void* stream);

/* Host buffers in, host CRCs out (segments arriving from disk/NIC buffers,
 * src/BackupStorage.h:227): pinned staging + H2D + kernel + D2H, synchronous.
 * ptrs[i]/lens[i] describe buffer i; init may be NULL. */
int ramcrc_batch_host(ramcrc_ctx* ctx, const void* const* ptrs, const uint64_t* lens,
                      const uint32_t* init, uint32_t* out, uint64_t n, uint32_t flags);

/* Streaming segments host-to-host with H2D on a copy stream overlapped with
 * kernels on a compute stream (BASELINE config 5).  Segment i = h_base +
 * i*seg_bytes (host memory, pinned or pageable); CRCs to h_out.  Uses up to
 * `depth` in-flight device slots of `batch` segments each. */
int ramcrc_stream_host(ramcrc_ctx* ctx, const void* h_base, uint64_t seg_bytes,
                       uint64_t nseg, uint32_t* h_out, uint32_t flags, int batch, int depth);

/* ------------------------------------------- recovery-segment verify --- */

/* SegmentCertificate (src/LogMetadata.h:85-128): 8 bytes, packed. */
typedef struct ramcrc_seg_cert {
    uint32_t segment_length;
    uint32_t checksum;
} ramcrc_seg_cert;

/* One walked log entry (src/Segment.h:99-195): `offset` is the entry's
 * EntryHeader byte within its segment, `header` that byte (type = header &
 * 0x3f, length bytes = ((header >> 6) & 3) + 1) plus RAMCRC_SEG_ENTRY_OVERLONG
 * when the payload would run past the segment capacity (reachable only
 * through the uint32_t offset wrap of the reference's walk), `length` the
 * payload length; the payload starts at offset + 1 + length bytes. */
#define RAMCRC_SEG_ENTRY_OVERLONG 0x100u
typedef struct ramcrc_seg_entry {
    uint32_t segment;
    uint32_t offset;
    uint32_t length;
    uint32_t header;
} ramcrc_seg_entry;

/* Per-segment result of the walk (and of the object verify). */
typedef struct ramcrc_seg_status {
    uint32_t flags;        /* RAMCRC_SEG_* */
    uint32_t checksum;     /* metadata checksum the walk computed (over the entries walked + length) */
    uint32_t entries;      /* entries walked */
    uint32_t bad_objects;  /* replay records whose checksum check failed: objects, tombstones,
                              safe versions and transaction records (see
                              ramcrc_verify_objects_device) */
} ramcrc_seg_status;

#define RAMCRC_SEG_OK 1u              /* Segment::checkMetadataIntegrity returned true */
#define RAMCRC_SEG_PAST_CAPACITY 2u   /* an entry ran past the segment capacity (src/Segment.cc:777-783) */
#define RAMCRC_SEG_PAST_LENGTH 4u     /* entries ran past certificate.segmentLength (:786-790) */
#define RAMCRC_SEG_BAD_CHECKSUM 8u    /* certificate checksum mismatch (:795-797) */
#define RAMCRC_SEG_TABLE_FULL 16u     /* entry table capacity exhausted: records of this segment
                                         were dropped, so it is NOT verified -- RAMCRC_SEG_OK is
                                         never set with this flag and none of its records are
                                         checked; size entries_cap for the smallest entry the
                                         segments can hold and walk again */
#define RAMCRC_SEG_CYCLE 32u          /* the walk revisited an offset (uint32_t wrap): the
                                         reference's loop would not terminate; stopped */
#define RAMCRC_LOG_ENTRY_TYPE_OBJ 2u          /* LOG_ENTRY_TYPE_OBJ, src/LogEntryTypes.h:35 */
#define RAMCRC_LOG_ENTRY_TYPE_OBJTOMB 3u      /* LOG_ENTRY_TYPE_OBJTOMB, src/LogEntryTypes.h:38 */
#define RAMCRC_LOG_ENTRY_TYPE_SAFEVERSION 5u  /* LOG_ENTRY_TYPE_SAFEVERSION, src/LogEntryTypes.h:44 */
#define RAMCRC_LOG_ENTRY_TYPE_PREP 8u         /* LOG_ENTRY_TYPE_PREP, src/LogEntryTypes.h:53 */
#define RAMCRC_LOG_ENTRY_TYPE_PREPTOMB 9u     /* LOG_ENTRY_TYPE_PREPTOMB, src/LogEntryTypes.h:56 */
#define RAMCRC_LOG_ENTRY_TYPE_TXDECISION 10u  /* LOG_ENTRY_TYPE_TXDECISION, src/LogEntryTypes.h:59 */
#define RAMCRC_LOG_ENTRY_TYPE_TXPLIST 11u     /* LOG_ENTRY_TYPE_TXPLIST, src/LogEntryTypes.h:62 */

/* Segment::checkMetadataIntegrity (src/Segment.cc:758-800) for n_seg segments
 * at d_base + i*seg_stride, each of seg_capacity bytes (a multiple of 16; the
 * reference's segletBlocks.size() * segletSize), against d_certs[i].  The
 * length-prefixed entries are walked in parallel over parts of every segment
 * (about 64 entries per part, 64 KiB .. 1 MiB, chosen per batch on the device from
 * the entry density; see RAMCRC_OPT_SERIAL_WALK, RAMCRC_OPT_WALK_PART_SHIFT).  Writes d_status[i] and one
 * ramcrc_seg_entry per complete entry to d_entries (up to entries_cap; the
 * order across segments is unspecified, within a segment it is increasing).  *d_n_entries (device) receives the
 * number of entries walked (may exceed entries_cap: see TABLE_FULL).
 * d_base 16-byte aligned, seg_stride a multiple of 16.  Stream-ordered. */
int ramcrc_segment_walk_device(ramcrc_ctx* ctx, const void* d_base, uint64_t seg_stride,
                               uint32_t seg_capacity, uint64_t n_seg,
                               const ramcrc_seg_cert* d_certs, ramcrc_seg_status* d_status,
                               ramcrc_seg_entry* d_entries, uint64_t entries_cap,
                               uint64_t* d_n_entries, void* stream);

/* Certificates of rebuilt segments (second half): a
 * backup seals every recovery segment it rebuilt with
 * Segment::getAppendedLength (src/Segment.cc:672-684, called at
 * src/BackupMasterRecovery.cc:367-368 for the segments
 * RecoverySegmentBuilder::build appended, src/RecoverySegmentBuilder.cc:195).
 * For n_seg segments at d_base + i*seg_stride (seg_capacity bytes each, the
 * walk's geometry rules) whose entries were appended from offset 0 up to
 * d_heads[i] (Segment::head), writes d_certs[i] = {head, checksum}: the
 * running Crc32C over every entry's header byte and length bytes, then over
 * the 4 head bytes, finalized -- the metadata the walk covers.  d_flags
 * (nullable) receives RAMCRC_SEG_OK when the entries end exactly at the head,
 * else the walk's RAMCRC_SEG_PAST_CAPACITY / _PAST_LENGTH / _CYCLE findings
 * (the certificate then covers the entries the walk read).  Stream-ordered. */
int ramcrc_segments_certify_device(ramcrc_ctx* ctx, const void* d_base, uint64_t seg_stride,
                                   uint32_t seg_capacity, uint64_t n_seg, const uint32_t* d_heads,
                                   ramcrc_seg_cert* d_certs, uint32_t* d_flags, void* stream);

/* ObjectManager::replaySegment's checksum checks for every record of a walk
 * whose segment passed the metadata check (d_status flags RAMCRC_SEG_OK;
 * records of failed segments are skipped, as RecoverySegmentBuilder::build
 * stops there):
 *   LOG_ENTRY_TYPE_OBJ          Object::computeChecksum (src/Object.cc:805-819)
 *                               over payload bytes [4, length) vs. the stored
 *                               checksum at [0, 4) (src/ObjectManager.cc:659-669);
 *   LOG_ENTRY_TYPE_OBJTOMB      ObjectTombstone::checkIntegrity
 *                               (src/ObjectManager.cc:752-758): bytes [0, 28) and
 *                               the key [32, length) vs. the checksum at [28, 32);
 *   LOG_ENTRY_TYPE_SAFEVERSION  ObjectSafeVersion::checkIntegrity
 *                               (src/ObjectManager.cc:873-880): bytes [0, 8) vs.
 *                               the checksum at [8, 12);
 *   LOG_ENTRY_TYPE_PREP         PreparedOp::checkIntegrity (src/ObjectManager.cc:956,
 *                               src/PreparedOp.cc:177-190): header bytes [0, 28)
 *                               and the object from its byte 4, [36, length), vs.
 *                               the checksum at [28, 32);
 *   LOG_ENTRY_TYPE_PREPTOMB     PreparedOpTombstone::checkIntegrity (:1013,
 *                               src/PreparedOp.cc:271-282): bytes [0, 40) vs. [40, 44);
 *   LOG_ENTRY_TYPE_TXDECISION   TxDecisionRecord::checkIntegrity (:1060,
 *                               src/TxDecisionRecord.cc:209-223): bytes [0, 44) and
 *                               24 * participantCount (uint32, at [36, 40)) bytes
 *                               from 48, clipped to the entry as Buffer::Iterator
 *                               does, vs. the checksum at [44, 48);
 *   LOG_ENTRY_TYPE_TXPLIST      ParticipantList::checkIntegrity (:1084,
 *                               src/ParticipantList.cc:96-110): bytes [0, 20) and
 *                               24 * participantCount (uint32, at [16, 20)) bytes
 *                               from 24 vs. the checksum at [20, 24); a list
 *                               longer than the entry fails (the reference's
 *                               getRange returns NULL there).
 * The computed CRC goes to d_obj_crc[i] (other records: not written), and
 * d_status[segment].bad_objects += 1 per failed check (records shorter than
 * their type's header, 24 / 32 / 12 / 56 / 44 / 48 / 24 bytes, or flagged
 * OVERLONG fail).  Objects of >= 64 KiB are scanned by all CUs, smaller ones
 * by the small-entry kernels; the other types by one thread each.  Stream-ordered
 * after the walk that produced the table. */
int ramcrc_verify_objects_device(ramcrc_ctx* ctx, const void* d_base, uint64_t seg_stride,
                                 const ramcrc_seg_entry* d_entries, uint64_t entries_cap,
                                 const uint64_t* d_n_entries, uint32_t* d_obj_crc,
                                 ramcrc_seg_status* d_status, void* stream);

/* The walk and the checks above in one call, as a recovery master replays a
 * batch of segments right after walking them (RecoverySegmentBuilder::build
 * then ObjectManager::replaySegment, src/RecoverySegmentBuilder.cc:61-203,
 * src/ObjectManager.cc:585-1115): exactly ramcrc_segment_walk_device
 * followed by ramcrc_verify_objects_device on the table it wrote (same
 * arguments, same results, same record table), with one shortcut the split
 * calls cannot take -- the walk notes whether any record it writes needs more
 * than the one-window object path (a larger object, or a tombstone, safe
 * version or transaction record), and when none does (RecoverSegmentBenchmark's
 * small-value segments) the checks skip the binning pass over the table.
 * Stream-ordered. */
int ramcrc_replay_verify_device(ramcrc_ctx* ctx, const void* d_base, uint64_t seg_stride,
                                uint32_t seg_capacity, uint64_t n_seg,
                                const ramcrc_seg_cert* d_certs, ramcrc_seg_status* d_status,
                                ramcrc_seg_entry* d_entries, uint64_t entries_cap,
                                uint64_t* d_n_entries, uint32_t* d_obj_crc, void* stream);

/* Host append path (src/Segment.cc:197-228 with src/Object.cc:213-218):
 * appends LOG_ENTRY_TYPE_OBJ entries holding objects {tableId 0, key = 8-byte
 * counter from first_key, version 0, timestamp 0, value_len value bytes} to an
 * empty segment of `capacity` bytes until the next one does not fit, as
 * RecoverSegmentBenchmark::run fills its segments
 * (nanobenchmarks/RecoverSegmentBenchmark.cc:131-146).  The value bytes are
 * whatever `seg` already holds at their positions; bytes after the last entry
 * are zeroed.  Writes the certificate (Segment::getAppendedLength,
 * src/Segment.cc:672-684) and the object count. */
int ramcrc_segment_fill_objects(uint8_t* seg, uint32_t capacity, uint32_t value_len,
                                uint64_t first_key, uint32_t* n_objects, ramcrc_seg_cert* cert);

/* Device form of ramcrc_segment_fill_objects for n_seg segments at d_base +
 * i*seg_stride (RecoverSegmentBenchmark::run's input, the BASELINE C4 shard,
 * built where it is scanned): segment i holds keys first_key + i*per ..
 * first_key + (i+1)*per - 1, per = objects per segment; value bytes are
 * whatever the segments already hold; bytes after the last entry are zeroed;
 * every Object::Header::checksum is computed by the batch kernels.  The
 * layout equals ramcrc_segment_fill_objects' byte for byte.  Every segment
 * gets the same certificate (the metadata checksum covers only entry headers
 * and lengths): written to *h_cert, to d_certs[i] when d_certs (device) is
 * not NULL, and per to *h_objects.  seg_stride >= capacity.  Synchronous. */
int ramcrc_segment_fill_objects_device(ramcrc_ctx* ctx, void* d_base, uint64_t seg_stride,
                                       uint32_t capacity, uint64_t n_seg, uint32_t value_len,
                                       uint64_t first_key, ramcrc_seg_cert* d_certs,
                                       ramcrc_seg_cert* h_cert, uint32_t* h_objects);

/* ------------------------------------------- multi-GPU recovery shard --- */

/* The recovery-scan batch sharded across GPUs: a backup's
 * replicas are verified independently (BackupMasterRecovery::
 * CyclicReplicaBuffer::buildNext, src/BackupMasterRecovery.cc:743-809), so
 * rank r of N scans the contiguous segment range ramcrc_shard_range(nseg, N,
 * r) held in its own GPU's HBM, and one RCCL all-gather of the 4-byte
 * results (the only exchange) leaves every rank with all CRCs in segment
 * order.  Segment bytes never cross xGMI.  RCCL (librccl.so.1) is loaded
 * at the first shard call; without it the shard calls return RAMCRC_ERCCL.
 *
 * Two ways to build one:
 *   ramcrc_shard_create_all  one process drives `ndev` GPUs (ncclCommInitAll);
 *                            local rank k = devices[k] = global rank k;
 *   ramcrc_shard_create_rank one process per GPU (ncclCommInitRank): every
 *                            process passes the same unique id (made by one
 *                            of them with ramcrc_shard_unique_id and sent to
 *                            the others out of band) and its own rank.
 * A shard owns one stream and one ramcrc_ctx per local rank. */
typedef struct ramcrc_shard ramcrc_shard;
#define RAMCRC_SHARD_ID_BYTES 128

int ramcrc_shard_unique_id(void* id /* RAMCRC_SHARD_ID_BYTES */);
int ramcrc_shard_create_all(const int* devices, int ndev, ramcrc_shard** out);
int ramcrc_shard_create_rank(const void* id, int nranks, int rank, int device,
                             ramcrc_shard** out);
int ramcrc_shard_destroy(ramcrc_shard* shard);

/* Contiguous [lo, hi) of segment indices owned by `rank` (sizes differ by at
 * most one; lower ranks get the extra ones).  Pure host arithmetic. */
int ramcrc_shard_range(uint64_t nseg, int nranks, int rank, uint64_t* lo, uint64_t* hi);

/* Local ranks this handle drives, and the global rank / device / stream /
 * context of local rank k (for callers that order their own work against
 * the shard, or time it with ramcrc_ctx_set_timing). */
int ramcrc_shard_local_count(const ramcrc_shard* shard);
int ramcrc_shard_info(const ramcrc_shard* shard, int k, int* rank, int* device, void** stream,
                      ramcrc_ctx** ctx);

/* One recovery-scan step.  For every local rank k (global rank r):
 * d_shard[k] (on that rank's device) holds segments [lo_r, hi_r) of the
 * batch at seg_bytes stride; after the step, d_all[k] (device, nseg uint32)
 * holds the CRCs of all nseg segments in segment order -- or, when d_all is
 * NULL, the shard's own result buffers do (ramcrc_shard_results).  flags:
 * RAMCRC_FINALIZE as for ramcrc_segments_device.  Asynchronous on the
 * shard's streams; a single-process shard issues the ranks' collectives in
 * one RCCL group.  Every rank must pass the same nseg.
 *
 * Liveness (ramcloud_amd/csrc/shard_plan.h): no rank leaves a step before a
 * collective its peers wait in.  A step whose nseg exceeds every earlier one
 * grows the shard's internal buffers on every rank and then exchanges one
 * status word per rank, synchronously; if any rank could not allocate, every
 * rank returns an error before the data collective (RAMCRC_ENOMEM on that
 * rank, RAMCRC_EPEER on the others).  Any other failure of a rank (bad
 * arguments, a failed launch) is returned by it, and it still joins the
 * all-gather with its segments' slots set to 0xFFFFFFFF; its status word
 * travels with the CRCs, so its peers' next ramcrc_shard_sync returns
 * RAMCRC_EPEER. */
int ramcrc_shard_segments(ramcrc_shard* shard, const void* const* d_shard, uint64_t seg_bytes,
                          uint64_t nseg, uint32_t* const* d_all, uint32_t flags);

/* Wait for every local rank's stream.  Returns RAMCRC_ERCCL if RCCL reported
 * an asynchronous error, a device launch's refusal (ramcrc_ctx_check), this
 * rank's own failure of the last step, RAMCRC_EPEER when the last step's
 * gathered status words show that another rank failed (the results then hold
 * 0xFFFFFFFF for its segments), RAMCRC_OK when every CRC of the last step is
 * valid.  Device-side refusals are only seen by the rank that hit them (the
 * uniform-segment scan never refuses). */
int ramcrc_shard_sync(ramcrc_shard* shard);

/* Copy local rank k's gathered CRCs of the last step (when it ran with d_all
 * == NULL) to host memory; synchronous. */
int ramcrc_shard_results(ramcrc_shard* shard, int k, uint32_t* h_out, uint64_t nseg);

/* ------------------------------------------------- batched write path --- */

/* Object::assembleForLog's checksum (src/Object.cc:213-238; the value is
 * Object::computeChecksum, src/Object.cc:770-819) for a batch of serialized
 * objects in device memory, e.g. the objects of a multi-write batch before
 * Log::append (src/ObjectManager.cc:1274-1297): object i is d_len[i] bytes at
 * d_base + d_off[i] -- Object::Header {checksum, timestamp, version, tableId}
 * (src/Object.h:137-182) followed by keysAndValue.  For every object of at
 * least the 24-byte header, the finalized CRC32C of bytes [4, len) is stored
 * little-endian into bytes [0, 4) (Header::checksum) and into d_out[i] when
 * d_out is not NULL; shorter objects are left unchanged (d_out[i] = 0).
 * Objects must not overlap.  Stream-ordered. */
int ramcrc_assemble_objects_device(ramcrc_ctx* ctx, void* d_base, const uint64_t* d_off,
                                   const uint64_t* d_len, uint32_t* d_out, uint64_t n,
                                   void* stream);

/* The same for objects in host memory (a write batch still in its RPC
 * buffers): staged through pinned memory, CRCs computed on the GPU, each
 * Header::checksum written back into the host object.  Synchronous. */
int ramcrc_assemble_objects_host(ramcrc_ctx* ctx, void* const* objs, const uint64_t* lens,
                                 uint64_t n);

/* Context options.
 *   RAMCRC_OPT_SERIAL_WALK  nonzero: ramcrc_segment_walk_device walks every
 *                           segment with one wavefront (the chain followed
 *                           hop by hop); 0 (default): the parallel walk,
 *                           which finds the chain in every 64 KiB part of a
 *                           segment at once and hands only anomalous segments
 *                           (offset wraps) to the serial walker.  Both give
 *                           identical results. */
#define RAMCRC_OPT_SERIAL_WALK 1
/*   RAMCRC_OPT_WALK_PART_SHIFT  log2 of the parallel walk's part size, 13..20
 *                           (8 KiB .. 1 MiB), forced for every batch; 0: the
 *                           default, chosen per batch from the entry density
 *                           (about 64 entries per part, 64 KiB .. 1 MiB).
 *                           Results are identical for every part size (the
 *                           parity tests run several). */
#define RAMCRC_OPT_WALK_PART_SHIFT 2
/*   RAMCRC_OPT_TEST_FAIL_AFTER_COUNT  test hook: the next `value` small-entry
 *                           launch sequences return RAMCRC_EHIP right after
 *                           their histogram pass is enqueued (the launch
 *                           failure the error paths must survive); 0: off. */
#define RAMCRC_OPT_TEST_FAIL_AFTER_COUNT 3
/*   RAMCRC_OPT_TEST_DIRTY_BINS  test hook: the next small-entry launch adds
 *                           (value & 0xffff) to the histogram count of bin
 *                           value >> 16 between its count and scatter passes;
 *                           the launch must then refuse (RAMCRC_EINTERNAL from
 *                           ramcrc_ctx_check) rather than read stale slots. */
#define RAMCRC_OPT_TEST_DIRTY_BINS 4
/*   RAMCRC_OPT_TEST_BIN_STRAGGLER  test hook: the next one-launch binning
 *                           (k_bin_one, batches of at most one 4,096-entry
 *                           tile per CU) waits for one workgroup more than it
 *                           launched, as if part of the grid were never
 *                           dispatched; it must abort after its stall period
 *                           (no arrival for 30 us) and the launch complete
 *                           through the two-launch binning with exact results. */
#define RAMCRC_OPT_TEST_BIN_STRAGGLER 5
/*   RAMCRC_OPT_BIN_ONE     small-entry batches of at most one 4,096-entry
 *                           tile per CU: 1 bins them with the one-launch
 *                           k_bin_one (a grid-wide vote), 0
 *                           (default since round 6) with the two-launch count
 *                           and scatter.  Identical results. */
#define RAMCRC_OPT_BIN_ONE 6
/*   RAMCRC_OPT_VERIFY_IN_WALK  ramcrc_replay_verify_device with small entries
 *                           (the objects of 64- and 128-byte values): 1
 *                           (default) checks each object while its record is
 *                           copied, from the object bytes staged in LDS, and
 *                           skips the binned object scan; 2 does so for every
 *                           batch; 0 always runs the binned scan.  Identical
 *                           results. */
#define RAMCRC_OPT_VERIFY_IN_WALK 7
int ramcrc_ctx_set_option(ramcrc_ctx* ctx, int option, int64_t value);

/* Kernel timing (for benchmarks): when enabled, every launch brackets its
 * byte-scan kernel (k_chunks, or k_entries on the small path; in the fused
 * replay call also the two k_walk_copyv launches, which do the object checks
 * in verify-in-walk mode) with HIP events on the launch stream.  ramcrc_ctx_scan_time waits for the recorded events,
 * returns the summed kernel milliseconds and the number of bracketed launches
 * since the last call, and resets both. */
int ramcrc_ctx_set_timing(ramcrc_ctx* ctx, int enable);
int ramcrc_ctx_scan_time(ramcrc_ctx* ctx, double* total_ms, uint64_t* launches);

/* Replay pipelining (a recovery master replaying a stream of segment batches,
 * src/ObjectManager.cc:580-1100): the segment walk is one latency-bound wave
 * per segment, the object scan a bandwidth-bound persistent grid whose
 * workgroups take most of a CU's LDS, so the two cannot share CUs.
 * ramcrc_stream_create_cu_mask creates a stream whose kernels run only on
 * the CUs set in cu_mask (hipExtStreamCreateWithCUMask; bit i of word i/32 =
 * CU i, mask_words <= 8); ramcrc_ctx_set_cus(ctx, n) sizes the context's
 * persistent grids (k_chunks, k_entries*) for n CUs (0 = all of them), to
 * match the mask of the stream the context launches on.  Walking batch k on
 * one masked stream while batch k-1 is scanned on the complementary one
 * overlaps the two. */
int ramcrc_stream_create_cu_mask(int device, const uint32_t* cu_mask, uint32_t mask_words,
                                 void** out_stream);
int ramcrc_stream_destroy(void* stream);
int ramcrc_ctx_set_cus(ramcrc_ctx* ctx, int ncu);

/* Raw launch status word of the context (bit 0: the latest planned launch
 * found more chunks than the scratch holds and wrote none of its outputs;
 * bit 1: some launch refused since the last ramcrc_ctx_check; bit 2: one of
 * them was a small-entry launch whose bin layout was inconsistent).
 * Synchronous. */
int ramcrc_ctx_status(ramcrc_ctx* ctx, uint32_t* status);

/* Waits for `stream`, then returns RAMCRC_EINTERNAL or RAMCRC_EREFUSED (and
 * clears the sticky bits, atomically on the device) if any launch of this
 * context was refused since the last check, RAMCRC_OK otherwise.  A refusal
 * needs a general batch whose buffers
 * overlap or total more bytes than the device holds (ramcrc_batch_device,
 * ramcrc_verify_objects_device, ramcrc_assemble_objects_device); raise
 * ramcrc_ctx_reserve and retry.  The host entry points (ramcrc_batch_host,
 * ramcrc_assemble_objects_host) check by themselves. */
int ramcrc_ctx_check(ramcrc_ctx* ctx, void* stream);

/* Diagnostics.  ramcrc_ctx_debug_bins waits for the device and copies the
 * small-entry bin table's counts, both counter copies' cursors and
 * histograms (5 x 161 words), then the number of one-launch binnings that
 * aborted and completed through the two-launch path (1 word), to host, and
 * the parity of the next sequence. */
int ramcrc_ctx_debug_bins(ramcrc_ctx* ctx, uint64_t* host, uint64_t nwords, uint32_t* par_next);
const char* ramcrc_strerror(int code);
int ramcrc_last_hip_error(void);            /* last hipError_t seen (thread-local) */
int ramcrc_device_count(void);
const char* ramcrc_build_info(void);

#ifdef __cplusplus
}
#endif

#endif /* RAMCRC_H */
