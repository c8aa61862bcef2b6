/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * A CPU restatement of RAMCloud's CRC32C integrity checksum, used solely as
 * the checker for the MI355X product path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's `cpu_baseline` leg may load this code; the product library
 * (ramcloud_amd/lib/libramcrc.so) never links or calls it.
 *
 * Parity pin: every function here is checked by tests/test_oracle.py against
 *   - the 82 known-answer CRCs of src/Crc32CTest.cc:27-58 (tests/golden/),
 *   - Segment certificate goldens src/SegmentTest.cc:159,369,373,
 *   - the Object checksum golden src/ObjectTest.cc:171,
 *   - and, when the reference is present, oracle/_ref/libref_crc32c.so, which
 *     is the reference's own src/Crc32C.h (intelCrc32C) compiled from
 *     /root/reference by oracle/Makefile.
 *
 * Algorithm (reference citations are /root/reference paths):
 *   - CRC-32C (Castagnoli), reflected polynomial 0x82F63B78
 *     (src/Crc32C.cc:73, :96-100).
 *   - The running state starts at 0xFFFFFFFF (src/Crc32C.h:177), update()
 *     advances it with no inversion (src/Crc32C.h:200-206), getResult()
 *     returns ~state without resetting it (src/Crc32C.h:247-249).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <sched.h>

#define ORACLE_POLY 0x82F63B78u

static uint32_t g_slice[8][256];
static int g_ready = 0;

/* Tables follow the generator described at src/Crc32C.cc:71-91:
 * slice[0][i] is the bitwise CRC step of byte i, slice[k][i] extends
 * slice[k-1][i] by one more zero byte.  Generated, never copied. */
void oracle_init(void)
{
    if (g_ready)
        return;
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t x = i;
        for (int j = 0; j < 8; j++)
            x = (x >> 1) ^ (ORACLE_POLY & (0u - (x & 1u)));
        g_slice[0][i] = x;
    }
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = g_slice[0][i];
        for (int k = 1; k < 8; k++) {
            c = g_slice[0][c & 0xFF] ^ (c >> 8);
            g_slice[k][i] = c;
        }
    }
    g_ready = 1;
}

const uint32_t* oracle_table(int k) { oracle_init(); return g_slice[k]; }

/* Bit-at-a-time definition; the slowest and most obviously correct form. */
uint32_t oracle_bitwise(uint32_t state, const void* data, uint64_t n)
{
    const uint8_t* p = (const uint8_t*)data;
    for (uint64_t i = 0; i < n; i++) {
        state ^= p[i];
        for (int b = 0; b < 8; b++)
            state = (state >> 1) ^ (ORACLE_POLY & (0u - (state & 1u)));
    }
    return state;
}

static inline uint32_t ld32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t ld64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint16_t ld16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }

/* Restates softwareCrc32C (src/Crc32C.h:96-153): byte steps until the pointer
 * is 4-aligned (:118-123), slicing-by-8 over 8-byte blocks (:125-146), byte
 * tail (:148-150).  Same arithmetic, written independently. */
uint32_t oracle_slicing8(uint32_t crc, const void* data, uint64_t n)
{
    oracle_init();
    const uint8_t* p = (const uint8_t*)data;
    uint64_t lead = (4u - ((uintptr_t)p & 3u)) & 3u;
    if (lead > n)
        lead = n;
    for (uint64_t i = 0; i < lead; i++)
        crc = g_slice[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
    n -= lead;
    for (uint64_t blocks = n >> 3; blocks > 0; blocks--) {
        uint32_t lo = crc ^ ld32(p);
        uint32_t hi = ld32(p + 4);
        crc = g_slice[7][lo & 0xFF] ^ g_slice[6][(lo >> 8) & 0xFF] ^
              g_slice[5][(lo >> 16) & 0xFF] ^ g_slice[4][lo >> 24] ^
              g_slice[3][hi & 0xFF] ^ g_slice[2][(hi >> 8) & 0xFF] ^
              g_slice[1][(hi >> 16) & 0xFF] ^ g_slice[0][hi >> 24];
        p += 8;
    }
    for (uint64_t i = 0; i < (n & 7); i++)
        crc = g_slice[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
    return crc;
}

/* Restates the instruction schedule of intelCrc32C (src/Crc32C.h:39-93):
 * four crc32q per 32 B (:52-61), crc32q per remaining 8 B (:63-69), crc32w
 * per remaining 2 B (:71-78), crc32b for an odd last byte (:80-84), one
 * dependency chain, no inversion inside.  Falls back to slicing-by-8 when
 * the build has no SSE4.2 (the reference throws there, :89-91). */
uint32_t oracle_sse42(uint32_t crc, const void* data, uint64_t n)
{
#if defined(__SSE4_2__)
    const uint8_t* p = (const uint8_t*)data;
    uint64_t c = crc;
    for (uint64_t k = n >> 5; k > 0; k--) {
        c = __builtin_ia32_crc32di(c, ld64(p));
        c = __builtin_ia32_crc32di(c, ld64(p + 8));
        c = __builtin_ia32_crc32di(c, ld64(p + 16));
        c = __builtin_ia32_crc32di(c, ld64(p + 24));
        p += 32;
    }
    for (uint64_t k = (n & 31) >> 3; k > 0; k--) {
        c = __builtin_ia32_crc32di(c, ld64(p));
        p += 8;
    }
    uint32_t s = (uint32_t)c;
    for (uint64_t k = (n & 7) >> 1; k > 0; k--) {
        s = __builtin_ia32_crc32hi(s, ld16(p));
        p += 2;
    }
    if (n & 1)
        s = __builtin_ia32_crc32qi(s, *p);
    return s;
#else
    return oracle_slicing8(crc, data, n);
#endif
}

int oracle_have_sse42(void)
{
#if defined(__SSE4_2__)
    return 1;
#else
    return 0;
#endif
}

/* ---------------------------------------------------------------------- */
/* GF(2) helpers used by the tests to pin the combine identities.           */
/* Reflected representation: bit 31 is x^0, bit 0 is x^31.                  */

uint32_t oracle_mulmod(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
    for (int i = 0; i < 32; i++) {
        if (a & (0x80000000u >> i))
            p ^= b;
        b = (b >> 1) ^ (ORACLE_POLY & (0u - (b & 1u)));
    }
    return p;
}

/* x^(8n) mod P: the operator that appends n zero bytes to a raw state. */
uint32_t oracle_xpow8(uint64_t n)
{
    uint32_t result = 0x80000000u, sq = 0x00800000u; /* 1, x^8 */
    while (n) {
        if (n & 1)
            result = oracle_mulmod(result, sq);
        sq = oracle_mulmod(sq, sq);
        n >>= 1;
    }
    return result;
}

/* raw(0, A||B) = shift(raw(0,A), |B|) ^ raw(0,B): the linearity identity the
 * device kernels are built on (zlib crc32_combine, restated). */
uint32_t oracle_shift(uint32_t state, uint64_t nbytes)
{
    return oracle_mulmod(state, oracle_xpow8(nbytes));
}

/* ---------------------------------------------------------------------- */
/* Synthetic inputs shared with the device generator (bench + tests).       */

static inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* splitmix64 stream: word j is mix64(seed + (j+1)*gamma), little-endian. */
void oracle_splitmix_fill(uint64_t seed, void* dst, uint64_t nbytes)
{
    uint8_t* d = (uint8_t*)dst;
    uint64_t j = 0;
    for (; (j + 1) * 8 <= nbytes; j++) {
        uint64_t v = mix64(seed + (j + 1) * 0x9E3779B97F4A7C15ull);
        memcpy(d + j * 8, &v, 8);
    }
    if (j * 8 < nbytes) {
        uint64_t v = mix64(seed + (j + 1) * 0x9E3779B97F4A7C15ull);
        memcpy(d + j * 8, &v, nbytes - j * 8);
    }
}

/* ---------------------------------------------------------------------- */
/* Batch forms: out[i] = Crc32C(state=init[i]).update(buf_i, len_i), then
 * ~ when finalize (getResult) or the raw state otherwise. */

typedef uint32_t (*crc_fn)(uint32_t, const void*, uint64_t);

static crc_fn pick(int impl)
{
    switch (impl) {
    case 0: return oracle_sse42;
    case 1: return oracle_slicing8;
    default: return oracle_bitwise;
    }
}

void oracle_entries(const uint8_t* base, const uint64_t* off, const uint64_t* len,
                    const uint32_t* init, uint32_t* out, uint64_t n, int finalize,
                    int impl)
{
    crc_fn f = pick(impl);
    for (uint64_t i = 0; i < n; i++) {
        uint32_t s = init ? init[i] : 0xFFFFFFFFu;
        s = f(s, base + off[i], len[i]);
        out[i] = finalize ? ~s : s;
    }
}

struct seg_job {
    const uint8_t* base;
    uint64_t seg_bytes, nseg;
    uint32_t* out;
    int tid, nthreads, impl, pin;
};

static void* seg_worker(void* arg)
{
    struct seg_job* j = (struct seg_job*)arg;
    if (j->pin) {
        cpu_set_t all, one;
        if (sched_getaffinity(0, sizeof(all), &all) == 0) {
            int seen = 0;
            for (int c = 0; c < CPU_SETSIZE; c++) {
                if (!CPU_ISSET(c, &all))
                    continue;
                if (seen++ == j->tid) {
                    CPU_ZERO(&one);
                    CPU_SET(c, &one);
                    pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
                    break;
                }
            }
        }
    }
    crc_fn f = pick(j->impl);
    /* Whole segments, round-robin over threads, as RecoverSegmentBenchmark's
     * replay pool hands out segments (nanobenchmarks/RecoverSegmentBenchmark.cc:90-118). */
    for (uint64_t i = (uint64_t)j->tid; i < j->nseg; i += (uint64_t)j->nthreads)
        j->out[i] = ~f(0xFFFFFFFFu, j->base + i * j->seg_bytes, j->seg_bytes);
    return NULL;
}

int oracle_segments_mt(const uint8_t* base, uint64_t seg_bytes, uint64_t nseg,
                       uint32_t* out, int nthreads, int impl, int pin)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    pthread_t th[256];
    struct seg_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (struct seg_job){base, seg_bytes, nseg, out, t, nthreads, impl, pin};
        if (pthread_create(&th[t], NULL, seg_worker, &jobs[t]) != 0)
            return -1;
    }
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    return 0;
}

/* ------------------------------------------------------------------------
 * Segments and objects.  Restated from:
 *   - Segment::append (src/Segment.cc:197-228) and hasSpaceFor (:136-154):
 *     |EntryHeader (type | (lengthBytes-1) << 6)|length, 1-4 B LE|payload|,
 *     EntryHeader(type, length) picking lengthBytes (src/Segment.h:131-150);
 *     the segment's running Crc32C over each header byte and length bytes;
 *   - Segment::getAppendedLength (src/Segment.cc:672-684): certificate =
 *     {head, getResult() after also covering head (4 B LE)};
 *   - Segment::checkMetadataIntegrity (src/Segment.cc:758-800), including its
 *     uint32_t offset arithmetic and the order of its three failure checks;
 *   - Object::assembleForLog / computeChecksum (src/Object.cc:213-218,
 *     :805-819): Crc32C over the serialized object minus its first 4 bytes;
 *     Object(key, value, ...) key layout (src/Object.cc:107-141);
 *   - RecoverSegmentBenchmark::run's fill (nanobenchmarks/
 *     RecoverSegmentBenchmark.cc:131-146): tableId 0, 8-byte counter keys,
 *     version 0, timestamp 0.
 * Flags: 1 OK, 2 past capacity, 4 past certificate length, 8 bad checksum,
 * 16 entry table full, 32 cyclic walk (the product's RAMCRC_SEG_* values).
 * ---------------------------------------------------------------------- */
static uint32_t oracle_u32le(const uint8_t* p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

uint32_t oracle_build_object_segment(uint8_t* seg, uint32_t capacity, uint32_t value_len,
                                     uint64_t first_key, uint32_t* cert_len, uint32_t* cert_crc)
{
    uint32_t objlen = 24u + 1u + 2u + 8u + value_len;
    uint32_t lb = objlen < 0x100u ? 1 : objlen < 0x10000u ? 2 : objlen < 0x1000000u ? 3 : 4;
    uint32_t head = 0, n = 0, meta = 0xFFFFFFFFu;
    uint64_t key = first_key;
    for (;;) {
        uint32_t need = 1 + lb + objlen;
        uint32_t left = capacity - head;
        if (need > left)
            break;
        uint8_t* e = seg + head;
        uint8_t hb = (uint8_t)(2u | ((lb - 1) << 6));   /* LOG_ENTRY_TYPE_OBJ */
        e[0] = hb;
        meta = oracle_slicing8(meta, &hb, 1);
        uint8_t lenle[4] = {(uint8_t)objlen, (uint8_t)(objlen >> 8), (uint8_t)(objlen >> 16),
                            (uint8_t)(objlen >> 24)};
        memcpy(e + 1, lenle, lb);
        meta = oracle_slicing8(meta, lenle, lb);
        uint8_t* o = e + 1 + lb;
        memset(o, 0, 24);
        o[24] = 1;
        o[25] = 8;
        o[26] = 0;
        for (int k = 0; k < 8; k++)
            o[27 + k] = (uint8_t)(key >> (8 * k));
        uint32_t ck = ~oracle_slicing8(0xFFFFFFFFu, o + 4, objlen - 4);
        for (int k = 0; k < 4; k++)
            o[k] = (uint8_t)(ck >> (8 * k));
        head += need;
        n++;
        key++;
    }
    memset(seg + head, 0, capacity - head);
    uint8_t hl[4] = {(uint8_t)head, (uint8_t)(head >> 8), (uint8_t)(head >> 16), (uint8_t)(head >> 24)};
    *cert_len = head;
    *cert_crc = ~oracle_slicing8(meta, hl, 4);
    return n;
}

/* table: 4 uint32 per entry {segment, offset, length, header}; returns flags.
 * f: the CRC update used for the metadata bytes. */
static uint32_t check_metadata_f(const uint8_t* seg, uint64_t capacity, uint32_t cert_len,
                                 uint32_t cert_crc, uint32_t segment, uint32_t* checksum_out,
                                 uint32_t* n_out, uint32_t* table, uint64_t table_cap, crc_fn f);

uint32_t oracle_check_metadata(const uint8_t* seg, uint64_t capacity, uint32_t cert_len,
                               uint32_t cert_crc, uint32_t segment, uint32_t* checksum_out,
                               uint32_t* n_out, uint32_t* table, uint64_t table_cap)
{
    return check_metadata_f(seg, capacity, cert_len, cert_crc, segment, checksum_out, n_out,
                            table, table_cap, oracle_slicing8);
}

static uint32_t check_metadata_f(const uint8_t* seg, uint64_t capacity, uint32_t cert_len,
                                 uint32_t cert_crc, uint32_t segment, uint32_t* checksum_out,
                                 uint32_t* n_out, uint32_t* table, uint64_t table_cap, crc_fn f)
{
    uint32_t offset = 0, crc = 0xFFFFFFFFu, n = 0, flags = 0;
    uint64_t steps = 0;
    while (offset < cert_len && (uint64_t)offset < capacity) {
        /* The walk is deterministic in `offset` and stays below the capacity,
         * so more than `capacity` steps means a position repeated: through the
         * uint32_t wrap the reference's loop would never end.  Stop (flag 32). */
        if (++steps > capacity) {
            flags |= 32;
            break;
        }
        uint8_t hdr = seg[offset];
        crc = f(crc, &hdr, 1);
        uint32_t lb = (uint32_t)(hdr >> 6) + 1;
        uint8_t lenle[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < lb; k++)   /* copyOut: bytes past the capacity stay 0 */
            if ((uint64_t)offset + 1 + k < capacity)
                lenle[k] = seg[offset + 1 + k];
        uint32_t length = oracle_u32le(lenle);
        crc = f(crc, lenle, lb);
        uint32_t next = offset + 1 + lb + length;   /* uint32_t, as the reference */
        if ((uint64_t)next > capacity) {
            flags |= 2;
            break;
        }
        if (table && n < table_cap) {
            /* 0x100: the payload runs past the capacity (only reachable through
             * the uint32_t wrap of `offset`); such an object cannot be read */
            uint64_t end = (uint64_t)offset + 1 + lb + length;
            table[4 * (uint64_t)n + 0] = segment;
            table[4 * (uint64_t)n + 1] = offset;
            table[4 * (uint64_t)n + 2] = length;
            table[4 * (uint64_t)n + 3] = hdr | (end > capacity ? 0x100u : 0u);
        }
        n++;
        offset = next;
    }
    uint8_t cl[4] = {(uint8_t)cert_len, (uint8_t)(cert_len >> 8), (uint8_t)(cert_len >> 16),
                     (uint8_t)(cert_len >> 24)};
    uint32_t fin = ~f(crc, cl, 4);
    if (!(flags & (2 | 32))) {
        if (offset > cert_len)
            flags |= 4;
        else
            flags |= fin == cert_crc ? 1 : 8;
    }
    if (table && n > table_cap)
        flags = (flags | 16) & ~1u;   /* records dropped: the segment is not verified */
    if (checksum_out)
        *checksum_out = fin;
    if (n_out)
        *n_out = n;
    return flags;
}

/* The checksum checks ObjectManager::replaySegment makes on the records (4
 * uint32 each) of segments at base + segment*stride whose metadata check
 * passed (seg_ok[segment] != 0, or every segment when seg_ok is NULL) --
 * RecoverySegmentBuilder::build stops at a failed check
 * (src/RecoverySegmentBuilder.cc:61-203), so nothing of such a segment is
 * replayed:
 *   OBJ (2)          Object::computeChecksum (src/Object.cc:805-819): bytes
 *                    [4, len) against the stored header.checksum at [0, 4)
 *                    (src/ObjectManager.cc:659-663);
 *   OBJTOMB (3)      ObjectTombstone::computeChecksum (src/Object.cc:1042-1057):
 *                    header bytes [0, 28) then the key [32, len), against
 *                    header.checksum at [28, 32) (src/ObjectManager.cc:752-758);
 *   SAFEVERSION (5)  ObjectSafeVersion::computeChecksum (src/Object.cc:1135-1143):
 *                    bytes [0, 8) against header.checksum at [8, 12)
 *                    (src/ObjectManager.cc:873-880);
 *   PREP (8)         PreparedOp::computeChecksum (src/PreparedOp.cc:177-190):
 *                    its header (src/PreparedOp.h:63-100, 32 bytes) up to the
 *                    checksum, [0, 28), then Object::applyChecksum of the
 *                    object at 32 (src/Object.cc:748-765): [36, len); against
 *                    [28, 32) (src/ObjectManager.cc:956);
 *   PREPTOMB (9)     PreparedOpTombstone::computeChecksum (src/PreparedOp.cc:271-282):
 *                    [0, 40) of the 44-byte header against [40, 44) (:1013);
 *   TXDECISION (10)  TxDecisionRecord::computeChecksum (src/TxDecisionRecord.cc:209-223):
 *                    [0, 44) of the 48-byte header, then
 *                    sizeof32(TxParticipant) * participantCount (uint32 product;
 *                    count at [36, 40)) bytes from 48 through a Buffer::Iterator,
 *                    which clips to the entry (src/Buffer.cc:838-868); against
 *                    [44, 48) (:1060);
 *   TXPLIST (11)     ParticipantList::computeChecksum (src/ParticipantList.cc:96-110):
 *                    [0, 20) of the 24-byte header, then 24 * count (count at
 *                    [16, 20)) bytes from 24, against [20, 24) (:1084).  A list
 *                    past the entry fails: getRange (src/Buffer.cc:530-549)
 *                    returns NULL there and the reference would fault.
 * crc_out[i] receives the computed CRC of each readable record of these types
 * that holds at least its header (24, 32, 12, 56, 44, 48, 24 bytes).  Returns the number of
 * failed checks; shorter or unreadable records count as failures (the
 * reference would read past the entry there).  Failures are added to
 * bad_per_seg[segment] when that is non-NULL. */
static uint64_t verify_objects_f(const uint8_t* base, uint64_t stride, const uint32_t* table,
                                 uint64_t n, const uint8_t* seg_ok, uint32_t* crc_out,
                                 uint32_t* bad_per_seg, crc_fn f);

uint64_t oracle_verify_objects(const uint8_t* base, uint64_t stride, const uint32_t* table,
                               uint64_t n, const uint8_t* seg_ok, uint32_t* crc_out,
                               uint32_t* bad_per_seg)
{
    /* Crc32C picks the crc32 instruction when the CPU has it
     * (src/Crc32C.h:200-206); both forms agree bit for bit */
    return verify_objects_f(base, stride, table, n, seg_ok, crc_out, bad_per_seg,
                            oracle_have_sse42() ? oracle_sse42 : oracle_slicing8);
}

static uint64_t verify_objects_f(const uint8_t* base, uint64_t stride, const uint32_t* table,
                                 uint64_t n, const uint8_t* seg_ok, uint32_t* crc_out,
                                 uint32_t* bad_per_seg, crc_fn f)
{
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t* r = table + 4 * i;
        const uint32_t type = r[3] & 0x3f;
        static const uint32_t hdr_of[12] = {0, 0, 24, 32, 0, 12, 0, 0, 56, 44, 48, 24};
        const uint32_t hdr = type < 12 ? hdr_of[type] : 0;
        if (hdr == 0 || (seg_ok && !seg_ok[r[0]]))
            continue;
        int ok = 0;
        if (r[2] >= hdr && !(r[3] & 0x100)) {
            const uint8_t* payload = base + (uint64_t)r[0] * stride + r[1] + 1 + ((r[3] >> 6) & 3) + 1;
            const uint32_t len = r[2];
            uint32_t c, stored;
            int fits = 1;
            if (type == 2) {
                c = ~f(0xFFFFFFFFu, payload + 4, len - 4);
                stored = oracle_u32le(payload);
            } else {
                /* CRC of [0, at) then [from, from + tail); checksum at [at, at + 4) */
                uint32_t at = hdr - 4, from = hdr, tail = 0;
                if (type == 3) {
                    tail = len - 32;
                } else if (type == 8) {
                    at = 28;
                    from = 36;
                    tail = len - 36;
                } else if (type == 10) {
                    tail = 24u * oracle_u32le(payload + 36);
                    if (tail > len - 48)
                        tail = len - 48;
                } else if (type == 11) {
                    tail = 24u * oracle_u32le(payload + 16);
                    fits = tail <= len - 24;
                }
                c = ~f(f(0xFFFFFFFFu, payload, at), payload + from, fits ? tail : 0);
                stored = oracle_u32le(payload + at);
            }
            if (fits) {
                if (crc_out)
                    crc_out[i] = c;
                ok = c == stored;
            }
        }
        if (!ok) {
            bad++;
            if (bad_per_seg)
                bad_per_seg[r[0]]++;
        }
    }
    return bad;
}

/* ------------------------------------------------------------------------
 * Replay baseline (bench.py): the checksum work of RecoverSegmentBenchmark's
 * replay threads (nanobenchmarks/RecoverSegmentBenchmark.cc:90-118) -- per
 * segment, Segment::checkMetadataIntegrity (restated walk above) and then the
 * replaySegment checks of every record -- with whole segments round-robin
 * over `nthreads` pinned threads.  Every CRC byte goes through `ext` (the
 * reference's own intelCrc32C from oracle/_ref when the caller passes it),
 * else through the SSE4.2 restatement.  certs: 2 uint32 per segment
 * {segmentLength, checksum}.  Returns the number of segments that failed
 * their metadata check or held a failed record. */
struct replay_job {
    const uint8_t* base;
    uint64_t seg_bytes, nseg;
    const uint32_t* certs;
    crc_fn f;
    int tid, nthreads, pin;
    uint64_t failed;
};

static void* replay_worker(void* arg)
{
    struct replay_job* j = (struct replay_job*)arg;
    if (j->pin) {
        cpu_set_t all, one;
        if (sched_getaffinity(0, sizeof(all), &all) == 0) {
            int seen = 0;
            for (int c = 0; c < CPU_SETSIZE; c++) {
                if (!CPU_ISSET(c, &all))
                    continue;
                if (seen++ == j->tid) {
                    CPU_ZERO(&one);
                    CPU_SET(c, &one);
                    pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
                    break;
                }
            }
        }
    }
    const uint64_t cap = j->seg_bytes / 2 + 1;
    uint32_t* table = (uint32_t*)malloc(cap * 16);
    if (!table) {
        j->failed = ~(uint64_t)0;
        return NULL;
    }
    for (uint64_t i = (uint64_t)j->tid; i < j->nseg; i += (uint64_t)j->nthreads) {
        const uint8_t* seg = j->base + i * j->seg_bytes;
        uint32_t ck = 0, n = 0;
        const uint32_t fl = check_metadata_f(seg, j->seg_bytes, j->certs[2 * i], j->certs[2 * i + 1],
                                             0, &ck, &n, table, cap, j->f);
        uint64_t bad = 0;
        if (fl == 1)
            bad = verify_objects_f(seg, j->seg_bytes, table, n, NULL, NULL, NULL, j->f);
        j->failed += (fl != 1) || bad;
    }
    free(table);
    return NULL;
}

int64_t oracle_replay_mt(const uint8_t* base, uint64_t seg_bytes, uint64_t nseg,
                         const uint32_t* certs, int nthreads, int pin, crc_fn ext)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    pthread_t th[256];
    struct replay_job jobs[256];
    crc_fn f = ext ? ext : (oracle_have_sse42() ? oracle_sse42 : oracle_slicing8);
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (struct replay_job){base, seg_bytes, nseg, certs, f, t, nthreads, pin, 0};
        if (pthread_create(&th[t], NULL, replay_worker, &jobs[t]) != 0)
            return -1;
    }
    uint64_t failed = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        failed += jobs[t].failed;
    }
    return (int64_t)failed;
}
