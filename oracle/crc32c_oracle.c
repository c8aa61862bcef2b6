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
