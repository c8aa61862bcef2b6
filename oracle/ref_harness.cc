/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Thin C entry points around the reference's own CRC32C code, compiled from
 * /root/reference/src/Crc32C.h where it lies (see oracle/Makefile, target
 * _ref).  Only the header-inline hardware path is built: RAMCloud::intelCrc32C
 * (src/Crc32C.h:39-93).  src/Crc32C.cc is not compiled because it includes
 * Logger.h -> SpinLock.h -> SpinLockStatistics.pb.h (generated protobuf code
 * absent from this image); building it would need stand-in headers, which we
 * do not write.  softwareCrc32C (src/Crc32C.h:96-153) needs the tables defined
 * in that .cc, so it is covered by the oracle restatement plus the
 * src/Crc32CTest.cc known answers instead.
 *
 * The output library oracle/_ref/libref_crc32c.so is git-ignored and travels
 * to the GPU box with the snapshot; no reference source is copied.
 */
#include "Crc32C.h"

#include <pthread.h>
#include <sched.h>
#include <stdint.h>

extern "C" {

uint32_t ref_intel_crc32c(uint32_t state, const void* p, uint64_t n)
{
    return RAMCloud::intelCrc32C(state, p, n);
}

struct RefSegJob {
    const uint8_t* base;
    uint64_t segBytes, nseg;
    uint32_t* out;
    int tid, nthreads, pin;
};

static void* refSegWorker(void* arg)
{
    RefSegJob* j = static_cast<RefSegJob*>(arg);
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
    // Crc32C().update(seg, len).getResult() per whole segment, round-robin
    // over threads (nanobenchmarks/RecoverSegmentBenchmark.cc:90-118 shape).
    for (uint64_t i = j->tid; i < j->nseg; i += j->nthreads)
        j->out[i] = ~RAMCloud::intelCrc32C(0xFFFFFFFFu, j->base + i * j->segBytes,
                                           j->segBytes);
    return NULL;
}

int ref_segments_mt(const uint8_t* base, uint64_t segBytes, uint64_t nseg,
                    uint32_t* out, int nthreads, int pin)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    pthread_t th[256];
    RefSegJob jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = RefSegJob{base, segBytes, nseg, out, t, nthreads, pin};
        if (pthread_create(&th[t], NULL, refSegWorker, &jobs[t]) != 0)
            return -1;
    }
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    return 0;
}

// Per-entry form: one Crc32C per log entry / object, as the reference's
// replay and append loops call it (src/ObjectManager.cc:659-669,
// src/Object.cc:805-819): out[i] = getResult() of an update over
// base[off[i], off[i] + len[i]) from init[i] (0xFFFFFFFF when init is NULL),
// or the raw state when finalize is 0.  Blocks of 4096 consecutive entries
// are dealt round-robin to the threads, so each thread reads packed log bytes
// sequentially.
struct RefEntJob {
    const uint8_t* base;
    const uint64_t *off, *len;
    const uint32_t* init;
    uint32_t* out;
    uint64_t n;
    int tid, nthreads, pin, finalize;
};

static void pin_to(int tid)
{
    cpu_set_t all, one;
    if (sched_getaffinity(0, sizeof(all), &all) != 0)
        return;
    int seen = 0;
    for (int c = 0; c < CPU_SETSIZE; c++) {
        if (!CPU_ISSET(c, &all))
            continue;
        if (seen++ == tid) {
            CPU_ZERO(&one);
            CPU_SET(c, &one);
            pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
            return;
        }
    }
}

static void* refEntWorker(void* arg)
{
    RefEntJob* j = static_cast<RefEntJob*>(arg);
    if (j->pin)
        pin_to(j->tid);
    const uint64_t kBlk = 4096;
    for (uint64_t b = uint64_t(j->tid) * kBlk; b < j->n; b += uint64_t(j->nthreads) * kBlk) {
        const uint64_t e = b + kBlk < j->n ? b + kBlk : j->n;
        for (uint64_t i = b; i < e; i++) {
            const uint32_t s = RAMCloud::intelCrc32C(j->init ? j->init[i] : 0xFFFFFFFFu,
                                                     j->base + j->off[i], j->len[i]);
            j->out[i] = j->finalize ? ~s : s;
        }
    }
    return NULL;
}

int ref_entries_mt(const uint8_t* base, const uint64_t* off, const uint64_t* len,
                   const uint32_t* init, uint32_t* out, uint64_t n, int nthreads, int pin,
                   int finalize)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    pthread_t th[256];
    RefEntJob jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = RefEntJob{base, off, len, init, out, n, t, nthreads, pin, finalize};
        if (pthread_create(&th[t], NULL, refEntWorker, &jobs[t]) != 0)
            return -1;
    }
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    return 0;
}

}  // extern "C"
