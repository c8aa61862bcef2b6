// Host-path microbenchmark in the shape of RAMCloud's own CRC benchmark
// (src/misc/crc32c.cc:57-104): sizes 1..127 B and 128 B..16 MiB doubling, a
// random buffer, one Crc32C::update per run, MB/s (2^20 B/s, as the reference
// prints).  It times the drop-in host path that Crc32C::update now calls
// (ramcrc_update_hw / _sw in libramcrc) next to the reference's own
// intelCrc32C (src/Crc32C.h:39-93) compiled from the reference source into
// oracle/_ref -- the reference leg is the CPU baseline, loaded with dlopen
// only when that library was shipped.
//
//   host_bench [oracle/_ref/libref_crc32c.so]     -> one JSON object per size
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <vector>

#include "ramcrc.h"

typedef uint32_t (*crc_fn)(uint32_t, const void*, uint64_t);

static double now()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

// Best of 5 timings of `runs` back-to-back updates (each from the previous
// result, so the calls cannot be elided), in MB/s.
static double measure(crc_fn f, const uint8_t* buf, uint64_t n, int runs, uint32_t* sink)
{
    double best = 1e30;
    for (int rep = 0; rep < 5; rep++) {
        uint32_t s = 0xFFFFFFFFu;
        const double t0 = now();
        for (int r = 0; r < runs; r++)
            s = f(s, buf, n);
        const double dt = now() - t0;
        *sink ^= s;
        if (dt < best)
            best = dt;
    }
    return double(n) * runs / best / (1 << 20);
}

int main(int argc, char** argv)
{
    crc_fn ref = NULL;
    if (argc > 1) {
        void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
        if (h)
            ref = reinterpret_cast<crc_fn>(dlsym(h, "ref_intel_crc32c"));
    }
    const uint64_t maxn = 16u << 20;
    std::vector<uint8_t> buf(maxn);
    uint64_t x = 88172645463325252ull;
    for (uint64_t i = 0; i < maxn; i++) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        buf[i] = uint8_t(x);
    }
    std::vector<uint64_t> sizes;
    for (uint64_t n = 1; n < 128; n++)
        sizes.push_back(n);
    for (uint64_t n = 128; n <= maxn; n *= 2)
        sizes.push_back(n);
    uint32_t sink = 0;
    int mismatches = 0;
    for (uint64_t n : sizes) {
        // enough runs for >= ~2 ms per timing
        const int runs = n < 4096 ? int(200000 / (n / 64 + 1)) : int((64u << 20) / n + 1);
        const double hw = measure(ramcrc_update_hw, buf.data(), n, runs, &sink);
        const double sw = measure(ramcrc_update_sw, buf.data(), n, runs, &sink);
        double rv = -1;
        if (ref) {
            rv = measure(ref, buf.data(), n, runs, &sink);
            if (ref(0xFFFFFFFFu, buf.data(), n) != ramcrc_update_hw(0xFFFFFFFFu, buf.data(), n))
                mismatches++;
        }
        printf("{\"bytes\": %llu, \"ramcrc_hw_MBps\": %.1f, \"ramcrc_sw_MBps\": %.1f, "
               "\"reference_intelCrc32C_MBps\": %.1f}\n",
               (unsigned long long)n, hw, sw, rv);
    }
    printf("{\"summary\": true, \"reference_loaded\": %s, \"mismatches\": %d, \"sink\": %u}\n",
           ref ? "true" : "false", mismatches, sink);
    return mismatches ? 1 : 0;
}
