// Host unit test of the parallel walk's synchronisation filter
// (ramcloud_amd/csrc/walk_rules.h): first_hop4, the byte-parallel first-hop
// test k_walk_sync applies to four candidates at once, must pass every
// candidate the exact rule plausible() passes (a superset: the exact rule is
// applied again at the first chase level).  Checked over every header byte x
// top length byte with random middle bytes and random positions, and over
// random 16-byte windows, for capacities on both sides of the 2^23 / 2^24
// cut-offs.  Prints "violations=N checked=M".
#include <stdint.h>
#include <stdio.h>

#include "walk_rules.h"

using namespace ramcrc_walk;

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next64()
{
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
}

static uint64_t violations = 0, checked = 0, passed_exact = 0, passed_filter = 0;

// bytes b[0..15] at offset c0 (multiple of 8): candidates c0 .. c0 + 7
static void check_window(const uint8_t* b, uint32_t c0, uint32_t capacity)
{
    uint32_t d[4];
    for (int u = 0; u < 4; u++)
        d[u] = uint32_t(b[4 * u]) | uint32_t(b[4 * u + 1]) << 8 | uint32_t(b[4 * u + 2]) << 16 |
               uint32_t(b[4 * u + 3]) << 24;
    const bool kill4 = capacity <= (1u << 24), kill3 = capacity <= (1u << 23);
    uint32_t alive = 0;
    for (int g = 0; g < 2; g++) {
        const uint32_t top3 = uint32_t(((uint64_t(d[g + 1]) << 32) | d[g]) >> 24);
        alive |= first_hop4(d[g], top3, kill4, kill3) << (4 * g);
    }
    for (int j = 0; j < 8; j++) {
        const uint64_t q = ((uint64_t(d[j / 4 + 1]) << 32) | d[j / 4]) >> (8 * (j & 3));
        const uint32_t c = c0 + uint32_t(j);
        if (c >= capacity)
            continue;
        const Hop h = hop_of(q, c);
        const bool exact = plausible(q, h, capacity);
        const bool filt = (alive >> j) & 1;
        checked++;
        passed_exact += exact;
        passed_filter += filt;
        if (exact && !filt) {
            if (violations < 5)
                fprintf(stderr, "violation: q=%016llx c=%u cap=%u\n", (unsigned long long)q, c,
                        capacity);
            violations++;
        }
    }
}

int main()
{
    const uint32_t caps[] = {1u << 16, (1u << 20) + 4096, 8u << 20, (1u << 23) + 16, 1u << 24,
                             (1u << 24) + 16, 64u << 20, 0xFFFFFFF0u};
    uint8_t b[16];
    for (uint32_t cap : caps) {
        // every header byte x top length byte, at the first candidate slot
        for (uint32_t hb = 0; hb < 256; hb++)
            for (uint32_t top = 0; top < 256; top++)
                for (int rep = 0; rep < 4; rep++) {
                    for (int k = 0; k < 16; k++)
                        b[k] = uint8_t(next64());
                    const int j = int(next64() & 7);
                    b[j] = uint8_t(hb);
                    b[j + 3] = uint8_t(top);
                    const uint32_t c0 = uint32_t(next64() % cap) & ~7u;
                    check_window(b, c0, cap);
                }
        // random windows
        for (int it = 0; it < 400000; it++) {
            for (int k = 0; k < 16; k++)
                b[k] = uint8_t(next64());
            check_window(b, uint32_t(next64() % cap) & ~7u, cap);
        }
    }
    printf("violations=%llu checked=%llu exact=%llu filter=%llu\n", (unsigned long long)violations,
           (unsigned long long)checked, (unsigned long long)passed_exact,
           (unsigned long long)passed_filter);
    return violations ? 1 : 0;
}
