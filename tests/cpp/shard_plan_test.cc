// Host unit test of the recovery-scan shard's layout and step orchestration
// (ramcloud_amd/csrc/shard_plan.h), the code ramcrc_shard_segments runs on
// every rank, with host stand-ins for the scan kernel (a known value per
// segment), the HIP streams (per-rank queues executed later) and the RCCL
// all-gather (executed only when every rank has reached it -- a rank that
// skipped it would hang the real collective, and fails the test here).
//
//   layout:  nseg 0..4100 x N 1..8: ranges partition [0, nseg), sizes differ
//            by at most one, every segment's gather slot is inside its owner's
//            block and distinct;
//   steps:   N 1..8, both process models (one process driving all ranks, one
//            process per rank), with and without a caller output array, on
//            divisible and ragged batches: every rank ends with every CRC in
//            segment order;
//   faults:  a rank whose scan fails still takes part in the collective, its
//            slots are poisoned, it reports the error; the other ranks finish.
// Prints "layout_checked=A steps_checked=B failures=C".
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <functional>
#include <vector>

#include "shard_plan.h"

using namespace ramcrc_shard_plan;

static uint64_t failures = 0;
#define EXPECT(c)                                                                     \
    do {                                                                              \
        if (!(c)) {                                                                   \
            if (failures < 20)                                                        \
                fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);          \
            failures++;                                                               \
        }                                                                             \
    } while (0)

static uint32_t crc_of(uint64_t s) { return uint32_t(s * 0x9E3779B1u) ^ 0xA5A5A5A5u; }
static const uint32_t kPoison = 0xFFFFFFFFu;

static uint64_t check_layout()
{
    uint64_t checked = 0;
    for (uint64_t N = 1; N <= 8; N++) {
        for (uint64_t nseg = 0; nseg <= 4100; nseg++) {
            const uint64_t w = width(nseg, N);
            uint64_t next = 0;
            for (uint64_t r = 0; r < N; r++) {
                uint64_t lo, hi;
                range(nseg, N, r, &lo, &hi);
                EXPECT(lo == next);
                EXPECT(hi >= lo && hi - lo <= w);
                EXPECT(hi - lo == nseg / N || hi - lo == nseg / N + 1);
                EXPECT((hi - lo == nseg / N + 1) == (r < nseg % N));
                next = hi;
            }
            EXPECT(next == nseg);
            std::vector<uint8_t> used(w * N, 0);
            for (uint64_t s = 0; s < nseg; s++) {
                const uint64_t q = owner(s, nseg, N);
                uint64_t lo, hi;
                range(nseg, N, q, &lo, &hi);
                EXPECT(q < N && lo <= s && s < hi);
                const uint64_t g = gather_index(s, nseg, N);
                EXPECT(g == q * w + (s - lo));
                EXPECT(g < w * N);
                if (g < w * N) {
                    EXPECT(!used[g]);
                    used[g] = 1;
                }
                checked++;
            }
        }
    }
    return checked;
}

// ---------------------------------------------------------------- steps
struct Rank {
    std::vector<uint32_t> gather, all, caller;   // device buffers
    std::vector<std::function<void()>> before, after;   // stream work around the collective
    bool gathered = false;
    uint64_t off = 0, count = 0;
    bool to_caller = false;
    int failed = 0;
};

struct World {
    int N;
    std::vector<Rank> r;
    int fail_rank = -1;   // scan of this rank fails
    void run_streams(uint64_t nseg)
    {
        for (Rank& k : r)
            for (auto& f : k.before)
                f();
        bool all = true;
        for (Rank& k : r)
            all = all && k.gathered;
        EXPECT(all);   // otherwise the real collective would block forever
        if (all) {
            // every rank contributes [off, off + count) of its buffer
            std::vector<std::vector<uint32_t>*> bufs;
            for (Rank& k : r)
                bufs.push_back(k.to_caller ? &k.caller : &k.gather);
            for (int src = 0; src < N; src++)
                for (int dst = 0; dst < N; dst++)
                    if (src != dst)
                        memcpy(bufs[dst]->data() + r[src].off, bufs[src]->data() + r[src].off,
                               r[src].count * sizeof(uint32_t));
        }
        for (Rank& k : r)
            for (auto& f : k.after)
                f();
        for (Rank& k : r) {
            k.before.clear();
            k.after.clear();
            k.gathered = false;
        }
    }
};

// Ops of one process driving local ranks `ranks` of the world.
struct HostOps {
    World* w;
    std::vector<int> ranks;
    bool have_all;
    Rank& R(int k) { return w->r[ranks[k]]; }
    std::vector<uint32_t>& recv(int k, bool caller) { return caller ? R(k).caller : R(k).gather; }
    int check(int, uint64_t, uint64_t) { return 0; }
    int reserve(int k, uint64_t g, uint64_t a)
    {
        if (g)
            R(k).gather.assign(g, 0xDEADBEEFu);
        if (a)
            R(k).all.assign(a, 0xDEADBEEFu);
        R(k).failed = 0;
        return 0;
    }
    int scan(int k, uint64_t lo, uint64_t hi, bool caller, uint64_t off)
    {
        if (ranks[k] == w->fail_rank)
            return -3;
        std::vector<uint32_t>* b = &recv(k, caller);
        EXPECT(off + (hi - lo) <= b->size());
        R(k).before.push_back([b, lo, hi, off] {
            for (uint64_t s = lo; s < hi; s++)
                (*b)[off + s - lo] = crc_of(s);
        });
        return 0;
    }
    int poison(int k, bool caller, uint64_t off, uint64_t count)
    {
        std::vector<uint32_t>* b = &recv(k, caller);
        R(k).before.push_back([b, off, count] {
            for (uint64_t j = 0; j < count; j++)
                (*b)[off + j] = kPoison;
        });
        return 0;
    }
    int group_start() { return 0; }
    int group_end() { return 0; }
    int all_gather(int k, bool caller, uint64_t off, uint64_t count)
    {
        Rank& x = R(k);
        x.gathered = true;
        x.off = off;
        x.count = count;
        x.to_caller = caller;
        EXPECT((off + count) <= recv(k, caller).size());
        return 0;
    }
    int unpad(int k, uint64_t nseg, uint64_t nranks)
    {
        Rank* x = &R(k);
        const bool to_caller = have_all;
        x->after.push_back([x, nseg, nranks, to_caller] {
            std::vector<uint32_t>& dst = to_caller ? x->caller : x->all;
            for (uint64_t s = 0; s < nseg; s++)
                dst[s] = x->gather[gather_index(s, nseg, nranks)];
        });
        return 0;
    }
    void set_failed(int k, int rc) { R(k).failed = rc; }
};

static uint64_t check_steps()
{
    uint64_t checked = 0;
    const uint64_t sizes[] = {0, 1, 2, 3, 7, 8, 9, 15, 16, 17, 255, 256, 257, 1000, 2048, 2049};
    for (int N = 1; N <= 8; N++) {
        for (uint64_t nseg : sizes) {
            for (int have_all = 0; have_all < 2; have_all++) {
                for (int per_process = 0; per_process < 2; per_process++) {
                    for (int fail = -1; fail < (N > 1 ? 1 : 0); fail++) {
                        World w;
                        w.N = N;
                        w.r.resize(N);
                        w.fail_rank = fail < 0 ? -1 : N - 1;
                        for (Rank& k : w.r)
                            k.caller.assign(nseg, 0xDEADBEEFu);
                        std::vector<int> rcs(N, 0);
                        if (per_process) {
                            for (int p = 0; p < N; p++) {
                                HostOps ops{&w, {p}, bool(have_all)};
                                int one = p;
                                rcs[p] = run_step(ops, 1, &one, N, nseg, have_all);
                            }
                        } else {
                            HostOps ops{&w, {}, bool(have_all)};
                            std::vector<int> ranks(N);
                            for (int p = 0; p < N; p++)
                                ops.ranks.push_back(p), ranks[p] = p;
                            const int rc = run_step(ops, N, ranks.data(), N, nseg, have_all);
                            for (int p = 0; p < N; p++)
                                rcs[p] = rc;
                        }
                        if (nseg == 0)
                            continue;
                        w.run_streams(nseg);
                        uint64_t flo = 0, fhi = 0;
                        if (w.fail_rank >= 0)
                            range(nseg, N, w.fail_rank, &flo, &fhi);
                        for (int p = 0; p < N; p++) {
                            const bool failed_here = w.fail_rank == p || (!per_process && w.fail_rank >= 0);
                            EXPECT((rcs[p] != 0) == failed_here);
                            EXPECT((w.r[p].failed != 0) == (w.fail_rank == p));
                            const std::vector<uint32_t>& got = have_all ? w.r[p].caller : w.r[p].all;
                            for (uint64_t s = 0; s < nseg; s++) {
                                const bool poisoned = s >= flo && s < fhi;
                                EXPECT(got[s] == (poisoned ? kPoison : crc_of(s)));
                                checked++;
                            }
                        }
                    }
                }
            }
        }
    }
    return checked;
}

int main()
{
    const uint64_t a = check_layout();
    const uint64_t b = check_steps();
    printf("layout_checked=%llu steps_checked=%llu failures=%llu\n", (unsigned long long)a,
           (unsigned long long)b, (unsigned long long)failures);
    return failures ? 1 : 0;
}
