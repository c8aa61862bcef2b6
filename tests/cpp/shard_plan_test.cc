// Host unit test of the recovery-scan shard's layout and step orchestration
// (ramcloud_amd/csrc/shard_plan.h), the code ramcrc_shard_segments runs on
// every rank, with host stand-ins for the scan kernel (a known value per
// segment), the HIP streams (per-rank queues executed later), the RCCL
// all-gathers (executed only when every rank has reached them -- a rank that
// skipped one would hang the real collective, and fails the test here) and
// the synchronous status exchange of growth steps (a real rendezvous of
// threads: one thread per process).
//
//   layout:  nseg 0..4100 x N 1..8: ranges partition [0, nseg), sizes differ
//            by at most one, every segment's gather slot is inside its owner's
//            block and distinct;
//   steps:   N 1..8, both process models (one process driving all ranks, one
//            process -- thread -- per rank), with and without a caller output
//            array, on divisible and ragged batches: every rank ends with
//            every CRC in segment order, and a repeated step allocates and
//            exchanges nothing before its collective;
//   faults:  on one rank of N = 2..8, (a) the scan launch fails, (b) the
//            arguments fail their check, (c) the buffer growth fails.  In (a)
//            and (b) the rank still takes part in the collective, its slots
//            are poisoned and every peer's sync reports kPeerFailed; in (c)
//            every rank returns before the data collective (the failing rank
//            its own error, the others kPeerFailed) and the next step, whose
//            growth succeeds, completes on every rank.
// Prints "layout_checked=A steps_checked=B failures=C".
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "shard_plan.h"

using namespace ramcrc_shard_plan;

static std::atomic<uint64_t> failures{0};
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
static const uint32_t kUnset = 0xDEADBEEFu;
static const int kScanErr = -3, kCheckErr = -1, kNoMem = -2;

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
enum Fault { kNone, kScan, kCheck, kReserve };

struct Rank {
    std::vector<uint32_t> gather, all, caller, status;   // device buffers
    std::vector<std::function<void()>> before, after;    // stream work around the collective
    bool gathered = false, status_gathered = false;
    uint64_t off = 0, count = 0;
    bool to_caller = false;
    int failed = 0;
};

struct World {
    int N = 0;
    std::vector<Rank> r;
    int fault_rank = -1;
    Fault fault = kNone;
    bool reserve_fails = false;   // armed for the first growth step only
    // rendezvous of the synchronous status exchange (agree)
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<uint32_t> exchange;

    void run_streams()
    {
        for (Rank& k : r)
            for (auto& f : k.before)
                f();
        int ng = 0, ns = 0;
        for (Rank& k : r) {
            ng += k.gathered;
            ns += k.status_gathered;
        }
        // all ranks in the collective, or none (a step every rank left early)
        EXPECT(ng == 0 || ng == N);
        EXPECT(ns == ng);
        if (ng == N) {
            std::vector<std::vector<uint32_t>*> bufs;
            for (Rank& k : r)
                bufs.push_back(k.to_caller ? &k.caller : &k.gather);
            for (int src = 0; src < N; src++)
                for (int dst = 0; dst < N; dst++)
                    if (src != dst) {
                        memcpy(bufs[dst]->data() + r[src].off, bufs[src]->data() + r[src].off,
                               r[src].count * sizeof(uint32_t));
                        r[dst].status[src] = r[src].status[src];
                    }
        }
        for (Rank& k : r)
            for (auto& f : k.after)
                f();
        for (Rank& k : r) {
            k.before.clear();
            k.after.clear();
            k.gathered = k.status_gathered = false;
        }
    }
};

// Ops of one process driving local ranks `ranks` of the world.
struct HostOps {
    World* w;
    std::vector<int> ranks;
    bool have_all;
    uint64_t cap = 0;
    int agrees = 0, reserves = 0;
    Rank& R(int k) { return w->r[ranks[k]]; }
    std::vector<uint32_t>& recv(int k, bool caller) { return caller ? R(k).caller : R(k).gather; }
    uint64_t capacity() const { return cap; }
    void set_capacity(uint64_t c) { cap = c; }
    int reserve(int k, uint64_t elems)
    {
        reserves++;
        if (w->fault == kReserve && w->reserve_fails && ranks[k] == w->fault_rank)
            return kNoMem;
        if (R(k).gather.size() < elems)
            R(k).gather.assign(elems, kUnset);
        if (R(k).all.size() < elems)
            R(k).all.assign(elems, kUnset);
        return 0;
    }
    int agree(const int* st)
    {
        agrees++;
        std::unique_lock<std::mutex> lk(w->mu);
        for (size_t k = 0; k < ranks.size(); k++)
            w->exchange[ranks[k]] = uint32_t(st[k]);
        w->arrived += int(ranks.size());
        const uint64_t g0 = w->gen;
        if (w->arrived == w->N) {
            for (Rank& x : w->r)
                x.status = w->exchange;
            w->arrived = 0;
            w->gen++;
            w->cv.notify_all();
        } else {
            w->cv.wait(lk, [&] { return w->gen != g0; });
        }
        int own = 0;
        for (size_t k = 0; k < ranks.size(); k++)
            if (!own && st[k])
                own = st[k];
        return own ? own : peer_status(0, R(0).status.data(), w->N);
    }
    int check(int k, uint64_t, uint64_t)
    {
        return w->fault == kCheck && ranks[k] == w->fault_rank ? kCheckErr : 0;
    }
    int scan(int k, uint64_t lo, uint64_t hi, bool caller, uint64_t off)
    {
        if (w->fault == kScan && ranks[k] == w->fault_rank)
            return kScanErr;
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
        EXPECT(off + count <= b->size());
        R(k).before.push_back([b, off, count] {
            for (uint64_t j = 0; j < count; j++)
                (*b)[off + j] = kPoison;
        });
        return 0;
    }
    int put_status(int k, int rc)
    {
        Rank* x = &R(k);
        const int me = ranks[k];
        x->before.push_back([x, me, rc] { x->status[me] = uint32_t(rc); });
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
    int all_gather_status(int k)
    {
        R(k).status_gathered = true;
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

// One step of the whole world; returns each rank's return code.
static std::vector<int> world_step(World& w, std::vector<HostOps>& procs, bool per_process,
                                   uint64_t nseg, bool have_all)
{
    const int N = w.N;
    std::vector<int> rcs(N, 0);
    for (Rank& k : w.r)
        k.failed = 0;
    if (per_process) {
        std::vector<std::thread> th;
        for (int p = 0; p < N; p++)
            th.emplace_back([&, p] {
                int one = p;
                rcs[p] = run_step(procs[p], 1, &one, N, nseg, have_all);
            });
        for (auto& t : th)
            t.join();
    } else {
        std::vector<int> ranks(N);
        for (int p = 0; p < N; p++)
            ranks[p] = p;
        const int rc = run_step(procs[0], N, ranks.data(), N, nseg, have_all);
        for (int p = 0; p < N; p++)
            rcs[p] = rc;
    }
    w.run_streams();
    return rcs;
}

static uint64_t check_steps()
{
    uint64_t checked = 0;
    const uint64_t sizes[] = {0, 1, 2, 3, 7, 8, 9, 15, 16, 17, 255, 256, 257, 1000, 2048, 2049};
    for (int N = 1; N <= 8; N++)
        for (uint64_t nseg : sizes)
            for (int have_all = 0; have_all < 2; have_all++)
                for (int per_process = 0; per_process < 2; per_process++)
                    for (int f = kNone; f <= (N > 1 ? kReserve : kNone); f++) {
                        World w;
                        w.N = N;
                        w.r.resize(N);
                        w.exchange.assign(N, 0);
                        w.fault = Fault(f);
                        w.fault_rank = f == kNone ? -1 : N - 1 - int(nseg % N);
                        w.reserve_fails = true;
                        for (Rank& k : w.r) {
                            k.caller.assign(nseg, kUnset);
                            k.status.assign(N, 0);
                        }
                        std::vector<HostOps> procs;
                        if (per_process)
                            for (int p = 0; p < N; p++)
                                procs.push_back(HostOps{&w, {p}, bool(have_all)});
                        else {
                            procs.push_back(HostOps{&w, {}, bool(have_all)});
                            for (int p = 0; p < N; p++)
                                procs[0].ranks.push_back(p);
                        }
                        for (int step = 0; step < 2; step++) {
                            const std::vector<int> rcs =
                                world_step(w, procs, per_process, nseg, have_all);
                            if (nseg == 0) {
                                for (int p = 0; p < N; p++)
                                    EXPECT(rcs[p] == 0);
                                continue;
                            }
                            // growth only on the first step, or again after a failed one
                            const bool grow_failed = f == kReserve && step == 0;
                            for (HostOps& o : procs)
                                EXPECT(o.agrees == (f == kReserve ? step + 1 : 1));
                            const Fault eff = f == kReserve && step > 0 ? kNone : Fault(f);
                            uint64_t flo = 0, fhi = 0;
                            if (eff == kScan || eff == kCheck)
                                range(nseg, N, w.fault_rank, &flo, &fhi);
                            for (int p = 0; p < N; p++) {
                                const bool me = p == w.fault_rank;
                                const int own = eff == kScan ? kScanErr
                                               : eff == kCheck ? kCheckErr
                                               : eff == kReserve ? kNoMem : 0;
                                // return code of the step
                                if (eff == kNone)
                                    EXPECT(rcs[p] == 0);
                                else if (eff == kReserve)
                                    EXPECT(rcs[p] == (me || !per_process ? own : kPeerFailed));
                                else
                                    EXPECT(rcs[p] == (me || !per_process ? own : 0));
                                // what the rank's sync would report
                                const int sync = peer_status(w.r[p].failed, w.r[p].status.data(), N);
                                EXPECT(sync == (eff == kNone ? 0 : me ? own : kPeerFailed));
                                if (grow_failed || (eff == kCheck && me))
                                    continue;   // no results on this rank
                                const std::vector<uint32_t>& got = have_all ? w.r[p].caller : w.r[p].all;
                                for (uint64_t s = 0; s < nseg; s++) {
                                    const bool poisoned = s >= flo && s < fhi;
                                    EXPECT(got[s] == (poisoned ? kPoison : crc_of(s)));
                                    checked++;
                                }
                            }
                            w.reserve_fails = false;
                        }
                    }
    return checked;
}

int main()
{
    const uint64_t a = check_layout();
    const uint64_t b = check_steps();
    printf("layout_checked=%llu steps_checked=%llu failures=%llu\n", (unsigned long long)a,
           (unsigned long long)b, (unsigned long long)failures.load());
    return failures ? 1 : 0;
}
