// The multi-GPU recovery-scan shard entry (ramcrc_shard_*, Crc32CShard) as a
// RAMCloud backup process would drive it from BackupMasterRecovery::
// CyclicReplicaBuffer::buildNext (src/BackupMasterRecovery.cc:743-809): a
// batch of loaded replicas, each rank's range in its own GPU's memory, CRCs
// of the whole batch back in segment order.
//   shard_test args                 argument validation (no GPU needed)
//   shard_test gpu NSEG SEG_BYTES   every visible GPU one rank; prints
//                                   "crc <i> <hex>" for the parity test
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <stdexcept>
#include <vector>

#include "Crc32CBatch.h"

using namespace RAMCloud;

static int failures = 0;
#define EXPECT(cond)                                                        \
    do {                                                                    \
        if (!(cond)) {                                                      \
            fprintf(stderr, "%s:%d: EXPECT(%s) failed\n", __FILE__, __LINE__, #cond); \
            failures++;                                                     \
        }                                                                   \
    } while (0)

// splitmix64 stream of ramcloud_amd/workloads.py: word j (from 1) of seed s.
static void
splitmix(uint64_t seed, uint8_t* out, uint64_t n)
{
    for (uint64_t j = 0; j < n / 8; j++) {
        uint64_t z = seed + (j + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        memcpy(out + 8 * j, &z, 8);
    }
}

static int
args()
{
    uint64_t lo = 0, hi = 0;
    EXPECT(ramcrc_shard_range(2048, 8, 7, &lo, &hi) == RAMCRC_OK && lo == 1792 && hi == 2048);
    EXPECT(ramcrc_shard_range(11, 3, 0, &lo, &hi) == RAMCRC_OK && lo == 0 && hi == 4);
    EXPECT(ramcrc_shard_range(11, 3, 2, &lo, &hi) == RAMCRC_OK && lo == 8 && hi == 11);
    EXPECT(ramcrc_shard_range(2, 4, 3, &lo, &hi) == RAMCRC_OK && lo == 2 && hi == 2);
    EXPECT(ramcrc_shard_range(8, 0, 0, &lo, &hi) == RAMCRC_EINVAL);
    EXPECT(ramcrc_shard_range(8, 2, 2, &lo, &hi) == RAMCRC_EINVAL);
    EXPECT(ramcrc_shard_range(8, 2, 0, NULL, &hi) == RAMCRC_EINVAL);
    ramcrc_shard* sh = NULL;
    EXPECT(ramcrc_shard_create_all(NULL, 1, &sh) == RAMCRC_EINVAL && sh == NULL);
    const int none[1] = {0};
    EXPECT(ramcrc_shard_create_all(none, 0, &sh) == RAMCRC_EINVAL);
    EXPECT(ramcrc_shard_create_all(none, 1, NULL) == RAMCRC_EINVAL);
    const int dup[2] = {0, 0};
    const int rc_dup = ramcrc_shard_create_all(dup, 2, &sh);
    EXPECT(rc_dup == RAMCRC_EINVAL || rc_dup == RAMCRC_ENODEV);
    const int bad[1] = {-1};
    EXPECT(ramcrc_shard_create_all(bad, 1, &sh) == RAMCRC_ENODEV);
    uint8_t id[RAMCRC_SHARD_ID_BYTES] = {0};
    EXPECT(ramcrc_shard_create_rank(NULL, 1, 0, 0, &sh) == RAMCRC_EINVAL);
    EXPECT(ramcrc_shard_create_rank(id, 2, 2, 0, &sh) == RAMCRC_EINVAL);
    EXPECT(ramcrc_shard_create_rank(id, 0, 0, 0, &sh) == RAMCRC_EINVAL);
    EXPECT(ramcrc_shard_create_rank(id, 1, 0, -1, &sh) == RAMCRC_ENODEV);
    EXPECT(ramcrc_shard_segments(NULL, NULL, 1, 1, NULL, 0) == RAMCRC_EINVAL);
    EXPECT(ramcrc_shard_sync(NULL) == RAMCRC_EINVAL);
    EXPECT(ramcrc_shard_results(NULL, 0, NULL, 0) == RAMCRC_EINVAL);
    EXPECT(ramcrc_shard_local_count(NULL) == 0);
    EXPECT(ramcrc_shard_destroy(NULL) == RAMCRC_OK);
    EXPECT(ramcrc_shard_unique_id(NULL) == RAMCRC_EINVAL);
    // the wrapper throws on the same errors
    bool threw = false;
    try {
        Crc32CShard s(std::vector<int>(1, -1));
    } catch (const std::runtime_error&) {
        threw = true;
    }
    EXPECT(threw);
    EXPECT(Crc32CShard::range(10, 4, 1) == std::make_pair(uint64_t(3), uint64_t(6)));
    printf("args: failures=%d\n", failures);
    return failures ? 1 : 0;
}

static int
gpu(uint64_t nseg, uint64_t seg_bytes)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        fprintf(stderr, "no GPU\n");
        return 1;
    }
    std::vector<int> devs;
    for (int d = 0; d < ndev; d++)
        devs.push_back(d);
    // each rank's replicas land in its own GPU's memory, as the frames a
    // backup loads for one recovery batch
    std::vector<uint8_t> host(seg_bytes);
    std::vector<const void*> shards;
    std::vector<uint32_t*> outs;
    for (int k = 0; k < ndev; k++) {
        std::pair<uint64_t, uint64_t> r = Crc32CShard::range(nseg, ndev, k);
        if (hipSetDevice(devs[k]) != hipSuccess)
            return 1;
        void* d = NULL;
        uint32_t* o = NULL;
        if (hipMalloc(&d, (r.second - r.first) * seg_bytes + 1) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&o), nseg * 4 + 4) != hipSuccess)
            return 1;
        for (uint64_t i = r.first; i < r.second; i++) {
            splitmix(0x52414D43ull + i, host.data(), seg_bytes);
            if (hipMemcpy(static_cast<uint8_t*>(d) + (i - r.first) * seg_bytes, host.data(),
                          seg_bytes, hipMemcpyHostToDevice) != hipSuccess)
                return 1;
        }
        shards.push_back(d);
        outs.push_back(o);
    }
    std::vector<uint32_t> all;
    {
        // single process, every GPU a rank (ncclCommInitAll)
        Crc32CShard shard(devs);
        all = shard.deviceShard(shards, seg_bytes, nseg);
        // the same step into caller-owned device arrays (all-gather straight
        // into them when the split is even)
        ramcrc_shard* raw = NULL;
        EXPECT(ramcrc_shard_create_all(&devs[0], ndev, &raw) == RAMCRC_OK);
        EXPECT(ramcrc_shard_segments(raw, &shards[0], seg_bytes, nseg, &outs[0],
                                     RAMCRC_FINALIZE) == RAMCRC_OK);
        EXPECT(ramcrc_shard_sync(raw) == RAMCRC_OK);
        for (int k = 0; k < ndev; k++) {
            std::vector<uint32_t> got(nseg);
            EXPECT(hipSetDevice(devs[k]) == hipSuccess);
            EXPECT(hipMemcpy(got.data(), outs[k], nseg * 4, hipMemcpyDeviceToHost) == hipSuccess);
            EXPECT(got == all);
        }
        // raw (un-finalized) states: ~ of the results
        EXPECT(ramcrc_shard_segments(raw, &shards[0], seg_bytes, nseg, NULL, 0) == RAMCRC_OK);
        EXPECT(ramcrc_shard_sync(raw) == RAMCRC_OK);
        std::vector<uint32_t> rawv(nseg);
        EXPECT(ramcrc_shard_results(raw, 0, rawv.data(), nseg) == RAMCRC_OK);
        for (uint64_t i = 0; i < nseg; i++)
            EXPECT(rawv[i] == ~all[i]);
        // a rank's bad arguments fail inside the step (it still joins the
        // collectives): no shard pointers, then a zero segment size
        EXPECT(ramcrc_shard_segments(raw, NULL, seg_bytes, nseg, NULL, 0) == RAMCRC_EINVAL);
        EXPECT(ramcrc_shard_sync(raw) == RAMCRC_EINVAL);
        EXPECT(ramcrc_shard_segments(raw, &shards[0], 0, nseg, NULL, 0) == RAMCRC_EINVAL);
        EXPECT(ramcrc_shard_sync(raw) == RAMCRC_EINVAL);
        // an empty step after a failed one reports nothing of the failed one
        EXPECT(ramcrc_shard_segments(raw, &shards[0], seg_bytes, 0, NULL, 0) == RAMCRC_OK);
        EXPECT(ramcrc_shard_sync(raw) == RAMCRC_OK);
        // and the next real step is exact again
        EXPECT(ramcrc_shard_segments(raw, &shards[0], seg_bytes, nseg, NULL, RAMCRC_FINALIZE) ==
               RAMCRC_OK);
        EXPECT(ramcrc_shard_sync(raw) == RAMCRC_OK);
        EXPECT(ramcrc_shard_results(raw, 0, rawv.data(), nseg) == RAMCRC_OK);
        EXPECT(rawv == all);
        ramcrc_shard_destroy(raw);
    }
    if (ndev == 1) {
        // one process per GPU (ncclCommInitRank) with a world of one
        Crc32CShard rank0(Crc32CShard::uniqueId(), 1, 0, devs[0]);
        std::vector<uint32_t> again = rank0.deviceShard(shards, seg_bytes, nseg);
        EXPECT(again == all);
    }
    for (uint64_t i = 0; i < nseg; i++)
        printf("crc %llu %08x\n", static_cast<unsigned long long>(i), all[i]);
    printf("gpu: ranks=%d segments=%llu failures=%d\n", ndev,
           static_cast<unsigned long long>(nseg), failures);
    return failures ? 1 : 0;
}

int
main(int argc, char** argv)
{
    if (argc > 1 && !strcmp(argv[1], "args"))
        return args();
    if (argc > 3 && !strcmp(argv[1], "gpu"))
        return gpu(strtoull(argv[2], NULL, 0), strtoull(argv[3], NULL, 0));
    fprintf(stderr, "usage: shard_test args | gpu NSEG SEG_BYTES\n");
    return 2;
}
