// Multi-GPU recovery-scan shard (include/ramcrc.h, "multi-GPU recovery
// shard"): the C-ABI a RAMCloud backup process (C++, no torch) calls to
// spread one recovery batch of replicas over the GPUs of a node.
//
// Reference behaviour: BackupMasterRecovery::CyclicReplicaBuffer::buildNext
// (src/BackupMasterRecovery.cc:743-809) verifies every loaded 8 MiB replica
// on its own -- no replica needs another's bytes -- so the batch partitions
// into contiguous segment ranges, one per GPU, with no data exchange.  The
// only collective is one RCCL all-gather of the 4-byte per-segment results
// (1 KiB per rank at 256 segments per GPU), after which every rank holds the
// whole batch's CRCs in segment order for host-side comparison.
//
// Layout of one step on rank r of N (nseg segments, width = ceil(nseg / N)):
//   gather[r * width + j] = CRC of segment lo_r + j      (ramcrc_segments_device)
//   ncclAllGather in place: gather[q * width + j] on every rank
//   all[s] = gather[q(s) * width + (s - lo_q)]            (k_unpad; skipped
//                                                         when N divides nseg
//                                                         and all == gather)
// RCCL is resolved with dlopen at the first shard call: torch (when present)
// has already loaded librccl.so.1 under the same soname, so one RCCL serves
// the process either way, and programs that never shard need no RCCL at all.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <new>
#include <vector>

#include "ramcrc.h"
#include "shard_plan.h"

static_assert(ramcrc_shard_plan::kPeerFailed == RAMCRC_EPEER, "peer failure code");

namespace {

struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId*);
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*);
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int);
    ncclResult_t (*comm_destroy)(ncclComm_t);
    ncclResult_t (*comm_async_error)(ncclComm_t, ncclResult_t*);
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                               hipStream_t);
    ncclResult_t (*group_start)();
    ncclResult_t (*group_end)();
    const char* (*error_string)(ncclResult_t);
};

const Rccl* rccl()
{
    static Rccl r;
    static bool ok = false;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h)
            h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            fprintf(stderr, "ramcrc: RCCL not loadable: %s\n", dlerror());
            return;
        }
        bool all = true;
        auto sym = [&](const char* name) {
            void* p = dlsym(h, name);
            all = all && p;
            return p;
        };
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
        r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(sym("ncclCommInitAll"));
        r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
        r.comm_async_error =
            reinterpret_cast<decltype(r.comm_async_error)>(sym("ncclCommGetAsyncError"));
        r.all_gather = reinterpret_cast<decltype(r.all_gather)>(sym("ncclAllGather"));
        r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
        r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
        ok = all;
        if (!ok)
            fprintf(stderr, "ramcrc: librccl.so.1 lacks a required symbol\n");
    });
    return ok ? &r : nullptr;
}

int rccl_fail(const Rccl* r, ncclResult_t e, const char* what)
{
    fprintf(stderr, "ramcrc: %s: %s\n", what, r ? r->error_string(e) : "rccl unavailable");
    return RAMCRC_ERCCL;
}

#define RCCLCHK(r, expr, what)                    \
    do {                                          \
        ncclResult_t e_ = (expr);                 \
        if (e_ != ncclSuccess)                    \
            return rccl_fail((r), e_, (what));    \
    } while (0)

#define HIPCHK_S(expr)                            \
    do {                                          \
        if ((expr) != hipSuccess)                 \
            return RAMCRC_EHIP;                   \
    } while (0)

// all[s] = gather[gather_index(s)] (shard_plan.h).
__global__ __launch_bounds__(256) void k_unpad(const uint32_t* gather, uint32_t* all, uint64_t nseg,
                                               uint64_t nranks)
{
    const uint64_t s = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (s >= nseg)
        return;
    all[s] = gather[ramcrc_shard_plan::gather_index(s, nseg, nranks)];
}

struct Local {
    int rank = 0;
    int device = 0;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    ramcrc_ctx* ctx = nullptr;
    uint32_t* gather = nullptr;   // width * nranks
    uint64_t gather_cap = 0;
    uint32_t* all = nullptr;      // nseg (results when the caller passes no d_all)
    uint64_t all_cap = 0;
    uint32_t* status = nullptr;   // nranks words: every rank's status of the last exchange
    uint32_t* h_status = nullptr; // pinned host copy read by ramcrc_shard_sync
    uint64_t last_nseg = 0;
    bool last_internal = false;
    int failed = 0;               // a step's failure after its collective was enqueued
    bool step_status = false;     // the last step exchanged status words (nseg > 0)
};

struct DevGuard {
    int prev = -1;
    explicit DevGuard(int d)
    {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
        (void)hipSetDevice(d);
    }
    ~DevGuard()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

int grow(uint32_t** p, uint64_t* cap, uint64_t n)
{
    if (*cap >= n && *p)
        return RAMCRC_OK;
    // the new buffer first: a failed growth keeps the old one
    uint32_t* q = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&q), n * sizeof(uint32_t)) != hipSuccess)
        return RAMCRC_ENOMEM;
    if (*p) {
        if (hipDeviceSynchronize() != hipSuccess) {
            (void)hipFree(q);
            return RAMCRC_EHIP;
        }
        (void)hipFree(*p);
    }
    *p = q;
    *cap = n;
    return RAMCRC_OK;
}

}  // namespace

struct ramcrc_shard {
    int nranks = 0;
    uint64_t capacity = 0;   // watermark of every local rank's gather/all buffers (shard_plan.h)
    std::vector<Local> local;
    std::mutex mu;
};

namespace {

// Streams and contexts for every local rank (communicators already set).
int finish_create(ramcrc_shard* sh)
{
    for (Local& l : sh->local) {
        DevGuard g(l.device);
        HIPCHK_S(hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking));
        int rc = ramcrc_ctx_create(l.device, &l.ctx);
        if (rc)
            return rc;
        const size_t sb = size_t(sh->nranks) * sizeof(uint32_t);
        if (hipMalloc(reinterpret_cast<void**>(&l.status), sb) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&l.h_status), sb, hipHostMallocDefault) !=
                hipSuccess)
            return RAMCRC_ENOMEM;
        HIPCHK_S(hipMemset(l.status, 0, sb));
        memset(l.h_status, 0, sb);
    }
    return RAMCRC_OK;
}

// The environment of ramcrc_shard_plan::run_step: HIP streams, contexts and RCCL.
struct StepOps {
    ramcrc_shard* sh;
    const Rccl* r;
    const void* const* d_shard;
    uint32_t* const* d_all;
    uint64_t seg_bytes;
    uint32_t flags;

    uint32_t* recv(int k, bool caller) { return caller ? d_all[k] : sh->local[k].gather; }
    // Every argument a rank can get wrong is checked here, inside the step, so
    // that the rank still joins the collectives (shard_plan.h's liveness rule).
    int check(int k, uint64_t lo, uint64_t hi)
    {
        if (hi > lo && (!d_shard || !d_shard[k] || seg_bytes == 0))
            return RAMCRC_EINVAL;
        if (d_all && !d_all[k])
            return RAMCRC_EINVAL;
        return RAMCRC_OK;
    }
    uint64_t capacity() const { return sh->capacity; }
    void set_capacity(uint64_t c) { sh->capacity = c; }
    int reserve(int k, uint64_t elems)
    {
        Local& l = sh->local[k];
        DevGuard g(l.device);
        int rc = grow(&l.gather, &l.gather_cap, elems);
        if (!rc)
            rc = grow(&l.all, &l.all_cap, elems);
        return rc;
    }
    // status[rank] = rc on local rank k's stream
    int put_status(int k, int rc)
    {
        Local& l = sh->local[k];
        DevGuard g(l.device);
        HIPCHK_S(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(l.status + l.rank), rc, 1,
                                   l.stream));
        return RAMCRC_OK;
    }
    int all_gather_status(int k)
    {
        Local& l = sh->local[k];
        RCCLCHK(r, r->all_gather(l.status + l.rank, l.status, 1, ncclUint32, l.comm, l.stream),
                "ncclAllGather(status)");
        return RAMCRC_OK;
    }
    // One status word per rank, exchanged and read back before returning.
    int agree(const int* st)
    {
        const int nlocal = int(sh->local.size());
        int own = 0;
        for (int k = 0; k < nlocal; k++) {
            const int prc = put_status(k, st[k]);
            if (!own)
                own = st[k] ? st[k] : prc;
        }
        int rc = group_start();
        if (rc)
            return rc;
        for (int k = 0; k < nlocal && !rc; k++)
            rc = all_gather_status(k);
        const int ge = group_end();
        if (rc || ge)
            return rc ? rc : ge;
        int peer = 0;
        for (int k = 0; k < nlocal; k++) {
            Local& l = sh->local[k];
            DevGuard g(l.device);
            HIPCHK_S(hipMemcpyAsync(l.h_status, l.status, size_t(sh->nranks) * sizeof(uint32_t),
                                    hipMemcpyDeviceToHost, l.stream));
            HIPCHK_S(hipStreamSynchronize(l.stream));
            if (!peer)
                peer = ramcrc_shard_plan::peer_status(0, l.h_status, sh->nranks);
        }
        return own ? own : peer;
    }
    int scan(int k, uint64_t lo, uint64_t hi, bool caller, uint64_t off)
    {
        Local& l = sh->local[k];
        DevGuard g(l.device);
        return ramcrc_segments_device(l.ctx, d_shard[k], seg_bytes, hi - lo, nullptr,
                                      recv(k, caller) + off, flags, l.stream);
    }
    int poison(int k, bool caller, uint64_t off, uint64_t count)
    {
        Local& l = sh->local[k];
        DevGuard g(l.device);
        HIPCHK_S(hipMemsetAsync(recv(k, caller) + off, 0xFF, count * sizeof(uint32_t), l.stream));
        return RAMCRC_OK;
    }
    int group_start()
    {
        RCCLCHK(r, r->group_start(), "ncclGroupStart");
        return RAMCRC_OK;
    }
    int group_end()
    {
        RCCLCHK(r, r->group_end(), "ncclGroupEnd");
        return RAMCRC_OK;
    }
    int all_gather(int k, bool caller, uint64_t off, uint64_t count)
    {
        Local& l = sh->local[k];
        uint32_t* buf = recv(k, caller);
        RCCLCHK(r, r->all_gather(buf + off, buf, count, ncclUint32, l.comm, l.stream),
                "ncclAllGather");
        return RAMCRC_OK;
    }
    int unpad(int k, uint64_t nseg, uint64_t nranks)
    {
        Local& l = sh->local[k];
        DevGuard g(l.device);
        uint32_t* dst = d_all ? d_all[k] : l.all;
        hipLaunchKernelGGL(k_unpad, dim3((nseg + 255) / 256), dim3(256), 0, l.stream, l.gather,
                           dst, nseg, nranks);
        HIPCHK_S(hipGetLastError());
        return RAMCRC_OK;
    }
    void set_failed(int k, int rc) { sh->local[k].failed = rc; }
};

}  // namespace

extern "C" {

int ramcrc_shard_range(uint64_t nseg, int nranks, int rank, uint64_t* lo, uint64_t* hi)
{
    if (nranks < 1 || rank < 0 || rank >= nranks || !lo || !hi)
        return RAMCRC_EINVAL;
    ramcrc_shard_plan::range(nseg, uint64_t(nranks), uint64_t(rank), lo, hi);
    return RAMCRC_OK;
}

int ramcrc_shard_unique_id(void* id)
{
    if (!id)
        return RAMCRC_EINVAL;
    const Rccl* r = rccl();
    if (!r)
        return RAMCRC_ERCCL;
    ncclUniqueId u;
    RCCLCHK(r, r->get_unique_id(&u), "ncclGetUniqueId");
    static_assert(sizeof(u) == RAMCRC_SHARD_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, sizeof(u));
    return RAMCRC_OK;
}

int ramcrc_shard_create_all(const int* devices, int ndev, ramcrc_shard** out)
{
    if (!out)
        return RAMCRC_EINVAL;
    *out = nullptr;
    if (!devices || ndev < 1)
        return RAMCRC_EINVAL;
    int navail = 0;
    if (hipGetDeviceCount(&navail) != hipSuccess)
        return RAMCRC_ENODEV;
    for (int k = 0; k < ndev; k++) {
        if (devices[k] < 0 || devices[k] >= navail)
            return RAMCRC_ENODEV;
        for (int j = 0; j < k; j++)
            if (devices[j] == devices[k])
                return RAMCRC_EINVAL;   // one rank per GPU
    }
    const Rccl* r = rccl();
    if (!r)
        return RAMCRC_ERCCL;
    ramcrc_shard* sh = new (std::nothrow) ramcrc_shard();
    if (!sh)
        return RAMCRC_ENOMEM;
    sh->nranks = ndev;
    sh->local.resize(ndev);
    std::vector<ncclComm_t> comms(ndev, nullptr);
    ncclResult_t e = r->comm_init_all(comms.data(), ndev, devices);
    if (e != ncclSuccess) {
        delete sh;
        return rccl_fail(r, e, "ncclCommInitAll");
    }
    for (int k = 0; k < ndev; k++) {
        sh->local[k].rank = k;
        sh->local[k].device = devices[k];
        sh->local[k].comm = comms[k];
    }
    int rc = finish_create(sh);
    if (rc) {
        ramcrc_shard_destroy(sh);
        return rc;
    }
    *out = sh;
    return RAMCRC_OK;
}

int ramcrc_shard_create_rank(const void* id, int nranks, int rank, int device, ramcrc_shard** out)
{
    if (!out)
        return RAMCRC_EINVAL;
    *out = nullptr;
    if (!id || nranks < 1 || rank < 0 || rank >= nranks)
        return RAMCRC_EINVAL;
    int navail = 0;
    if (hipGetDeviceCount(&navail) != hipSuccess || device < 0 || device >= navail)
        return RAMCRC_ENODEV;
    const Rccl* r = rccl();
    if (!r)
        return RAMCRC_ERCCL;
    ramcrc_shard* sh = new (std::nothrow) ramcrc_shard();
    if (!sh)
        return RAMCRC_ENOMEM;
    sh->nranks = nranks;
    sh->local.resize(1);
    Local& l = sh->local[0];
    l.rank = rank;
    l.device = device;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclResult_t e;
    {
        DevGuard g(device);
        e = r->comm_init_rank(&l.comm, nranks, u, rank);
    }
    if (e != ncclSuccess) {
        l.comm = nullptr;
        delete sh;
        return rccl_fail(r, e, "ncclCommInitRank");
    }
    int rc = finish_create(sh);
    if (rc) {
        ramcrc_shard_destroy(sh);
        return rc;
    }
    *out = sh;
    return RAMCRC_OK;
}

int ramcrc_shard_destroy(ramcrc_shard* sh)
{
    if (!sh)
        return RAMCRC_OK;
    const Rccl* r = rccl();
    for (Local& l : sh->local) {
        DevGuard g(l.device);
        if (l.stream)
            (void)hipStreamSynchronize(l.stream);
        if (l.comm && r)
            (void)r->comm_destroy(l.comm);
        if (l.ctx)
            ramcrc_ctx_destroy(l.ctx);
        if (l.gather)
            (void)hipFree(l.gather);
        if (l.all)
            (void)hipFree(l.all);
        if (l.status)
            (void)hipFree(l.status);
        if (l.h_status)
            (void)hipHostFree(l.h_status);
        if (l.stream)
            (void)hipStreamDestroy(l.stream);
    }
    delete sh;
    return RAMCRC_OK;
}

int ramcrc_shard_local_count(const ramcrc_shard* sh)
{
    return sh ? int(sh->local.size()) : 0;
}

int ramcrc_shard_info(const ramcrc_shard* sh, int k, int* rank, int* device, void** stream,
                      ramcrc_ctx** ctx)
{
    if (!sh || k < 0 || k >= int(sh->local.size()))
        return RAMCRC_EINVAL;
    const Local& l = sh->local[k];
    if (rank) *rank = l.rank;
    if (device) *device = l.device;
    if (stream) *stream = l.stream;
    if (ctx) *ctx = l.ctx;
    return RAMCRC_OK;
}

int ramcrc_shard_segments(ramcrc_shard* sh, const void* const* d_shard, uint64_t seg_bytes,
                          uint64_t nseg, uint32_t* const* d_all, uint32_t flags)
{
    // (only a missing handle returns here: a null d_shard or seg_bytes == 0
    // fail inside the step, StepOps::check, which still joins the collectives)
    if (!sh)
        return RAMCRC_EINVAL;
    const Rccl* r = rccl();
    if (!r)
        return RAMCRC_ERCCL;
    std::lock_guard<std::mutex> lk(sh->mu);
    const int nlocal = int(sh->local.size());
    std::vector<int> ranks(nlocal);
    for (int k = 0; k < nlocal; k++) {
        ranks[k] = sh->local[k].rank;
        sh->local[k].failed = 0;
    }
    StepOps ops{sh, r, d_shard, d_all, seg_bytes, flags};
    const int rc = ramcrc_shard_plan::run_step(ops, nlocal, ranks.data(), sh->nranks, nseg,
                                               d_all != nullptr);
    for (Local& l : sh->local) {
        l.last_nseg = rc ? 0 : nseg;
        l.last_internal = !d_all;
        // an empty step exchanges nothing (run_step returns before any
        // collective): the status words still on the device are an older
        // step's and must not be reported for this one
        l.step_status = nseg != 0;
    }
    return rc;
}

int ramcrc_shard_sync(ramcrc_shard* sh)
{
    if (!sh)
        return RAMCRC_EINVAL;
    const Rccl* r = rccl();
    for (Local& l : sh->local) {
        DevGuard g(l.device);
        // every rank's status word of the last exchange (shard_plan.h); none
        // for an empty step
        if (l.step_status)
            HIPCHK_S(hipMemcpyAsync(l.h_status, l.status, size_t(sh->nranks) * sizeof(uint32_t),
                                    hipMemcpyDeviceToHost, l.stream));
        else
            memset(l.h_status, 0, size_t(sh->nranks) * sizeof(uint32_t));
        HIPCHK_S(hipStreamSynchronize(l.stream));
        if (r && l.comm) {
            ncclResult_t ae = ncclSuccess;
            RCCLCHK(r, r->comm_async_error(l.comm, &ae), "ncclCommGetAsyncError");
            if (ae != ncclSuccess)
                return rccl_fail(r, ae, "RCCL asynchronous error");
        }
        int rc = ramcrc_ctx_check(l.ctx, l.stream);
        if (rc)
            return rc;
        // own failure (its slots of the last step were poisoned), else a peer's
        rc = ramcrc_shard_plan::peer_status(l.failed, l.h_status, sh->nranks);
        if (rc)
            return rc;
    }
    return RAMCRC_OK;
}

int ramcrc_shard_results(ramcrc_shard* sh, int k, uint32_t* h_out, uint64_t nseg)
{
    if (!sh || k < 0 || k >= int(sh->local.size()) || (nseg && !h_out))
        return RAMCRC_EINVAL;
    Local& l = sh->local[k];
    if (!l.last_internal || nseg != l.last_nseg)
        return RAMCRC_EINVAL;
    if (nseg == 0)
        return RAMCRC_OK;
    DevGuard g(l.device);
    HIPCHK_S(hipStreamSynchronize(l.stream));
    HIPCHK_S(hipMemcpy(h_out, l.all, nseg * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return RAMCRC_OK;
}

}  // extern "C"
