// Read-bandwidth microbenchmark for the access patterns the small-entry CRC
// kernel could use on gfx950 (design input, not product code).
//   coal     : lane l reads 16 B at block + 16 l (1 KiB per wave instruction)
//   lane<R>  : lane l walks its own contiguous R-byte range, 16 B per load
//   grp<G>   : groups of G lanes read G*16 contiguous bytes per instruction
// Each kernel keeps U loads in flight per lane and XOR-reduces the data.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g4;

#define CHECK(x)                                                        \
    do {                                                                \
        hipError_t e = (x);                                             \
        if (e != hipSuccess) {                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                    \
        }                                                               \
    } while (0)

// Each wave owns `per_wave` contiguous bytes; inside it the pattern decides
// which 16 B each lane reads at step k.  mode 0: coalesced; mode 1: lane
// contiguous (range per lane = per_wave/64); mode 2: groups of G lanes.
template <int U, int MODE, int G>
__global__ __launch_bounds__(1024) void k_read(const uint8_t* base, uint64_t per_wave, uint32_t* out)
{
    const int lane = threadIdx.x & 63;
    const uint64_t wave = blockIdx.x * 16 + threadIdx.x / 64;
    const uint64_t nw = gridDim.x * 16ull;
    uint32_t acc = 0;
    const uint64_t steps = per_wave / 1024;  // 16 B per lane per step
    for (uint64_t w = wave; w < 4096; w += nw) {
        const uint8_t* wb = base + w * per_wave;
        const g4* p;
        uint64_t stride;  // in u32x4 units between consecutive steps of this lane
        if (MODE == 0) {
            p = (const g4*)wb + lane;
            stride = 64;
        } else if (MODE == 1) {
            p = (const g4*)(wb + (uint64_t)lane * (per_wave / 64));
            stride = 1;
        } else {
            const int grp = lane / G, gl = lane % G;
            const uint64_t span = per_wave / (64 / G);
            p = (const g4*)(wb + grp * span) + gl;
            stride = G;
        }
        u32x4 buf[U];
#pragma unroll
        for (int j = 0; j < U; j++)
            buf[j] = __builtin_nontemporal_load(p + j * stride);
        for (uint64_t k = U; k < steps; k += U) {
#pragma unroll
            for (int j = 0; j < U; j++) {
                const u32x4 v = buf[j];
                buf[j] = __builtin_nontemporal_load(p + (k + j) * stride);
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        }
#pragma unroll
        for (int j = 0; j < U; j++)
            acc ^= buf[j].x ^ buf[j].y ^ buf[j].z ^ buf[j].w;
    }
    if (acc == 0x12345678u)
        out[0] = acc;
}

template <int U, int MODE, int G>
void run(const char* name, const uint8_t* d, uint64_t bytes, uint32_t* out, int blocks)
{
    const uint64_t per_wave = bytes / 4096;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    k_read<U, MODE, G><<<blocks, 1024>>>(d, per_wave, out);
    CHECK(hipDeviceSynchronize());
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
        CHECK(hipEventRecord(a));
        k_read<U, MODE, G><<<blocks, 1024>>>(d, per_wave, out);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (ms < best)
            best = ms;
    }
    printf("%-24s blocks=%4d  %8.1f GB/s  (%.3f ms)\n", name, blocks, bytes / (best * 1e-3) / 1e9,
           best);
    fflush(stdout);
}

int main()
{
    const uint64_t bytes = 4ull << 30;
    uint8_t* d;
    uint32_t* out;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(d, 0x5a, bytes));
    int ncu = 256;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    ncu = prop.multiProcessorCount;
    printf("device %s CUs=%d\n", prop.gcnArchName, ncu);
    run<8, 0, 1>("coal U8", d, bytes, out, ncu);
    run<16, 0, 1>("coal U16", d, bytes, out, ncu);
    run<4, 0, 1>("coal U4", d, bytes, out, ncu);
    run<8, 0, 1>("coal U8 2x blocks", d, bytes, out, 2 * ncu);
    run<8, 1, 1>("lane-contig U8", d, bytes, out, ncu);
    run<16, 1, 1>("lane-contig U16", d, bytes, out, ncu);
    run<8, 2, 8>("grp8 U8", d, bytes, out, ncu);
    run<16, 2, 8>("grp8 U16", d, bytes, out, ncu);
    run<8, 2, 4>("grp4 U8", d, bytes, out, ncu);
    run<16, 2, 4>("grp4 U16", d, bytes, out, ncu);
    run<8, 2, 16>("grp16 U8", d, bytes, out, ncu);
    run<8, 2, 2>("grp2 U8", d, bytes, out, ncu);
    return 0;
}
