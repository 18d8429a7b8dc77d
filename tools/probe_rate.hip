// Random 64-B bucket reads: one lane per bucket (four 16-B loads of one line, ld_bucket's
// pattern) against four lanes per bucket (one 16-B load each: a quad reads the line in one
// coalesced access), over tables of several sizes.  Lines per second, per mode.
//   probe_rate <table_MB> <probes> <mode 0|1> [iters]   -> one JSON line
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                                     \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
            exit(1);                                                                                 \
        }                                                                                            \
    } while (0)

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

template <int kMode>
__global__ __launch_bounds__(256) void k_probe(const uint4* __restrict__ tab, uint32_t bmask, uint32_t nprobe,
                                               uint32_t seed, uint32_t* __restrict__ out) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    if (kMode == 0) {
        for (uint64_t p = g; p < nprobe; p += nth) {
            const uint32_t b = mix32((uint32_t)p * 2654435761u ^ seed) & bmask;
            const uint4* q = tab + (size_t)b * 4;
            const uint4 a = q[0], c = q[1], d = q[2], e = q[3];
            acc ^= (a.x ^ a.y ^ a.z ^ a.w) + (c.x ^ c.y ^ c.z ^ c.w) + (d.x ^ d.y ^ d.z ^ d.w) + (e.x ^ e.y ^ e.z ^ e.w);
        }
    } else {
        for (uint64_t t = g; t < (uint64_t)nprobe * 4; t += nth) {
            const uint32_t p = (uint32_t)(t >> 2), part = (uint32_t)(t & 3);
            const uint32_t b = mix32(p * 2654435761u ^ seed) & bmask;
            const uint4 a = tab[(size_t)b * 4 + part];
            acc ^= a.x ^ a.y ^ a.z ^ a.w;
        }
    }
    if (acc == 0x9e3779b9u) out[g & 1023] = acc;
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    uint64_t t_bytes = (uint64_t)atof(argv[1]) * 1000000ull;
    const uint32_t nprobe = (uint32_t)strtoul(argv[2], nullptr, 10);
    const int mode = atoi(argv[3]);
    const int iters = argc > 4 ? atoi(argv[4]) : 12;
    uint32_t nb = 1;
    while ((uint64_t)nb * 2 * 64 <= t_bytes) nb *= 2;
    t_bytes = (uint64_t)nb * 64;
    uint4* d_t = nullptr;
    uint32_t* d_o = nullptr;
    CHECK(hipMalloc(&d_t, t_bytes));
    CHECK(hipMalloc(&d_o, 4096));
    CHECK(hipMemset(d_t, 0x22, t_bytes));
    const uint32_t blocks = 256 * 8 * 4;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float total = 0;
    for (int it = 0; it < iters; ++it) {
        CHECK(hipEventRecord(e0, 0));
        if (mode == 0) k_probe<0><<<blocks, 256>>>(d_t, nb - 1, nprobe, 0x1234567u + 977u * it, d_o);
        else k_probe<1><<<blocks, 256>>>(d_t, nb - 1, nprobe, 0x1234567u + 977u * it, d_o);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (it) total += ms;
    }
    const double us = total * 1e3 / (iters - 1);
    printf("{\"mode\": %d, \"table_bytes\": %llu, \"probes\": %u, \"us\": %.2f, \"glines_per_s\": %.2f}\n", mode,
           (unsigned long long)t_bytes, nprobe, us, nprobe / us / 1e3);
    CHECK(hipFree(d_o));
    CHECK(hipFree(d_t));
    return 0;
}
