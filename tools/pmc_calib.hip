// FETCH_SIZE calibration for k_rx's access patterns.
//
// One kernel, k_calib, with a known byte count per launch:
//   stream part: 16-B loads per lane, coalesced (a wave reads 1 KiB per step), over S bytes;
//                the frame-streaming pattern of k_rx's staging;
//   probe part:  P random 64-B buckets, each read as four 16-B loads by one lane: the
//                ld_bucket pattern of the Namespace / MAC / IP lookups (csrc/emurx_parse.h).
// rocprofv3 --pmc FETCH_SIZE (and the TCC request counters) on each mode then give the
// factor between the counter and the bytes each pattern actually moves.
//
//   pmc_calib <stream_MB> <table_MB> <probes> [iters]   -> one JSON line (per-launch us, bytes)
// table_MB is rounded down to a power of two of 64-B buckets; probes may be 0.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(256) void k_calib(const uint4* __restrict__ stream, uint64_t stream_vec,
                                               const uint4* __restrict__ tab, uint32_t bmask, uint32_t nprobe,
                                               uint32_t seed, uint32_t* __restrict__ out) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t v = g; v < stream_vec; v += nth) {
        const uint4 x = stream[v];
        acc ^= x.x ^ x.y ^ x.z ^ x.w;
    }
    for (uint64_t p = g; p < nprobe; p += nth) {
        const uint32_t b = mix32((uint32_t)p * 2654435761u ^ seed) & bmask;
        const uint4* q = tab + (size_t)b * 4;
        const uint4 a = q[0], c = q[1], d = q[2], e = q[3];
        acc ^= (a.x ^ a.y ^ a.z ^ a.w) + (c.x ^ c.y ^ c.z ^ c.w) + (d.x ^ d.y ^ d.z ^ d.w) + (e.x ^ e.y ^ e.z ^ e.w);
    }
    if (acc == 0x9e3779b9u) out[g & 1023] = acc;  // keeps the loads; never true for the fill
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s <stream_MB> <table_MB> <probes> [iters]\n", argv[0]);
        return 2;
    }
    const uint64_t s_bytes = (uint64_t)atof(argv[1]) * 1000000ull / 1024 * 1024;
    uint64_t t_bytes = (uint64_t)atof(argv[2]) * 1000000ull;
    const uint32_t nprobe = (uint32_t)strtoul(argv[3], nullptr, 10);
    const int iters = argc > 4 ? atoi(argv[4]) : 12;
    uint32_t nb = 1;
    while ((uint64_t)nb * 2 * 64 <= t_bytes) nb *= 2;
    if (t_bytes == 0) nb = 1;
    t_bytes = (uint64_t)nb * 64;
    uint4 *d_s = nullptr, *d_t = nullptr;
    uint32_t* d_o = nullptr;
    if (s_bytes) CHECK(hipMalloc(&d_s, s_bytes));
    CHECK(hipMalloc(&d_t, t_bytes));
    CHECK(hipMalloc(&d_o, 4096));
    if (s_bytes) CHECK(hipMemset(d_s, 0x11, s_bytes));
    CHECK(hipMemset(d_t, 0x22, t_bytes));
    const uint32_t blocks = 256 * 8 * 4;  // 2M lanes: 32 waves per CU
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float total = 0;
    for (int it = 0; it < iters; ++it) {
        CHECK(hipEventRecord(e0, 0));
        k_calib<<<blocks, 256>>>(d_s, s_bytes / 16, d_t, nb - 1, nprobe, 0x1234567u + 977u * it, d_o);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (it) total += ms;  // the first launch is cold
    }
    const double us = total * 1e3 / (iters > 1 ? iters - 1 : 1);
    printf("{\"stream_bytes\": %llu, \"table_bytes\": %llu, \"probes\": %u, \"probe_bytes\": %llu, "
           "\"iters\": %d, \"us_per_launch\": %.2f}\n",
           (unsigned long long)s_bytes, (unsigned long long)t_bytes, nprobe, (unsigned long long)nprobe * 64ull,
           iters, us);
    CHECK(hipFree(d_o));
    CHECK(hipFree(d_t));
    if (d_s) CHECK(hipFree(d_s));
    return 0;
}
