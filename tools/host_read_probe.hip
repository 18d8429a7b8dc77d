// host_read_probe.hip — how fast a kernel reads pinned host memory (the zero-copy reads of
// k_ingest_small), against hipMemcpyAsync H2D of the same bytes.
//   hipcc -O3 --offload-arch=gfx950 tools/host_read_probe.hip -o tools/host_read_probe && tools/host_read_probe
// Per size and grid: the kernel reads `bytes` of a pinned buffer (hipHostMallocDefault or
// NonCoherent) with 16-byte loads, kIn in flight per lane, into registers (summed, one word
// written per workgroup) or into LDS by LDS-DMA; median of 15 launches after 3 warm ones.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

template <int kIn>
__global__ __launch_bounds__(256) void k_reg(const uint4* __restrict__ src, size_t nv, unsigned* out) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * 256 * kIn;
    for (size_t b = (size_t)blockIdx.x * 256 * kIn + threadIdx.x; b < nv; b += stride) {
        uint4 x[kIn];
#pragma unroll
        for (int k = 0; k < kIn; ++k) {
            const size_t i = b + (size_t)k * 256;
            x[k] = i < nv ? src[i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < kIn; ++k) acc += x[k].x ^ x[k].y ^ x[k].z ^ x[k].w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int kIn>
__global__ __launch_bounds__(256) void k_lds(const uint4* __restrict__ src, size_t nv, unsigned* out) {
    __shared__ uint4 s[256 * kIn];
    const size_t stride = (size_t)gridDim.x * 256 * kIn;
    for (size_t b = (size_t)blockIdx.x * 256 * kIn + threadIdx.x; b < nv; b += stride) {
#pragma unroll
        for (int k = 0; k < kIn; ++k) {
            const size_t i = std::min(b + (size_t)k * 256, nv - 1);
            __builtin_amdgcn_global_load_lds(src + i, (__attribute__((address_space(3))) void*)&s[k * 256 + (threadIdx.x & ~63u)],
                                             16, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    __syncthreads();
    if (s[threadIdx.x].x == 0x12345678u) out[blockIdx.x] = 1;
}

template <typename K>
static float time_kernel(K k, int grid, const uint4* src, size_t nv, unsigned* out, hipStream_t st) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ms;
    for (int r = 0; r < 18; ++r) {
        CK(hipEventRecord(a, st));
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, src, nv, out);
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float m;
        CK(hipEventElapsedTime(&m, a, b));
        if (r >= 3) ms.push_back(m);
    }
    std::sort(ms.begin(), ms.end());
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms[ms.size() / 2];
}

int main() {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const size_t maxb = 8u << 20;
    unsigned* out;
    CK(hipMalloc(&out, 1 << 20));
    void* dev;
    CK(hipMalloc(&dev, maxb));
    const unsigned flags[2] = {hipHostMallocDefault, hipHostMallocNonCoherent};
    const char* fname[2] = {"default", "noncoherent"};
    for (int f = 0; f < 2; ++f) {
        void* h;
        CK(hipHostMalloc(&h, maxb, flags[f]));
        for (size_t i = 0; i < maxb / 4; ++i) static_cast<unsigned*>(h)[i] = (unsigned)i * 2654435761u;
        for (size_t bytes : {(size_t)65536, (size_t)262144, (size_t)1 << 20, (size_t)4 << 20}) {
            const size_t nv = bytes / 16;
            // H2D copy of the same bytes
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            std::vector<float> ms;
            for (int r = 0; r < 18; ++r) {
                CK(hipEventRecord(a, st));
                CK(hipMemcpyAsync(dev, h, bytes, hipMemcpyHostToDevice, st));
                CK(hipEventRecord(b, st));
                CK(hipEventSynchronize(b));
                float m;
                CK(hipEventElapsedTime(&m, a, b));
                if (r >= 3) ms.push_back(m);
            }
            std::sort(ms.begin(), ms.end());
            printf("{\"mem\": \"%s\", \"bytes\": %zu, \"how\": \"memcpy_h2d\", \"us\": %.2f, \"gbs\": %.2f}\n", fname[f], bytes,
                   ms[ms.size() / 2] * 1e3, bytes / (ms[ms.size() / 2] * 1e6));
            for (int grid : {16, 64, 256, 1024}) {
                const float r4 = time_kernel(k_reg<4>, grid, (const uint4*)h, nv, out, st);
                const float r8 = time_kernel(k_reg<8>, grid, (const uint4*)h, nv, out, st);
                const float l4 = time_kernel(k_lds<4>, grid, (const uint4*)h, nv, out, st);
                printf("{\"mem\": \"%s\", \"bytes\": %zu, \"grid\": %d, \"reg4_us\": %.2f, \"reg8_us\": %.2f, \"lds4_us\": %.2f, "
                       "\"reg4_gbs\": %.2f, \"reg8_gbs\": %.2f, \"lds4_gbs\": %.2f}\n",
                       fname[f], bytes, grid, r4 * 1e3, r8 * 1e3, l4 * 1e3, bytes / (r4 * 1e6), bytes / (r8 * 1e6),
                       bytes / (l4 * 1e6));
            }
            fflush(stdout);
        }
        CK(hipHostFree(h));
    }
    return 0;
}
