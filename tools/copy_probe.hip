// copy_probe.hip — HBM copy variants on one GPU, to pick the ceiling bench.py reports beside
// the roofline (emurx_copy_ceiling_dev).  Read + write bytes over HIP-event time.
//   hipcc -O3 --offload-arch=gfx950 tools/copy_probe.hip -o build/copy_probe && build/copy_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned v4 __attribute__((ext_vector_type(4)));

// kInFlight 16-byte vectors per lane per step, grid-stride; kNt: non-temporal loads and stores
template <int kInFlight, bool kNt>
__global__ __launch_bounds__(256) void k_copy(v4* __restrict__ dst, const v4* __restrict__ src, size_t nv) {
    const size_t stride = (size_t)gridDim.x * 256 * kInFlight;
    for (size_t base = (size_t)blockIdx.x * 256 * kInFlight + threadIdx.x; base < nv; base += stride) {
        v4 x[kInFlight];
#pragma unroll
        for (int k = 0; k < kInFlight; ++k) {
            const size_t i = base + (size_t)k * 256;
            if (kNt) x[k] = i < nv ? __builtin_nontemporal_load(src + i) : v4{0, 0, 0, 0};
            else x[k] = i < nv ? src[i] : v4{0, 0, 0, 0};
        }
#pragma unroll
        for (int k = 0; k < kInFlight; ++k) {
            const size_t i = base + (size_t)k * 256;
            if (i < nv) {
                if (kNt) __builtin_nontemporal_store(x[k], dst + i);
                else dst[i] = x[k];
            }
        }
    }
}

template <int kInFlight, bool kNt>
static void run(const char* name, v4* d, const v4* s, size_t nv, int grid) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_copy<kInFlight, kNt>), dim3(grid), dim3(256), 0, 0, d, s, nv);
    (void)hipEventRecord(e0, 0);
    const int reps = 8;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_copy<kInFlight, kNt>), dim3(grid), dim3(256), 0, 0, d, s, nv);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-22s grid %6d  %7.1f GB/s\n", name, grid, 2.0 * nv * 16 / (ms / reps * 1e-3) / 1e9);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main() {
    const size_t bytes = (size_t)1 << 30, nv = bytes / 16;
    v4 *s = nullptr, *d = nullptr;
    if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
    (void)hipMemset(s, 1, bytes);
    (void)hipMemset(d, 0, bytes);
    for (int grid : {1024, 2048, 4096, 8192, 16384}) {
        run<8, true>("nt x8 (bench's)", d, s, nv, grid);
        run<8, false>("plain x8", d, s, nv, grid);
        run<4, true>("nt x4", d, s, nv, grid);
        run<4, false>("plain x4", d, s, nv, grid);
        run<2, false>("plain x2", d, s, nv, grid);
    }
    (void)hipFree(s);
    (void)hipFree(d);
    return 0;
}
