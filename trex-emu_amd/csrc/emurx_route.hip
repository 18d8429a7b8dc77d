// emurx_route.hip — Namespace-partitioned exchange, device side (gfx950).
//
// After k_rx has classified a batch, every record whose Namespace was found is sent to the
// GPU that owns that Namespace (emurx_owner of its CTunnelKey hash).  Three
// launches build the all-to-all send buffer in frame order per destination:
//   k_route<false>  per tile of 256 records: destination of each record, counts per
//                   (tile, destination)                                   -> tile_cnt
//   k_route_scan    one workgroup: exclusive prefix over tiles per destination -> tile_off,
//                   totals -> send_count
//   k_route<true>   same ranks again (wave ballots, no atomics) -> send[d * cap + offset]
// The exchange itself (an equal-split all-to-all over RCCL) is issued by the caller on the
// same stream.  Bytes: 32 B read twice + 40 B written per routed record.
#include <hip/hip_runtime.h>

#include "../../include/emu_rx.h"
#include "emurx_kernels.h"
#include "emurx_parse.h"
#include "emurx_tables.h"

namespace emurx {

constexpr uint32_t kScanThreads = 1024;

template <bool kPack>
__global__ __launch_bounds__(kBlock) void k_route(const emurx_rec* __restrict__ rec, uint32_t n,
                                                  uint32_t n_parts, uint32_t my_rank,
                                                  uint32_t* __restrict__ tile_cnt,
                                                  const uint32_t* __restrict__ tile_off,
                                                  emurx_route_rec* __restrict__ send, uint32_t cap) {
    __shared__ uint32_t s_wcnt[kWaves][16];
    const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid / kWave, tile = blockIdx.x;
    const uint32_t i = tile * kBlock + tid;
    if (lane < 16) s_wcnt[wv][lane] = 0;
    uint4 a = make_uint4(EMURX_ID_NONE, 0, 0, 0), b = make_uint4(0, 0, 0, 0);
    if (i < n) {
        const uint4* p = reinterpret_cast<const uint4*>(rec + i);
        a = p[0];
        b = p[1];
    }
    // {ns, client, vlan0, vlan1} {vport | l3 << 16, ...}
    const uint32_t d = a.x != EMURX_ID_NONE ? emurx_owner(emurx_tk_hash(b.x & 0xffffu, a.z, a.w), n_parts) : 0xffu;
    uint32_t rank = 0;
    uint64_t left = __ballot(d != 0xffu);
    while (left) {
        const uint32_t lead = (uint32_t)__ffsll((long long)left) - 1;
        const uint32_t dd = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)lead);
        const uint64_t m = __ballot(d == dd);
        if (d == dd) rank = mbcnt(m);
        if (lane == lead) s_wcnt[wv][dd] = (uint32_t)__popcll(m);
        left &= ~m;
    }
    __syncthreads();
    if (!kPack) {
        if (tid < 16) tile_cnt[tile * 16 + tid] = s_wcnt[0][tid] + s_wcnt[1][tid] + s_wcnt[2][tid] + s_wcnt[3][tid];
        return;
    }
    if (d == 0xffu) return;
    uint32_t pos = tile_off[tile * 16 + d] + rank;
    for (uint32_t w = 0; w < wv; ++w) pos += s_wcnt[w][d];
    if (pos >= cap) return;  // overflow: send_count[d] > cap tells the caller
    uint32_t* o = reinterpret_cast<uint32_t*>(send + (size_t)d * cap + pos);  // 40 B, 8-B aligned
    reinterpret_cast<uint2*>(o)[0] = make_uint2(a.x, a.y);
    reinterpret_cast<uint2*>(o)[1] = make_uint2(a.z, a.w);
    reinterpret_cast<uint2*>(o)[2] = make_uint2(b.x, b.y);
    reinterpret_cast<uint2*>(o)[3] = make_uint2(b.z, b.w);
    reinterpret_cast<uint2*>(o)[4] = make_uint2(i, my_rank);
}

// exclusive prefix over tiles of tile_cnt[t][d], d < n_parts; one workgroup of 1024 lanes,
// each owning a contiguous run of tiles
__global__ __launch_bounds__(kScanThreads) void k_route_scan(const uint32_t* __restrict__ tile_cnt,
                                                              uint32_t ntiles, uint32_t n_parts,
                                                              uint32_t* __restrict__ tile_off,
                                                              uint32_t* __restrict__ send_count) {
    __shared__ uint32_t s[EMURX_MAX_PARTS][kScanThreads];
    const uint32_t t = threadIdx.x, lane = lane_id(), wv = t / kWave;
    const uint32_t per = (ntiles + kScanThreads - 1) / kScanThreads;
    const uint32_t t0 = min(t * per, ntiles), t1 = min(t0 + per, ntiles);
    uint32_t run[EMURX_MAX_PARTS];
#pragma unroll
    for (uint32_t d = 0; d < EMURX_MAX_PARTS; ++d) run[d] = 0;
    for (uint32_t k = t0; k < t1; ++k) {
        const uint4* p = reinterpret_cast<const uint4*>(tile_cnt + k * 16);
        const uint4 x = p[0], y = p[1];
        run[0] += x.x; run[1] += x.y; run[2] += x.z; run[3] += x.w;
        run[4] += y.x; run[5] += y.y; run[6] += y.z; run[7] += y.w;
    }
#pragma unroll
    for (uint32_t d = 0; d < EMURX_MAX_PARTS; ++d) s[d][t] = run[d];
    __syncthreads();
    // wave d scans destination d's 1024 run totals: 16 per lane, then across lanes
    if (wv < n_parts) {
        const uint32_t d = wv;
        uint32_t v[16], sum = 0;
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) { v[k] = s[d][lane * 16 + k]; sum += v[k]; }
        uint32_t incl = sum;
#pragma unroll
        for (uint32_t o = 1; o < kWave; o <<= 1) {
            const uint32_t up = (uint32_t)__shfl_up((int)incl, o);
            if (lane >= o) incl += up;
        }
        uint32_t ex = incl - sum;
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) { s[d][lane * 16 + k] = ex; ex += v[k]; }
        if (lane == kWave - 1) send_count[d] = incl;
    }
    __syncthreads();
    uint32_t base[EMURX_MAX_PARTS];
#pragma unroll
    for (uint32_t d = 0; d < EMURX_MAX_PARTS; ++d) base[d] = s[d][t];
    for (uint32_t k = t0; k < t1; ++k) {
        const uint4* p = reinterpret_cast<const uint4*>(tile_cnt + k * 16);
        const uint4 x = p[0], y = p[1];
        uint4* q = reinterpret_cast<uint4*>(tile_off + k * 16);
        q[0] = make_uint4(base[0], base[1], base[2], base[3]);
        q[1] = make_uint4(base[4], base[5], base[6], base[7]);
        base[0] += x.x; base[1] += x.y; base[2] += x.z; base[3] += x.w;
        base[4] += y.x; base[5] += y.y; base[6] += y.z; base[7] += y.w;
    }
}

}  // namespace emurx

int emurx_launch_route(const emurx_rec* rec, uint32_t n, uint32_t n_parts, uint32_t my_rank, uint32_t cap,
                       emurx_route_rec* send, uint32_t* send_count, uint32_t* tile_cnt, uint32_t* tile_off,
                       hipStream_t st) {
    using namespace emurx;
    const uint32_t ntiles = (n + kBlock - 1) / kBlock;
    if (n == 0) return hipMemsetAsync(send_count, 0, n_parts * sizeof(uint32_t), st) == hipSuccess ? 0 : -1;
    hipLaunchKernelGGL(k_route<false>, dim3(ntiles), dim3(kBlock), 0, st, rec, n, n_parts, my_rank, tile_cnt,
                       (const uint32_t*)nullptr, send, cap);
    hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(kScanThreads), 0, st, tile_cnt, ntiles, n_parts, tile_off,
                       send_count);
    hipLaunchKernelGGL(k_route<true>, dim3(ntiles), dim3(kBlock), 0, st, rec, n, n_parts, my_rank, tile_cnt,
                       tile_off, send, cap);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
