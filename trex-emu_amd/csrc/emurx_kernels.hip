// emurx_kernels.hip — CDNA4 (gfx950) kernel of the TRex-EMU receive path.
//
// ONE wait-free launch per batch (no workgroup ever reads another's output):
//   k_rx  one frame per lane, wave64, one tile of EMURX_QUEUE_TILE frames per workgroup:
//         descriptors -> per-wave LDS staging of the frames' bytes (coalesced 16-B loads of
//         the wave's contiguous byte range) -> header decode + IPv4 / L4 checksum ->
//         Namespace / Client probes (emurx_parse.h) -> 32-B record -> the frame's index in
//         its callback's queue segment for this tile (rank by wave ballots, waves in order)
//         -> per-tile queue counts -> outcome histogram (one of EMURX_HIST_SHARDS copies).
// Queue q is the concatenation over tiles of qlist[q*qcap + t*TILE .. + tile_cnt[t][q]):
// stable (frame order) without any cross-tile prefix, so no scan launch and no waiting.
// No MFMA: there is no dense contraction on this path; it is HBM / latency bound.
#include <hip/hip_runtime.h>

#include "../../include/emu_rx.h"
#include "emurx_kernels.h"
#include "emurx_parse.h"
#include "emurx_tables.h"

namespace emurx {

static_assert(EMURX_QUEUE_TILE == kBlock, "one frame per lane per tile");

template <bool kClassify>
__global__ __launch_bounds__(kBlock) void k_rx(const uint8_t* __restrict__ frames,
                                               const emurx_desc* __restrict__ desc, uint32_t n,
                                               emurx_dev_tables T, emurx_rec* __restrict__ rec,
                                               uint32_t* __restrict__ qlist, uint32_t qcap,
                                               uint32_t* __restrict__ tile_cnt,
                                               unsigned long long* __restrict__ hist) {
    __shared__ __attribute__((aligned(16))) uint32_t slab[kWaves * kStage / 4];
    __shared__ uint32_t s_wcnt[kWaves][16];
    __shared__ unsigned long long s_hpk[EMURX_HIST_BINS], s_hby[EMURX_HIST_BINS];

    const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid / kWave;
    const uint32_t tile = blockIdx.x;
    const uint32_t i = tile * EMURX_QUEUE_TILE + tid;
    const bool valid = i < n;
    if (tid < EMURX_HIST_BINS) { s_hpk[tid] = 0; s_hby[tid] = 0; }

    const uint2 dd = valid ? *reinterpret_cast<const uint2*>(desc + i) : make_uint2(0, 0);
    const uint32_t off = dd.x, len = dd.y & 0xffff, vport = (dd.y >> 16) & 0xff;

    // the wave's byte range [lo, hi) -> stage into LDS when it fits
    const uint32_t lo = wave_min_u32(valid ? off : 0xffffffffu);
    const uint32_t hi = wave_max_u32(valid ? off + len : 0u);
    const uint32_t start = lo & ~15u;
    const uint32_t nvec = hi > lo ? (hi - start + 15) >> 4 : 0;
    const bool staged = nvec > 0 && nvec <= kStage / 16;
    uint4* wslab = reinterpret_cast<uint4*>(slab) + wv * (kStage / 16);
    if (staged) {  // all loads in flight before the first LDS write (one HBM round trip)
        static_assert(kStage / 16 / kWave == 8, "staging unroll assumes 8 vectors per lane");
        const uint4* src = reinterpret_cast<const uint4*>(frames + start);
        // clamped (always in-bounds) loads: no predication, duplicates hit the cache
#define EMURX_LD(k) const uint4 v##k = src[min(lane + k * kWave, nvec - 1)]
        EMURX_LD(0); EMURX_LD(1); EMURX_LD(2); EMURX_LD(3);
        EMURX_LD(4); EMURX_LD(5); EMURX_LD(6); EMURX_LD(7);
#undef EMURX_LD
#define EMURX_ST(k) if (lane + k * kWave < nvec) wslab[lane + k * kWave] = v##k
        EMURX_ST(0); EMURX_ST(1); EMURX_ST(2); EMURX_ST(3);
        EMURX_ST(4); EMURX_ST(5); EMURX_ST(6); EMURX_ST(7);
#undef EMURX_ST
    }
    // each wave reads only its own slab: a wave-level barrier orders the LDS writes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    Rec r;
    if (valid) {
        if (staged) {
            LdsSrc s{reinterpret_cast<const uint8_t*>(slab), slab, wv * kStage + (off - start)};
            parse_packet(s, len, vport, T.cb_mask, r);
            if (kClassify && !(EMURX_ABL & 2)) classify(s, len, T, r);
        } else {
            GlbSrc s{frames + off};
            parse_packet(s, len, vport, T.cb_mask, r);
            if (kClassify && !(EMURX_ABL & 2)) classify(s, len, T, r);
        }
        if (rec && !(EMURX_ABL & 16)) {
            uint4* o = reinterpret_cast<uint4*>(rec + i);
            o[0] = make_uint4(r.ns, r.cl, r.vlan0, r.vlan1);
            o[1] = make_uint4(r.vport | (r.l3 << 16), r.l4 | (r.l7 << 16),
                              r.l7len | (r.nh << 16) | (r.proto << 24), r.status | (r.flags << 8));
        }
    }
    const uint32_t q = valid ? (r.status == EMURX_ST_OK ? r.proto : EMURX_Q_DROP) : 0xffu;

    // rank inside (wave, queue) and the wave's count per queue
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint32_t rank = 0, mycnt = 0;
#pragma unroll
    for (uint32_t qq = 0; qq < ((EMURX_ABL & 8) ? 0 : EMURX_NUM_QUEUES); ++qq) {
        const uint64_t m = __ballot(q == qq);
        if (q == qq) rank = (uint32_t)__popcll(m & lt);
        if (lane == qq) mycnt = (uint32_t)__popcll(m);
    }
    if (lane < 16) s_wcnt[wv][lane] = mycnt;

    // outcome histogram: one LDS add per distinct (status, proto) bin per wave
    const uint32_t bin = valid ? EMURX_HIST_BIN(r.status, r.proto) : 0xffffffffu;
    uint64_t active = (EMURX_ABL & 4) ? 0 : __ballot(valid);
    while (active) {
        const int leader = __ffsll((long long)active) - 1;
        const uint32_t b = (uint32_t)__shfl((int)bin, leader);
        const uint64_t m = __ballot(bin == b);
        const uint64_t bytes = wave_sum_u64(bin == b ? (uint64_t)len : 0);
        if ((int)lane == leader) {
            atomicAdd(&s_hpk[b], (unsigned long long)__popcll(m));
            atomicAdd(&s_hby[b], (unsigned long long)bytes);
        }
        active &= ~m;
    }
    __syncthreads();

    // this tile's segment of every queue: frames in (wave, lane) order == frame order
    if (qlist && q < EMURX_NUM_QUEUES && !(EMURX_ABL & 8)) {
        uint32_t pos = rank;
        for (uint32_t w = 0; w < wv; ++w) pos += s_wcnt[w][q];
        const size_t at = (size_t)q * qcap + (size_t)tile * EMURX_QUEUE_TILE + pos;
        if ((size_t)tile * EMURX_QUEUE_TILE + pos < qcap) qlist[at] = i;
    }
    if (tile_cnt && tid < 16)
        tile_cnt[(size_t)tile * 16 + tid] =
            s_wcnt[0][tid] + s_wcnt[1][tid] + s_wcnt[2][tid] + s_wcnt[3][tid];
    // one of EMURX_HIST_SHARDS copies per workgroup: same-address memory-side atomics from
    // every workgroup would serialise; the shards are folded on the host
    if (tid >= 64 && tid < 64 + EMURX_HIST_BINS && s_hpk[tid - 64]) {
        const uint32_t b = tid - 64;
        unsigned long long* hs = hist + (size_t)(tile & (EMURX_HIST_SHARDS - 1)) * 2 * EMURX_HIST_BINS;
        atomicAdd(&hs[2 * b], s_hpk[b]);
        atomicAdd(&hs[2 * b + 1], s_hby[b]);
    }
}

}  // namespace emurx

// ---------------------------------------------------------------------------------------
// launcher (called by emurx_api.cpp)
// ---------------------------------------------------------------------------------------
int emurx_launch_batch(const uint8_t* frames, const emurx_desc* desc, uint32_t n,
                       const emurx_dev_tables& T, bool classify, const emurx_dev_out& out,
                       hipStream_t st, const hipEvent_t* ev) {
    using namespace emurx;
    if (ev) (void)hipEventRecord(ev[0], st);
    if (n) {
        const uint32_t ntiles = (n + EMURX_QUEUE_TILE - 1) / EMURX_QUEUE_TILE;
        unsigned long long* hist = reinterpret_cast<unsigned long long*>(out.hist);
        if (classify)
            hipLaunchKernelGGL(k_rx<true>, dim3(ntiles), dim3(kBlock), 0, st, frames, desc, n, T, out.rec,
                               out.qlist, out.qcap, out.tile_cnt, hist);
        else
            hipLaunchKernelGGL(k_rx<false>, dim3(ntiles), dim3(kBlock), 0, st, frames, desc, n, T, out.rec,
                               out.qlist, out.qcap, out.tile_cnt, hist);
    }
    if (ev) (void)hipEventRecord(ev[1], st);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
