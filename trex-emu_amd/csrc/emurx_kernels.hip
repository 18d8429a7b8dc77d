// emurx_kernels.hip — CDNA4 (gfx950) kernels of the TRex-EMU receive path.
//
// Two wait-free launches per batch (no workgroup ever waits for another):
//   k_rx  one frame per lane, wave64: descriptors -> per-wave LDS staging of the frames'
//         bytes (coalesced 16-B loads of the wave's contiguous byte range) -> header decode
//         + IPv4 / L4 checksum -> Namespace / Client probes (emurx_parse.h) -> 32-B record,
//         1-B queue tag, per-tile queue counts, per-group queue totals (atomic adds into
//         one of ngroups = ntiles/64 rows), outcome-histogram shard.
//   k_q   stable per-callback queues of frame indices: a tile's exclusive prefix is the
//         totals of the groups before it (one lane per group) + the counts of its earlier
//         group mates (one lane per tile) — two loads per lane, no scan launch, no chain;
//         ranks inside the tile by wave ballots.  The last workgroup to finish folds the
//         histogram shards into the caller's histogram and clears the group totals, so the
//         pair of launches needs no host-side state (replayable from a hipGraph).
// No MFMA: there is no dense contraction on this path; it is HBM / latency bound.
#include <hip/hip_runtime.h>

#include "../../include/emu_rx.h"
#include "emurx_kernels.h"
#include "emurx_parse.h"
#include "emurx_tables.h"

namespace emurx {

static_assert(EMURX_TILE == kBlock, "one frame per lane per tile");
constexpr uint32_t kGroup = 64;  // tiles per group total (one wave lane each)

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}

// ---------------------------------------------------------------------------------------
// k_rx: parse + classify, one tile of 256 frames per workgroup
// ---------------------------------------------------------------------------------------
template <bool kClassify>
__global__ __launch_bounds__(kBlock) void k_rx(const uint8_t* __restrict__ frames,
                                               const emurx_desc* __restrict__ desc, uint32_t n,
                                               emurx_dev_tables T, emurx_rec* __restrict__ rec,
                                               uint8_t* __restrict__ qtag,
                                               uint32_t* __restrict__ tile_cnt,
                                               uint32_t* __restrict__ gsum,
                                               unsigned long long* __restrict__ hshard) {
    __shared__ __attribute__((aligned(16))) uint32_t slab[kWaves * kStage / 4];
    __shared__ uint32_t s_qcnt[16];
    __shared__ unsigned long long s_hpk[EMURX_HIST_BINS], s_hby[EMURX_HIST_BINS];

    const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid / kWave;
    const uint32_t tile = blockIdx.x;
    const uint32_t i = tile * EMURX_TILE + tid;
    const bool valid = i < n;
    if (tid < 16) s_qcnt[tid] = 0;
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
            if (kClassify) classify(s, len, T, r);
        } else {
            GlbSrc s{frames + off};
            parse_packet(s, len, vport, T.cb_mask, r);
            if (kClassify) classify(s, len, T, r);
        }
        if (rec) {
            uint4* o = reinterpret_cast<uint4*>(rec + i);
            o[0] = make_uint4(r.ns, r.cl, r.vlan0, r.vlan1);
            o[1] = make_uint4(r.vport | (r.l3 << 16), r.l4 | (r.l7 << 16),
                              r.l7len | (r.nh << 16) | (r.proto << 24), r.status | (r.flags << 8));
        }
    }
    const uint32_t q = valid ? (r.status == EMURX_ST_OK ? r.proto : EMURX_Q_DROP) : 0xffu;
    if (valid) qtag[i] = (uint8_t)q;

    // per-wave queue counts -> tile counts
    uint32_t mycnt = 0;
#pragma unroll
    for (uint32_t qq = 0; qq < EMURX_NUM_QUEUES; ++qq) {
        const uint64_t m = __ballot(q == qq);
        if (lane == qq) mycnt = (uint32_t)__popcll(m);
    }
    if (lane < EMURX_NUM_QUEUES && mycnt) atomicAdd(&s_qcnt[lane], mycnt);

    // outcome histogram: one LDS add per distinct (status, proto) bin per wave
    const uint32_t bin = valid ? EMURX_HIST_BIN(r.status, r.proto) : 0xffffffffu;
    uint64_t active = __ballot(valid);
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
    if (tid < 16) {
        const uint32_t c = s_qcnt[tid];
        tile_cnt[tile * 16 + tid] = c;
        if (c) atomicAdd(&gsum[(tile / kGroup) * 16 + tid], c);
    }
    // one of EMURX_HIST_SHARDS copies per workgroup: same-address memory-side atomics from
    // every workgroup would serialise
    if (tid >= 64 && tid < 64 + EMURX_HIST_BINS && s_hpk[tid - 64]) {
        const uint32_t b = tid - 64;
        unsigned long long* hs = hshard + (size_t)(tile & (EMURX_HIST_SHARDS - 1)) * 2 * EMURX_HIST_BINS;
        atomicAdd(&hs[2 * b], s_hpk[b]);
        atomicAdd(&hs[2 * b + 1], s_hby[b]);
    }
}

// ---------------------------------------------------------------------------------------
// k_q: stable per-callback queue regions (runs after k_rx: every count is final)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_q(const uint8_t* __restrict__ qtag, uint32_t n,
                                              uint32_t ntiles,
                                              const uint32_t* __restrict__ tile_cnt,
                                              uint32_t* __restrict__ gsum,
                                              uint32_t* __restrict__ qlist, uint32_t qcap,
                                              uint32_t* __restrict__ qcount,
                                              unsigned long long* __restrict__ hshard,
                                              unsigned long long* __restrict__ hist_out,
                                              emurx_ctl* __restrict__ ctl) {
    __shared__ uint32_t s_excl[16], s_wcnt[kWaves][16], s_last;
    const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid / kWave;
    const uint32_t tile = blockIdx.x, g = tile / kGroup, j = tile % kGroup;
    const uint32_t i = tile * EMURX_TILE + tid;
    const uint32_t q = i < n ? qtag[i] : 0xffu;
    const uint32_t dbg = ctl->rsv[1];  // EMURX_DBG_KQ ablation bits (0 in production)

    if (wv == 0) {
        // exclusive prefix of every queue over tiles [0, tile)
        uint32_t part[EMURX_NUM_QUEUES];
#pragma unroll
        for (int k = 0; k < EMURX_NUM_QUEUES; ++k) part[k] = 0;
        for (uint32_t g0 = 0; g0 < ((dbg & 1u) ? 0u : g); g0 += kWave) {  // full groups before ours
            const uint32_t gl = g0 + lane;
            if (gl < g) {
                const uint4* p = reinterpret_cast<const uint4*>(gsum + (size_t)gl * 16);
                const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
                part[0] += a.x; part[1] += a.y; part[2] += a.z; part[3] += a.w;
                part[4] += b.x; part[5] += b.y; part[6] += b.z; part[7] += b.w;
                part[8] += c.x; part[9] += c.y; part[10] += c.z; part[11] += c.w;
                part[12] += d.x;
            }
        }
        if (lane < j) {  // earlier tiles of our group
            const uint4* p = reinterpret_cast<const uint4*>(tile_cnt + (size_t)(g * kGroup + lane) * 16);
            const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
            part[0] += a.x; part[1] += a.y; part[2] += a.z; part[3] += a.w;
            part[4] += b.x; part[5] += b.y; part[6] += b.z; part[7] += b.w;
            part[8] += c.x; part[9] += c.y; part[10] += c.z; part[11] += c.w;
            part[12] += d.x;
        }
        uint32_t mine = 0;
#pragma unroll
        for (int k = 0; k < EMURX_NUM_QUEUES; ++k) {
            const uint32_t v = wave_sum_u32(part[k]);
            if (lane == (uint32_t)k) mine = v;
        }
        if (lane < 16) {
            s_excl[lane] = lane < EMURX_NUM_QUEUES ? mine : 0;
            if (tile == ntiles - 1 && qcount)
                qcount[lane] = lane < EMURX_NUM_QUEUES ? mine + tile_cnt[tile * 16 + lane] : 0;
        }
    }
    // ranks inside the tile: per wave ballots, waves in order
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint32_t rank = 0, mycnt = 0;
#pragma unroll
    for (uint32_t qq = 0; qq < EMURX_NUM_QUEUES; ++qq) {
        const uint64_t m = __ballot(q == qq);
        if (q == qq) rank = (uint32_t)__popcll(m & lt);
        if (lane == qq) mycnt = (uint32_t)__popcll(m);
    }
    if (lane < 16) s_wcnt[wv][lane] = mycnt;
    __syncthreads();
    if (!(dbg & 8u) && qlist && q < EMURX_NUM_QUEUES) {
        uint32_t pos = s_excl[q] + rank;
        for (uint32_t w = 0; w < wv; ++w) pos += s_wcnt[w][q];
        if (pos < qcap) qlist[(size_t)q * qcap + pos] = i;
    }

    // Last workgroup out folds the histogram shards and clears the group rows.  The done
    // count is hierarchical: word 13 of each group row counts that group's workgroups and
    // only a group's last one touches the global word (one returning atomic per address
    // from every workgroup would serialise).  Nothing written here is read by another
    // workgroup of this launch, so relaxed atomics suffice.
    __syncthreads();  // this workgroup's gsum / tile_cnt reads are complete
    const uint32_t ngroups = (ntiles + kGroup - 1) / kGroup;
    if (tid == 0) {
        const uint32_t gsize = min(kGroup, ntiles - g * kGroup);
        uint32_t last = 0;
        if (!(dbg & 4u) && atomicAdd(&gsum[g * 16 + EMURX_NUM_QUEUES], 1u) == gsize - 1)
            last = atomicAdd(&ctl->done, 1u) == ngroups - 1;
        s_last = last && !(dbg & 2u);
    }
    __syncthreads();
    if (s_last) {
        __shared__ unsigned long long s_half[2 * EMURX_HIST_BINS];
        static_assert(kBlock == 2 * 2 * EMURX_HIST_BINS && EMURX_HIST_SHARDS == 64, "fold layout");
        const uint32_t w = tid & (2 * EMURX_HIST_BINS - 1), h = tid / (2 * EMURX_HIST_BINS);
        unsigned long long* p = hshard + (size_t)(32 * h) * 2 * EMURX_HIST_BINS + w;
        unsigned long long v[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) v[k] = p[(size_t)k * 2 * EMURX_HIST_BINS];  // 32 loads in flight
        unsigned long long sum = 0;
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            sum += v[k];
            if (v[k]) p[(size_t)k * 2 * EMURX_HIST_BINS] = 0;
        }
        if (h == 1) s_half[w] = sum;
        __syncthreads();
        if (h == 0 && (sum | s_half[w])) hist_out[w] += sum + s_half[w];
        for (uint32_t k = tid; k < ngroups * 16; k += kBlock) gsum[k] = 0;
        if (tid == 0) ctl->done = 0;
    }
}

}  // namespace emurx

// ---------------------------------------------------------------------------------------
// launcher (called by emurx_api.cpp)
// ---------------------------------------------------------------------------------------
int emurx_launch_batch(const uint8_t* frames, const emurx_desc* desc, uint32_t n,
                       const emurx_dev_tables& T, bool classify, const emurx_dev_out& out,
                       const emurx_scratch& s, hipStream_t st, const hipEvent_t* ev) {
    using namespace emurx;
    if (ev) (void)hipEventRecord(ev[0], st);
    if (n == 0) {
        if (out.qcount) (void)hipMemsetAsync(out.qcount, 0, 16 * sizeof(uint32_t), st);
    } else {
        const uint32_t ntiles = (n + EMURX_TILE - 1) / EMURX_TILE;
        emurx_rec* rec = out.rec;
        if (classify)
            hipLaunchKernelGGL(k_rx<true>, dim3(ntiles), dim3(kBlock), 0, st, frames, desc, n, T, rec,
                               s.qtag, s.tile_cnt, s.gsum, s.hshard);
        else
            hipLaunchKernelGGL(k_rx<false>, dim3(ntiles), dim3(kBlock), 0, st, frames, desc, n, T, rec,
                               s.qtag, s.tile_cnt, s.gsum, s.hshard);
        if (ev) (void)hipEventRecord(ev[1], st);
        hipLaunchKernelGGL(k_q, dim3(ntiles), dim3(kBlock), 0, st, s.qtag, n, ntiles, s.tile_cnt, s.gsum,
                           out.qlist, out.qcap, out.qcount, s.hshard,
                           reinterpret_cast<unsigned long long*>(out.hist), s.ctl);
    }
    if (ev && n == 0) (void)hipEventRecord(ev[1], st);
    if (ev) (void)hipEventRecord(ev[2], st);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
