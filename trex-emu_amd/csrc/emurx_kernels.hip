// emurx_kernels.hip — CDNA4 (gfx950) kernel of the TRex-EMU receive path.
//
// ONE wait-free launch per batch (no workgroup ever reads another's output):
//   k_rx  one frame per lane, wave64, one tile of EMURX_QUEUE_TILE frames per workgroup:
//         descriptors -> per-wave LDS staging of the frames' bytes (coalesced 16-B loads of
//         the wave's contiguous byte range) -> header decode + IPv4 / L4 checksum ->
//         Namespace / Client probes (emurx_parse.h) -> 32-B record -> the frame's index in
//         its callback's queue segment for this tile (rank by wave ballots, waves in order)
//         -> per-tile queue counts -> outcome histogram (one of EMURX_HIST_SHARDS copies).
//         Frames reach LDS by LDS-DMA (global_load_lds_dwordx4), with no VGPR round trip.
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


// LDS-DMA (global_load_lds_dwordx4): lane l's 16 source bytes land at dst + 16 * l.  kNt: the
// non-temporal policy (aux bit 1, `nt`) for bytes nothing reads again from memory
template <bool kNt>
__device__ __forceinline__ void glds16(const uint4* src, uint4* dst_wave_base) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst_wave_base, 16, 0,
                                     kNt ? 2 : 0);
}
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0)

// Timeline stamps (measurement-only build, -DEMURX_STAMP=1; tools/stamps.py): per wave the
// shader clock at entry, after the descriptors, after the staging, after the parse, after the
// lookup key, after the table lookups, at the histogram, before and after the tile barrier and
// at exit, then HW_ID, XCC_ID and the tile: 16 u64 per wave, written by lane 0 with vector
// stores.
#ifndef EMURX_STAMP
#define EMURX_STAMP 0
#endif
#if EMURX_STAMP
__device__ unsigned long long* g_stamp;
#define STAMP(k) \
    do { if constexpr (EMURX_STAMP) st_[k] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define STAMP(k) do {} while (0)
#endif

// k_rx's arguments as one struct (a single kernarg block; 91 SGPRs and 76 VGPRs against 106
// and 79 for the same arguments passed one by one)
// EMURX_TOL_PREFETCH (default 1): k_rx<2> issues the tile's owner-offset loads before the
// staging wait (0, A/B builds: wave 0 loads them inside the tile body, one more round trip)
#ifndef EMURX_TOL_PREFETCH
#define EMURX_TOL_PREFETCH 1
#endif
struct RxArgs {
    const uint8_t* frames;
    const emurx_desc* desc;
    uint32_t n;
    emurx_dev_tables T;
    emurx_rec* rec;
    uint32_t* qlist;
    uint32_t qcap;
    uint32_t* tile_cnt;
    unsigned long long* hist;
    uint32_t* flow;
    uint32_t* fb;
    uint32_t gen;
    emurx_route_args rt;
};

// a lane's descriptor of tile t (an empty slot past the batch)
__device__ __forceinline__ uint2 load_desc(const emurx_desc* __restrict__ desc, uint32_t n, uint32_t i) {
    return i < n ? *reinterpret_cast<const uint2*>(desc + i) : make_uint2(0, EMURX_DESC_HOLE << 24);
}

// EMURX_WIN_NT (build variant, A/B): non-temporal window loads (with EMURX_WSKIP the
// cooperative pass reads no window byte again)
#ifndef EMURX_WIN_NT
#define EMURX_WIN_NT 0
#endif
// The wave's staging of its 64 frames into its slab (wslab: the wave's kStage bytes):
// the byte range [lo, hi) of the wave's frames copied HBM -> LDS by LDS-DMA
// (global_load_lds_dwordx4, no VGPR round trip) when it fits the slab, else a window of each
// lane's own frame (headers; the window path).  Issues the loads and returns; the caller waits
// (vmcnt) before reading the slab.
struct Stage {
    uint32_t start, nvec;
    bool staged;
};
template <uint32_t kStage>
__device__ __forceinline__ Stage stage_issue(const uint8_t* __restrict__ frames, uint2 dd, uint32_t lane, uint4* wslab) {
    constexpr uint32_t kWinVec = kStage / 16 / kWave;  // window path: 16-byte vectors per lane
    const bool valid = (dd.y >> 24) != EMURX_DESC_HOLE;  // an empty slot is no frame at all
    const uint32_t off = dd.x, len = dd.y & 0xffff;
    const uint32_t lo = wave_min_u32(valid ? off : 0xffffffffu);
    const uint32_t hi = wave_max_u32(valid ? off + len : 0u);
    Stage sg;
    sg.start = lo & ~15u;
    sg.nvec = hi > lo ? (hi - sg.start + 15) >> 4 : 0;
    sg.staged = sg.nvec > 0 && sg.nvec <= kStage / 16;
    if (sg.staged) {  // all copies in flight before the wait; clamped sources stay in bounds
        static_assert(kStage / 16 <= 8 * kWave, "staging issues at most 8 vectors per lane");
        // each LDS-DMA instruction writes 64 vectors (1 KiB) of the slab; a slab that is not a
        // whole number of them would let the last one run into the next wave's slab
        static_assert(kStage % (16 * kWave) == 0, "slab = whole 1 KiB DMA rows");
        const uint4* src = reinterpret_cast<const uint4*>(frames + sg.start);
#pragma unroll
        for (uint32_t k = 0; k < kStage / 16 / kWave; ++k)
            if (k * kWave < sg.nvec) glds16<true>(src + min(lane + k * kWave, sg.nvec - 1), wslab + k * kWave);
    } else {  // too wide: each lane stages a window of its own frame (headers)
        const uintptr_t fa = (uintptr_t)(frames + off);
        const uint4* src = reinterpret_cast<const uint4*>(fa & ~(uintptr_t)15);
        const uint32_t nv = valid ? (uint32_t)(((fa & 15) + len + 15) >> 4) : 0;  // vectors of the frame
#pragma unroll
        for (uint32_t k = 0; k < kWinVec; ++k)
            if (k < nv) glds16<EMURX_WIN_NT != 0>(src + k, wslab + k * kWave);  // the span past it is read again
    }
    return sg;
}
// the slab's LDS-DMA writes are visible to this wave's reads: vmcnt(0), then a wave-level
// barrier (each wave reads only its own slab)
__device__ __forceinline__ void stage_wait() {
    wait_vm0();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// EMURX_MATCHRANK (build variant, A/B): rank the lanes of a queue / an owner by one ballot
// per bit of its id (the lanes holding the same id, as match_any) instead of one loop
// iteration of scalar bookkeeping per distinct id present in the wave
#ifndef EMURX_MATCHRANK
#define EMURX_MATCHRANK 0
#endif
template <int kBits>
__device__ __forceinline__ uint64_t match_lanes(uint32_t v, uint64_t act) {
    uint64_t m = act;
#pragma unroll
    for (int b = 0; b < kBits; ++b) {
        const bool bit = (v >> b) & 1u;
        const uint64_t x = __ballot(bit);
        m &= bit ? x : ~x;
    }
    return m;
}

// The workgroup's small LDS arrays of one tile
struct TileLds {
    uint32_t wcnt[kWaves][16];                   // queue counts per wave
    uint32_t csum[kWaves][kWave];                // window path: span sums; then the histogram rows
    uint32_t rcnt[kWaves][EMURX_MAX_PARTS];      // Namespace owners
    uint32_t toff[EMURX_MAX_PARTS];              // kKind 2: the tile's offset in each region
};

// kKind: 0 parse only, 1 parse + classify, 2 parse + lookup keys (the partitioned source:
// every frame's emurx_lookup_rec packed straight into its Namespace owner's send region, at
// the offsets the owner-count pass (k_owner_count + k_route_scan) fixed; no table reads).
// One tile (EMURX_QUEUE_TILE frames, one per lane) whose frames are staged in `slab` (the
// workgroup's kWaves slabs of kStage bytes): parse, classify, record, queue segment, counts.
template <int kKind, uint32_t kStage>
__device__ __forceinline__ void tile_body(const RxArgs& a, uint32_t tile, uint2 dd, Stage sg, const uint32_t* slab,
                                          TileLds& L, const TileOffLoads& tol, const unsigned long long* pre = nullptr) {
    constexpr bool kClassify = kKind == 1;
    constexpr uint32_t kWinVec = kStage / 16 / kWave;
    const emurx_dev_tables& T = a.T;
    const emurx_route_args& rt = a.rt;
    const uint32_t n = a.n;
    // outcome histogram per wave, {pkts << 23 | bytes}: <= 64 x 65535 B.  It shares the rows
    // of csum (a wave's span sums are done before its histogram is zeroed): 1 KiB less keeps
    // the narrow slab at 6 workgroups per CU (LDS 26 KiB)
    static_assert(EMURX_HIST_BINS == kWave, "one histogram bin per lane");
    uint32_t (*s_hist)[EMURX_HIST_BINS] = L.csum;

    const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid / kWave;
#if EMURX_STAMP
    // entry, descriptors, staging landed: taken by the caller
    unsigned long long st_[10] = {pre ? pre[0] : 0, pre ? pre[1] : 0, pre ? pre[2] : 0, 0, 0, 0, 0, 0, 0, 0};
#endif
    const uint32_t i = tile * EMURX_QUEUE_TILE + tid;
    if (lane < 16) L.wcnt[wv][lane] = 0;
    if (lane < EMURX_MAX_PARTS) L.rcnt[wv][lane] = 0;
    // kind 2: the tile's offset in every owner region, from the loads issued before the staging
    // wait (k_rx): in flight beside the tile's LDS-DMA instead of one more round trip here
    if (kKind == 2 && wv == 0) {
        const TileOffLoads t = EMURX_TOL_PREFETCH ? tol : tile_offsets_issue(rt.cnt, rt.goff, rt.parts, tile, lane);
        tile_offsets_sum(t, rt.parts, lane, L.toff, [](uint32_t v) { return wave_sum_u32(v); });
    }
    const bool valid = (dd.y >> 24) != EMURX_DESC_HOLE;
    const uint32_t off = dd.x, len = dd.y & 0xffff, vport = (dd.y >> 16) & 0xff;
    // stage-size feedback from every 64th tile (the launcher's choice, emurx_api.cpp): one
    // word per wave {gen, the wave has frames, its range fits the wide slab only}
    if (a.fb && (tile & 63) == 0 && lane == 0) {
        const uint32_t bytes = sg.nvec * 16;
        const uint32_t mid = bytes > kStageNarrow && bytes <= kStageWide;
        a.fb[((tile >> 6) & 63) * kWaves + wv] = (a.gen << 2) | ((sg.nvec > 0) << 1) | mid;
    }

    Rec r;
    r.dlen = 0;
    // kKind 2: the frame's lookup record (emurx_parse.h pack_lookup), parked in the wave's slab
    // from the end of the parse: the 32-byte heads (2 KiB) until the owner offsets are known
    // after the tile barrier, the tails (up to 48 B per lane, the next 3 KiB) until the wave has
    // taken their units: no registers held across either
    uint4* const wslab = reinterpret_cast<uint4*>(const_cast<uint32_t*>(slab)) + wv * (kStage / 16);
    uint4* lhead = wslab + lane * 2;
    uint4* ltail = wslab + kWave * 2 + lane * 3;
    static_assert(kStage >= kWave * (32 + 48), "a wave's lookup heads and tails fit its slab");
    uint32_t tun = 0;  // kKind 2: the frame's tail units (0, 1 or 3)
    if (sg.staged) {  // wave-uniform branch
        if (valid) {
            LdsSrc s{reinterpret_cast<const uint8_t*>(slab), slab, wv * kStage + (off - sg.start)};
            parse_flat(s, len, vport, T.cb_mask, r);
            STAMP(3);
            if (kClassify) classify(s, len, T, r);
            if (kKind == 2) tun = pack_lookup(s, len, r, i, r.status == EMURX_ST_OK, rt.tup_on, lhead, ltail);
        }
    } else {
        const uint32_t head = (uint32_t)((uintptr_t)(a.frames + off) & 15);
        WinSrc s{reinterpret_cast<const uint8_t*>(slab), slab, wv * kStage + lane * 16, head,
                 min(kWinVec * 16 - head, len), a.frames + off};
        if (valid) parse_packet(s, len, vport, T.cb_mask, r);
        coop_checksum_rows(r, a.frames + off, L.csum[wv]);  // the wave's long L4 spans, converged
        STAMP(3);
        if (valid && kClassify) classify(s, len, T, r);
        if (kKind == 2 && valid) tun = pack_lookup(s, len, r, i, r.status == EMURX_ST_OK, rt.tup_on, lhead, ltail);
    }
    STAMP(4);
    // kind 2: the frame's owner, its rank among the wave's frames of that owner, and its tail's
    // units: per (wave, owner) one atomic on the owner's cursor of this tile's shard (a line
    // each) takes the units of the wave's tails (tails of 1 and 3 units ranked by two ballots).
    // Issued here, consumed after the tile barrier (store_tails): the histogram, the queue ranks
    // and the barrier hide the atomic's round trip
    uint32_t rd = 0xffu, rrank = 0, tofs = 0, tlead = 0, tb = 0;
    const uint32_t shard = tile & (EMURX_TAIL_SHARDS - 1);
    if constexpr (kKind == 2) {
        const uint32_t pad = dd.y >> 24;
        // the owner the count pass used (a keyed descriptor's key, the same digest of the
        // CTunnelKey the parse left: packing and counts agree by construction)
        rd = !valid ? 0xffu
             : (pad & EMURX_DESC_KEYED) ? emurx_owner_of_key(pad, rt.parts)
                                        : emurx_owner(emurx_tk_hash(r.vport, r.vlan0, r.vlan1), rt.parts);
        uint64_t rl = __ballot(rd != 0xffu);
        while (rl) {
            const uint32_t lead = (uint32_t)__ffsll((long long)rl) - 1;
            const uint32_t d2 = (uint32_t)__builtin_amdgcn_readlane((int)rd, (int)lead);
            const uint64_t m = __ballot(rd == d2);
            const uint64_t m1 = __ballot(rd == d2 && tun == 1), m3 = __ballot(rd == d2 && tun == 3);
            if (rd == d2) {
                rrank = mbcnt(m);
                tofs = mbcnt(m1) + 3 * mbcnt(m3);
            }
            if (lane == lead) L.rcnt[wv][d2] = (uint32_t)__popcll(m);
            if (m1 | m3) {  // wave-uniform
                const uint32_t tl = (uint32_t)__ffsll((long long)(m1 | m3)) - 1;
                if (lane == tl)
                    tb = atomicAdd(&rt.tcur[(d2 * EMURX_TAIL_SHARDS + shard) * EMURX_TAIL_CURSOR_STRIDE],
                                   (uint32_t)(__popcll(m1) + 3 * __popcll(m3)));
                if (rd == d2) tlead = tl;
            }
            rl &= ~m;
        }
    }
    // each lane stores its tail at the units its wave took and writes their index into its
    // parked head (kind 2)
    auto store_tails = [&]() {
        if (!__ballot(tun != 0)) return;
        const uint32_t at = (uint32_t)__shfl((int)tb, (int)tlead) + tofs;
        if (tun) {
            uint32_t idx = EMURX_TAIL_NONE;
            if (at + tun <= rt.tcap) {
                idx = shard * rt.tcap + at;
                uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(rt.send) +
                                                      (uint64_t)rd * (rt.cap + 32ull * rt.tcap) * 32 +
                                                      (uint64_t)rt.cap * 32) + idx;
                dst[0] = ltail[0];
                if (tun == 3) {
                    dst[1] = ltail[1];
                    dst[2] = ltail[2];
                }
            } else {
                atomicMax(&rt.count[2 * rd + 1], at + tun);  // the shard overflowed: the caller regrows
            }
            reinterpret_cast<uint32_t*>(lhead)[7] = idx;
        }
    };
    // outcome histogram into the wave's LDS copy: a wave whose frames all share one
    // (status, proto) bin adds its count (ballot) and byte sum (DPP reduction) once, instead
    // of 64 LDS atomics serialised on one address; mixed waves add per frame
    s_hist[wv][lane] = 0;  // each wave owns its copy: no cross-wave ordering needed
    {
        const uint32_t bin = valid ? EMURX_HIST_BIN(r.status, r.proto) : 0xffu;
        const uint64_t vm = __ballot(valid);
        if (vm) {
            const uint32_t lead = (uint32_t)__ffsll((long long)vm) - 1;
            const uint32_t bb = (uint32_t)__builtin_amdgcn_readlane((int)bin, (int)lead);
            if (__ballot(bin == bb) == vm) {
                const uint32_t bytes = wave_sum_u32(valid ? len : 0u);  // <= 64 x 65535
                if (lane == lead) s_hist[wv][bb] += ((uint32_t)__popcll(vm) << 23) | bytes;
            } else if (valid) {
                atomicAdd(&s_hist[wv][bin], (1u << 23) | len);
            }
        }
    }
    const uint32_t q = valid ? (r.status == EMURX_ST_OK ? r.proto : EMURX_Q_DROP) : 0xffu;
    // rank inside (wave, queue): one ballot per distinct queue present in the wave
    uint32_t rank = 0;
#if EMURX_MATCHRANK
    if (EMURX_MATCHRANK == 2 && __ballot(valid && q != (uint32_t)__builtin_amdgcn_readfirstlane((int)q)) == 0) {
        // hybrid: one queue in the wave (or none)
        const uint64_t vm = __ballot(valid);
        rank = mbcnt(vm);
        if (valid && rank == 0) L.wcnt[wv][q] = (uint32_t)__popcll(vm);
    } else {
        const uint64_t m = match_lanes<4>(q, __ballot(valid));
        rank = mbcnt(m);
        if (valid && rank == 0) L.wcnt[wv][q] = (uint32_t)__popcll(m);
    }
#else
    uint64_t left = __ballot(valid);
    while (left) {
        const uint32_t lead = (uint32_t)__ffsll((long long)left) - 1;
        const uint32_t qq = (uint32_t)__builtin_amdgcn_readlane((int)q, (int)lead);
        const uint64_t m = __ballot(q == qq);
        if (q == qq) rank = mbcnt(m);
        if (lane == lead) L.wcnt[wv][qq] = (uint32_t)__popcll(m);
        left &= ~m;
    }
#endif
    STAMP(5);
    STAMP(6);
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    bool tails_out = false;
    if (kKind == 2 && a.rec) {  // the records' park below reuses the tails' LDS rows
        store_tails();
        tails_out = true;
    }
    if (a.rec) {
        // The wave's 64 records (32 B each) go out as two contiguous 1 KiB stores: every lane
        // parks its record in the wave's slab (free once the parse, the lookups and the lookup
        // record are done with the frame bytes; kind 2's lookup records hold its first 4 KiB),
        // then stores 16 B of the transposed block.  Whole lines per store instruction instead
        // of 16 of every 32 bytes (measured against two strided stores per lane on 8 rotating
        // batches: config B +3 %, C +0.5 %, E +1 %; non-temporal beats plain stores either way).
        // An empty descriptor slot gets a record too (no Namespace, status EMURX_ST_HOLE), so
        // every consumer of rec[0, n) sees defined bytes.
        constexpr uint32_t kPark = kKind == 2 ? 2u * kWave : 0u;  // in 16-B units: after the heads (the tails are stored)
        static_assert(kPark * 16 + kWave * 32 <= kStage, "the parked records fit the slab");
        uint4* park = reinterpret_cast<uint4*>(const_cast<uint32_t*>(slab)) + wv * (kStage / 16) + kPark;
        park[2 * lane] = valid ? make_uint4(r.ns, r.cl, r.vlan0, r.vlan1)
                               : make_uint4(EMURX_ID_NONE, EMURX_ID_NONE, 0, 0);
        park[2 * lane + 1] = valid ? make_uint4(r.vport | (r.l3 << 16), r.l4 | (r.l7 << 16),
                                                r.l7len | (r.nh << 16) | (r.proto << 24), r.status | (r.flags << 8))
                                   : make_uint4(0, 0, (uint32_t)EMURX_CB_NONE << 24, EMURX_ST_HOLE);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t r0 = tile * EMURX_QUEUE_TILE + wv * kWave;  // the wave's first record
        uint4* o = reinterpret_cast<uint4*>(a.rec + r0);
        const uint4 x0 = park[lane], x1 = park[kWave + lane];
        // streaming stores: the records are read once, by the host copy or the route kernel
        if (r0 + lane / 2 < n) __builtin_nontemporal_store(v4u{x0.x, x0.y, x0.z, x0.w}, reinterpret_cast<v4u*>(o + lane));
        if (r0 + kWave / 2 + lane / 2 < n)
            __builtin_nontemporal_store(v4u{x1.x, x1.y, x1.z, x1.w}, reinterpret_cast<v4u*>(o + kWave + lane));
    }
    if (a.flow && i < n) a.flow[i] = valid ? r.flow : EMURX_FLOW_NONE;
    // the Namespace owner of the record (classify + route: the records whose Namespace was
    // found), counted per (tile, owner): the first pass of emurx_route_dev, fused (k_route<false>
    // counts them the same way, emurx_route.hip); kind 2 ranked its owners above
    if (kKind == 1 && rt.cnt) {
        const bool routed = valid && r.ns != EMURX_ID_NONE;
        rd = !routed ? 0xffu : emurx_owner(emurx_tk_hash(r.vport, r.vlan0, r.vlan1), rt.parts);
#if EMURX_MATCHRANK
        const uint64_t m = match_lanes<3>(rd, __ballot(rd != 0xffu));
        rrank = mbcnt(m);
        if (rd != 0xffu && rrank == 0) L.rcnt[wv][rd] = (uint32_t)__popcll(m);
#else
        uint64_t rl = __ballot(rd != 0xffu);
        while (rl) {
            const uint32_t lead = (uint32_t)__ffsll((long long)rl) - 1;
            const uint32_t dd2 = (uint32_t)__builtin_amdgcn_readlane((int)rd, (int)lead);
            const uint64_t m = __ballot(rd == dd2);
            if (rd == dd2) rrank = mbcnt(m);
            if (lane == lead) L.rcnt[wv][dd2] = (uint32_t)__popcll(m);
            rl &= ~m;
        }
#endif
    }
    STAMP(7);
    __syncthreads();
    STAMP(8);
    if (kKind == 1 && rt.cnt && tid < 16) {
        const uint32_t c = tid < rt.parts ? L.rcnt[0][tid] + L.rcnt[1][tid] + L.rcnt[2][tid] + L.rcnt[3][tid] : 0u;
        rt.cnt[(size_t)tile * 16 + tid] = c;
        if (c) atomicAdd(&rt.grp[(tile / 64) * 16 + tid], c);
    }
    if constexpr (kKind == 2) {  // every frame's 32-byte lookup head into its owner's region
        if (!tails_out) {
            store_tails();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the patched heads, read by other lanes
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        // the head's slot in send, in 32-byte units (regions of cap + 32 tcap of them: the
        // launcher checks that the whole buffer's units fit 32 bits); none on overflow
        uint32_t dst = 0xffffffffu;
        if (rd != 0xffu) {
            uint32_t pos = L.toff[rd] + rrank;
            for (uint32_t w = 0; w < wv; ++w) pos += L.rcnt[w][rd];
            if (pos < rt.cap) dst = rd * (rt.cap + 32u * rt.tcap) + pos;  // overflow: send_count[2 d] > cap
        }
        // two lanes per head, 32 heads per store instruction: heads of one owner ranked next to
        // each other (every one of them at N = 1) make contiguous 1 KiB stores
        const uint4* parked = wslab;
#pragma unroll
        for (uint32_t k = 0; k < 2; ++k) {
            const uint32_t rr = k * (kWave / 2) + lane / 2, part = lane & 1;
            const uint32_t to = (uint32_t)__shfl((int)dst, (int)rr);
            if (to != 0xffffffffu) reinterpret_cast<uint4*>(rt.send + to)[part] = parked[rr * 2 + part];
        }
    }

    // this tile's segment of every queue: frames in (wave, lane) order == frame order
    if (a.qlist && q < EMURX_NUM_QUEUES) {
        uint32_t pos = rank;
        for (uint32_t w = 0; w < wv; ++w) pos += L.wcnt[w][q];
        const size_t at = (size_t)q * a.qcap + (size_t)tile * EMURX_QUEUE_TILE + pos;
        if ((size_t)tile * EMURX_QUEUE_TILE + pos < a.qcap) a.qlist[at] = i;
    }
    if (a.tile_cnt && tid < 16)
        a.tile_cnt[(size_t)tile * 16 + tid] = L.wcnt[0][tid] + L.wcnt[1][tid] + L.wcnt[2][tid] + L.wcnt[3][tid];
    // one of EMURX_HIST_SHARDS copies per workgroup: same-address memory-side atomics from
    // every workgroup would serialise; the shards are folded on the host
    if (tid >= 64 && tid < 64 + EMURX_HIST_BINS) {
        const uint32_t b = tid - 64;
        uint32_t pk = 0, by = 0;
#pragma unroll
        for (uint32_t w = 0; w < kWaves; ++w) {
            pk += s_hist[w][b] >> 23;
            by += s_hist[w][b] & ((1u << 23) - 1);
        }
        if (pk) {
            unsigned long long* hs = a.hist + (size_t)(tile & (EMURX_HIST_SHARDS - 1)) * 2 * EMURX_HIST_BINS;
            atomicAdd(&hs[2 * b], (unsigned long long)pk);
            atomicAdd(&hs[2 * b + 1], (unsigned long long)by);
        }
    }
#if EMURX_STAMP
    STAMP(9);
    if (g_stamp && lane == 0) {
        unsigned long long* o = g_stamp + ((size_t)tile * kWaves + wv) * 16;
        for (int k = 0; k < 10; ++k) o[k] = st_[k];
        o[10] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
        o[11] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
        o[12] = tile;
    }
#endif
}

// One tile per workgroup: stage, wait, process
template <int kKind, uint32_t kStage>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kStage == kStageNarrow ? 6 : 5))) void k_rx(const RxArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t slab[kWaves * kStage / 4];
    __shared__ TileLds L;
    const uint32_t tile = blockIdx.x, wv = threadIdx.x / kWave;
#if EMURX_STAMP
    unsigned long long pre[3];
    pre[0] = __builtin_amdgcn_s_memtime();
#endif
    const uint2 dd = load_desc(a.desc, a.n, tile * EMURX_QUEUE_TILE + threadIdx.x);
    TileOffLoads tol{make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), 0u};
    if (EMURX_TOL_PREFETCH && kKind == 2 && wv == 0) tol = tile_offsets_issue(a.rt.cnt, a.rt.goff, a.rt.parts, tile, lane_id());
#if EMURX_STAMP
    wait_vm0();
    pre[1] = __builtin_amdgcn_s_memtime();
#endif
    const Stage sg = stage_issue<kStage>(a.frames, dd, lane_id(), reinterpret_cast<uint4*>(slab) + wv * (kStage / 16));
    stage_wait();
#if EMURX_STAMP
    pre[2] = __builtin_amdgcn_s_memtime();
    tile_body<kKind, kStage>(a, tile, dd, sg, slab, L, tol, pre);
#else
    tile_body<kKind, kStage>(a, tile, dd, sg, slab, L, tol);
#endif
}

// table deltas (emurx_api.cpp ship_tables): 4 lanes per 64-byte block, 16 bytes each
__global__ __launch_bounds__(kBlock) void k_apply(const emurx_delta* __restrict__ d, uint32_t n) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x, e = i >> 2, q = i & 3;
    if (e >= n) return;
    const uint4 v = reinterpret_cast<const uint4*>(d[e].w)[q];
    reinterpret_cast<uint4*>((uintptr_t)d[e].dst)[q] = v;
}

}  // namespace emurx

int emurx_launch_apply(const emurx_delta* d, uint32_t n, hipStream_t st) {
    using namespace emurx;
    if (!n) return 0;
    return EMURX_HIP_OK(emurx_launch(k_apply, dim3((n * 4 + kBlock - 1) / kBlock), dim3(kBlock), 0, st, d, n)) ? 0 : -1;
}

// ---------------------------------------------------------------------------------------
// launcher (called by emurx_api.cpp)
// ---------------------------------------------------------------------------------------
int emurx_launch_batch(const uint8_t* frames, const emurx_desc* desc, uint32_t n,
                       const emurx_dev_tables& T, int kind, const emurx_dev_out& out,
                       hipStream_t st, const hipEvent_t* ev, bool narrow, uint32_t* fb, uint32_t gen,
                       const emurx_route_args* rt) {
    using namespace emurx;
    hipError_t e = hipSuccess;
#ifndef EMURX_RX_LDS_PAD  // measurement builds only: unused LDS per workgroup, to cap k_rx's occupancy
#define EMURX_RX_LDS_PAD 0
#endif
    if (ev && !EMURX_HIP_OK(hipEventRecord(ev[0], st))) return -1;
    if (n) {
        const uint32_t ntiles = (n + EMURX_QUEUE_TILE - 1) / EMURX_QUEUE_TILE;
        unsigned long long* hist = reinterpret_cast<unsigned long long*>(out.hist);
        const emurx_route_args none{};
        const RxArgs args{frames, desc, n, T, out.rec, out.qlist, out.qcap, out.tile_cnt, hist, out.flow, fb, gen,
                          rt ? *rt : none};
        auto k = kind == 1 ? (narrow ? k_rx<1, kStageNarrow> : k_rx<1, kStageWide>)
               : kind == 2 ? (narrow ? k_rx<2, kStageNarrow> : k_rx<2, kStageWide>)
                           : (narrow ? k_rx<0, kStageNarrow> : k_rx<0, kStageWide>);
        e = emurx_launch(k, dim3(ntiles), dim3(kBlock), EMURX_RX_LDS_PAD, st, args);
    }
    if (!EMURX_HIP_OK(e)) return -1;
    return ev && !EMURX_HIP_OK(hipEventRecord(ev[1], st)) ? -1 : 0;
}

namespace emurx {
// streaming copy for the measured HBM ceiling (emurx_copy_ceiling_dev): 4 independent 16-byte
// loads per lane in flight, non-temporal both ways, grid-stride over 16,384 workgroups (the
// fastest of the variants tools/copy_probe.hip times: 6.13 TB/s read + write on a 1 GiB copy,
// against 5.74 for 8 in flight over 2,048 workgroups)
constexpr int kCopyInFlight = 4;
constexpr int kCopyGrid = 16384;
__global__ __launch_bounds__(kBlock) void k_copy(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t nv) {
    typedef unsigned v4 __attribute__((ext_vector_type(4)));
    const size_t stride = (size_t)gridDim.x * kBlock * kCopyInFlight;
    for (size_t base = (size_t)blockIdx.x * kBlock * kCopyInFlight + threadIdx.x; base < nv; base += stride) {
        v4 x[kCopyInFlight];
#pragma unroll
        for (int k = 0; k < kCopyInFlight; ++k) {
            const size_t i = base + (size_t)k * kBlock;
            x[k] = i < nv ? __builtin_nontemporal_load(reinterpret_cast<const v4*>(src) + i) : v4{0, 0, 0, 0};
        }
#pragma unroll
        for (int k = 0; k < kCopyInFlight; ++k) {
            const size_t i = base + (size_t)k * kBlock;
            if (i < nv) __builtin_nontemporal_store(x[k], reinterpret_cast<v4*>(dst) + i);
        }
    }
}
}  // namespace emurx

#if EMURX_STAMP
// the stamp buffer of the timeline variant (tools/stamps.py): 16 u64 per wave of the launch
extern "C" int emurx_debug_set_stamps(void* dev_buf) {
    return EMURX_HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(emurx::g_stamp), &dev_buf, sizeof(dev_buf))) ? 0 : -1;
}
#endif

extern "C" int emurx_copy_ceiling_dev(void* d_dst, const void* d_src, size_t bytes, void* stream) {
    if (!d_dst || !d_src || (bytes & 15) || ((uintptr_t)d_dst & 15) || ((uintptr_t)d_src & 15)) return EMURX_EINVAL;
    if (!bytes) return EMURX_OK;
    return EMURX_HIP_OK(emurx_launch(emurx::k_copy, dim3(emurx::kCopyGrid), dim3(emurx::kBlock), 0, (hipStream_t)stream,
                                     reinterpret_cast<uint4*>(d_dst), reinterpret_cast<const uint4*>(d_src), bytes / 16))
               ? EMURX_OK
               : EMURX_EDEVICE;
}
