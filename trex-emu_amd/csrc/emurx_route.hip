// emurx_route.hip — Namespace-partitioned exchange, device side (gfx950).
//
// After k_rx has classified a batch, every record whose Namespace was found is sent to the
// GPU that owns that Namespace (emurx_owner of its CTunnelKey hash).  Three
// launches build the all-to-all send buffer in frame order per destination:
//   k_route<false>  per tile of 256 records: destination of each record, counts per
//                   (tile, destination) -> tile_cnt, and per group of 64 tiles -> grp (one
//                   atomic per tile and destination, 64 tiles per address)
//   k_route_scan    one workgroup, one lane per group: exclusive prefix over groups ->
//                   grp_off, totals -> send_count; clears grp for the next batch
//   k_route<true>   tile offset = grp_off + the counts of the group's earlier tiles (one
//                   coalesced load + wave reductions), ranks by wave ballots (no atomics)
//                   -> send[d * cap + offset]
// The exchange itself (an equal-split all-to-all over RCCL) is issued by the caller on the
// same stream.  Bytes: 32 B read twice + 40 B written per routed record.
#include <hip/hip_runtime.h>

#include "../../include/emu_rx.h"
#include "emurx_kernels.h"
#include "emurx_parse.h"
#include "emurx_tables.h"

namespace emurx {

constexpr uint32_t kScanThreads = 1024;  // groups per batch (64 tiles each): 16M frames
constexpr uint32_t kGroup = 64;          // tiles per group

template <bool kPack>
__global__ __launch_bounds__(kBlock) void k_route(const emurx_rec* __restrict__ rec, uint32_t n,
                                                  uint32_t n_parts, uint32_t my_rank,
                                                  uint32_t* __restrict__ tile_cnt, uint32_t* __restrict__ grp,
                                                  const uint32_t* __restrict__ grp_off,
                                                  emurx_route_rec* __restrict__ send, uint32_t cap) {
    __shared__ uint32_t s_wcnt[kWaves][16];
    __shared__ uint32_t s_toff[EMURX_MAX_PARTS];
    __shared__ uint2 s_park[kPack ? kWaves : 1][kPack ? kWave * 5 : 1];  // the wave's records, 40 B each
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
    if (kPack && wv == 0)  // this tile's offset: group offset + the group's earlier tiles
        tile_offsets(tile_cnt, grp_off, n_parts, tile, lane, s_toff, [](uint32_t v) { return wave_sum_u32(v); });
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
        if (tid < 16) {
            const uint32_t c = s_wcnt[0][tid] + s_wcnt[1][tid] + s_wcnt[2][tid] + s_wcnt[3][tid];
            tile_cnt[tile * 16 + tid] = c;
            if (c) atomicAdd(&grp[(tile / kGroup) * 16 + tid], c);
        }
        return;
    }
    uint32_t dst = 0xffffffffu;  // the record's slot in send (record units), none on overflow
    if (d != 0xffu) {
        uint32_t pos = s_toff[d] + rank;
        for (uint32_t w = 0; w < wv; ++w) pos += s_wcnt[w][d];
        if (pos < cap) dst = d * cap + pos;  // overflow: send_count[d] > cap tells the caller
    }
    // The wave's 40-B records go out through LDS as five 8-B pieces per record, spread over the
    // lanes (lane l of store k writes piece (64k + l) mod 5 of record (64k + l) / 5): records of
    // one owner ranked next to each other make contiguous 512-B stores, instead of each lane
    // writing five 8-B pieces 40 B apart
    uint2* park = s_park[wv];
    park[lane * 5 + 0] = make_uint2(a.x, a.y);
    park[lane * 5 + 1] = make_uint2(a.z, a.w);
    park[lane * 5 + 2] = make_uint2(b.x, b.y);
    park[lane * 5 + 3] = make_uint2(b.z, b.w);
    park[lane * 5 + 4] = make_uint2(i, my_rank);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (uint32_t k = 0; k < 5; ++k) {
        const uint32_t p = k * kWave + lane, rr = p / 5, part = p - rr * 5;
        const uint32_t to = (uint32_t)__shfl((int)dst, (int)rr);
        if (to != 0xffffffffu) reinterpret_cast<uint2*>(send + to)[part] = park[p];
    }
}

// exclusive prefix over groups of grp[g][d], d < n_parts; one lane per group; leaves grp zero.
// send_count[cstride * d] = the total of d (cstride 2: the partitioned source's {heads, tail
// overflow} pairs, the second word zeroed, and its tail cursors tcur cleared for k_rx kind 2)
__global__ __launch_bounds__(kScanThreads) void k_route_scan(uint32_t* __restrict__ grp, uint32_t ngroups,
                                                              uint32_t n_parts, uint32_t* __restrict__ grp_off,
                                                              uint32_t* __restrict__ send_count, uint32_t* __restrict__ tcur,
                                                              uint32_t cstride) {
    static_assert(EMURX_MAX_PARTS * EMURX_TAIL_SHARDS <= kScanThreads, "one cursor per lane");
    __shared__ uint32_t s_wsum[EMURX_MAX_PARTS][kScanThreads / kWave];
    __shared__ uint32_t s_ex[EMURX_MAX_PARTS][kScanThreads];
    const uint32_t t = threadIdx.x, lane = lane_id(), wv = t / kWave;
    if (tcur && t < n_parts * EMURX_TAIL_SHARDS) tcur[t * EMURX_TAIL_CURSOR_STRIDE] = 0;
    uint4 x = make_uint4(0, 0, 0, 0), y = x;
    if (t < ngroups) {
        uint4* p = reinterpret_cast<uint4*>(grp + t * 16);
        x = p[0];
        y = p[1];
        p[0] = make_uint4(0, 0, 0, 0);
        p[1] = make_uint4(0, 0, 0, 0);
    }
    for (uint32_t k = 0; k < n_parts; ++k) {  // inclusive wave scan per destination
        const uint32_t v = k == 0 ? x.x : k == 1 ? x.y : k == 2 ? x.z : k == 3 ? x.w
                         : k == 4 ? y.x : k == 5 ? y.y : k == 6 ? y.z : y.w;
        uint32_t incl = v;
#pragma unroll
        for (uint32_t o = 1; o < kWave; o <<= 1) {
            const uint32_t up = (uint32_t)__shfl_up((int)incl, o);
            if (lane >= o) incl += up;
        }
        if (lane == kWave - 1) s_wsum[k][wv] = incl;
        s_ex[k][t] = incl - v;
    }
    __syncthreads();
    for (uint32_t k = 0; k < n_parts; ++k) {
        uint32_t before = 0, total = 0;
        for (uint32_t w = 0; w < kScanThreads / kWave; ++w) {
            const uint32_t sw = s_wsum[k][w];
            before += w < wv ? sw : 0;
            total += sw;
        }
        if (t < ngroups) grp_off[t * 16 + k] = before + s_ex[k][t];
        if (t == 0) send_count[cstride * k] = total;
        if (t == 0 && cstride == 2) send_count[2 * k + 1] = 0;
    }
}

// ---- partitioned path -------------------------------------------------------------------
// k_owner_count: the owner of every frame, counted per (tile, owner) and per group of 64
// tiles, as k_route<false> counts records; k_rx kind 2 then packs at the offsets
// k_route_scan derives.  A keyed descriptor (EMURX_DESC_KEYED, written by the device framing
// walk or k_desc_keys) gives the owner by itself: a wave of keyed descriptors reads 512 bytes.
// For the other frames the owner comes from the L2 header (l2_vlans: bytes 12..19 + the
// length): a wave whose unkeyed frames' byte range fits kOcStage bytes copies that range into
// LDS with coalesced LDS-DMA (as k_rx stages) and reads each frame's bytes 12..19 there (a
// per-lane gather of one line per frame ran at the random-line rate); wider waves gather.
// 2 KiB per wave: 8 workgroups per CU (the wave limit) instead of 6 with 6 KiB. Keyed
// descriptors (the production path: the device framing walk keys them) read no frame byte, and
// the kernel falls 10.7 -> 8.0 us per 2M frames; unkeyed waves wider than 2 KiB gather instead
// (config D unkeyed: 39.2 -> 46.6 us; DESIGN.md §6 round 4, profiles/r04/ab_owner_count/)
#ifndef EMURX_OC_STAGE
#define EMURX_OC_STAGE 2048
#endif
// Tiles per workgroup: every tile's descriptors are loaded at the top (EMURX_OC_TPW loads in
// flight per lane), the tiles then counted one after the other, and the workgroup's counts
// added to its group once (its tiles share one group of 64)
#ifndef EMURX_OC_TPW
#define EMURX_OC_TPW 1
#endif
constexpr uint32_t kOcStage = EMURX_OC_STAGE;
constexpr uint32_t kOcTpw = EMURX_OC_TPW;
static_assert(kOcTpw >= 1 && kGroup % kOcTpw == 0, "a workgroup's tiles in one group");
__global__ __launch_bounds__(kBlock) void k_owner_count(const uint8_t* __restrict__ frames,
                                                        const emurx_desc* __restrict__ desc, uint32_t n,
                                                        uint32_t n_parts, uint32_t* __restrict__ tile_cnt,
                                                        uint32_t* __restrict__ grp) {
    __shared__ uint32_t s_wcnt[kWaves][16];
    // the wave's staged bytes + 32 bytes of slack for the aligned dword reads past its end
    __shared__ __attribute__((aligned(16))) uint32_t s_stage[kWaves][(kOcStage + 32) / 4];
    const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid / kWave, t0 = blockIdx.x * kOcTpw;
    const uint32_t ntiles = (n + kBlock - 1) / kBlock, tn = min(kOcTpw, ntiles - t0);
    uint2 dds[kOcTpw];
#pragma unroll
    for (uint32_t k = 0; k < kOcTpw; ++k) {
        const uint32_t i = (t0 + k) * kBlock + tid;
        dds[k] = k < tn && i < n ? *reinterpret_cast<const uint2*>(desc + i) : make_uint2(0, EMURX_DESC_HOLE << 24);
    }
    uint32_t gacc = 0;  // tid < 16: the workgroup's frames of owner tid
#pragma unroll
    for (uint32_t k = 0; k < kOcTpw; ++k) {
        if (k >= tn) break;
        const uint32_t tile = t0 + k;
        if (lane < 16) s_wcnt[wv][lane] = 0;
        const uint2 dd = dds[k];
        const uint32_t pad = dd.y >> 24;
        const bool valid = pad != EMURX_DESC_HOLE, keyed = valid && (pad & EMURX_DESC_KEYED);
        const bool need = valid && !keyed;  // the owner must come from the frame's bytes
        const uint32_t off = dd.x, len = dd.y & 0xffff;
        uint32_t start = 0, nvec = 0;
        if (__ballot(need)) {  // wave-uniform: a wave of keyed descriptors reads no frame byte
            const uint32_t lo = wave_min_u32(need ? off : 0xffffffffu);
            const uint32_t hi = wave_max_u32(need ? off + len : 0u);
            start = lo & ~15u;
            nvec = hi > lo ? (hi - start + 15) >> 4 : 0;
        }
        const bool staged = nvec > 0 && nvec <= kOcStage / 16;  // wave-uniform
        if (staged) {
            static_assert(kOcStage % (16 * kWave) == 0, "whole 1 KiB DMA rows");
            const uint4* src = reinterpret_cast<const uint4*>(frames + start);
            uint4* dst = reinterpret_cast<uint4*>(s_stage[wv]);
#pragma unroll
            for (uint32_t j = 0; j < kOcStage / 16 / kWave; ++j)
                if (j * kWave < nvec)
                    __builtin_amdgcn_global_load_lds(src + min(lane + j * kWave, nvec - 1),
                                                     (__attribute__((address_space(3))) void*)(dst + j * kWave), 16, 0, 2);
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the wave's DMA landed
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        uint32_t d = keyed ? emurx_owner_of_key(pad, n_parts) : 0xffu;
        if (need) {
            const uint32_t vport = (dd.y >> 16) & 0xff;
            uint32_t w0 = 0, w1 = 0, w2 = 0, sh;
            if (staged) {
                // bytes past the frame are the next frame's or stale: l2_vlans reads a word only
                // where len says its bytes exist
                const uint32_t rel = off - start + 12;
                sh = rel & 3;
                const uint32_t* q = s_stage[wv] + (rel >> 2);
                w0 = q[0]; w1 = q[1]; w2 = q[2];
            } else {
                // bytes 12..19 from the three aligned dwords around them, each loaded only when it
                // holds a byte of the frame (an aligned dword never crosses the 64-byte boundary the
                // buffer contract guarantees past the last byte, emu_rx.h): one 12-byte load for every
                // frame of 21 bytes or more; l2_vlans reads a word only where len says its bytes exist
                const uintptr_t a = (uintptr_t)(frames + off + 12);
                sh = (uint32_t)(a & 3);
                const uint32_t lim = len + sh;  // dword k holds a frame byte iff 12 + 4k < lim
                const void* wa = reinterpret_cast<const void*>(a & ~(uintptr_t)3);
                if (lim > 20) {
                    const uint3 w3 = gld12(wa);  // one 12-byte load
                    w0 = w3.x; w1 = w3.y; w2 = w3.z;
                } else {
                    if (lim > 12) w0 = gld4(wa);
                    if (lim > 16) w1 = gld4(reinterpret_cast<const uint8_t*>(wa) + 4);
                }
            }
            const uint32_t b12 = __builtin_bswap32(__builtin_amdgcn_alignbyte(w1, w0, sh));
            const uint32_t b16 = __builtin_bswap32(__builtin_amdgcn_alignbyte(w2, w1, sh));
            uint32_t v0, v1;
            l2_vlans(len, b12, b16, v0, v1);
            d = emurx_owner(emurx_tk_hash(vport, v0, v1), n_parts);
        }
        uint64_t left = __ballot(d != 0xffu);
        while (left) {
            const uint32_t lead = (uint32_t)__ffsll((long long)left) - 1;
            const uint32_t q = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)lead);
            const uint64_t m = __ballot(d == q);
            if (lane == lead) s_wcnt[wv][q] = (uint32_t)__popcll(m);
            left &= ~m;
        }
        __syncthreads();
        if (tid < 16) {
            const uint32_t c = s_wcnt[0][tid] + s_wcnt[1][tid] + s_wcnt[2][tid] + s_wcnt[3][tid];
            tile_cnt[tile * 16 + tid] = c;
            gacc += c;
        }
        if (kOcTpw > 1) __syncthreads();  // s_wcnt and the slabs are reused by the next tile
    }
    if (tid < 16 && gacc) atomicAdd(&grp[(t0 / kGroup) * 16 + tid], gacc);
}

// k_desc_keys: the owner key of every frame into its descriptor's pad byte (what the device
// framing walk writes, for descriptors built without it): one lane per descriptor, bytes
// 12..19 of the frame by the three aligned dwords around them (each loaded only where it
// holds a frame byte, as k_owner_count's gather).  Holes stay holes.
__global__ __launch_bounds__(kBlock) void k_desc_keys(const uint8_t* __restrict__ frames, emurx_desc* __restrict__ desc,
                                                      uint32_t n) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    uint2 dd = *reinterpret_cast<const uint2*>(desc + i);
    if ((dd.y >> 24) == EMURX_DESC_HOLE) return;
    const uint32_t off = dd.x, len = dd.y & 0xffff, vport = (dd.y >> 16) & 0xff;
    const uintptr_t a = (uintptr_t)(frames + off + 12);
    const uint32_t sh = (uint32_t)(a & 3), lim = len + sh;  // dword k holds a frame byte iff 12 + 4k < lim
    const uint8_t* wa = reinterpret_cast<const uint8_t*>(a & ~(uintptr_t)3);
    const uint32_t w0 = lim > 12 ? gld4(wa) : 0u, w1 = lim > 16 ? gld4(wa + 4) : 0u, w2 = lim > 20 ? gld4(wa + 8) : 0u;
    uint32_t v0, v1;
    l2_vlans(len, __builtin_bswap32(__builtin_amdgcn_alignbyte(w1, w0, sh)),
             __builtin_bswap32(__builtin_amdgcn_alignbyte(w2, w1, sh)), v0, v1);
    dd.y = (dd.y & 0x00ffffffu) | (emurx_owner_key(emurx_tk_hash(vport, v0, v1)) << 24);
    reinterpret_cast<uint2*>(desc)[i] = dd;
}

// k_lookup: the owner's half — GetNs + the callback's client rule + the flow decision for
// every received lookup head, against this partition's tables (classify()'s resolve).
// Output slot j = the input slot: n_parts regions of cap emurx_route_rec, valid up to
// recv_count[2 source].  Grid: (heads of a region / kBlock, source region): no division.
// A head with a tail (emurx_parse.h) loads it before the table probes: its units arrive in the
// probes' memory round trip.  An ICMPv6 key's client bucket comes from the hash in its head,
// so that probe need not wait for the tail either; a tuple is needed only by the flow probe.
// The heads are read once: non-temporal LDS-DMA (aux nt); the outputs are stored write-through
// (sc1), so their lines leave this XCD's L2 to the table lines the probes re-read (round 5:
// config D's partitioned step +1.3 %, k_lookup 111 -> 108 us in the phase times,
// profiles/r05/ab_lookup/).  EMURX_LOOKUP_NT=0: the default policies
#ifndef EMURX_LOOKUP_NT
#define EMURX_LOOKUP_NT 1
#endif
#ifndef EMURX_LOOKUP_WPE
#define EMURX_LOOKUP_WPE 6
#endif
template <class Flow>
__device__ __forceinline__ void resolve_owner(const emurx_dev_tables& T, Rec& r, LKey k, uint32_t chash, uint4 kw6,
                                              Flow flow) {
    Probe p;
    const uint32_t tk = emurx_tk_hash(r.vport, r.vlan0, r.vlan1);  // CTunnelKey words
    p.nb = tk & T.ns_mask;
    p.ne = ld_bucket(T.ns_tab, p.nb);
    p.mlo = k.kw[0];
    p.mhi = k.kw[1];
    p.cbk = 0;
    p.ctab = nullptr;
    // the table bases as SGPR values selected per lane (probe_issue)
    uintptr_t tm = (uintptr_t)T.mac_tab, t4 = (uintptr_t)T.ip4_tab, t6 = (uintptr_t)T.ip6_tab;
    asm volatile("" : "+s"(tm), "+s"(t4), "+s"(t6));
    if (k.key == kMac) {
        p.cbk = emurx_mac_hash(tk, p.mlo, p.mhi) & T.mac_mask;
        p.ctab = reinterpret_cast<const uint32_t*>(tm);
    } else if (k.key == kEui) {
        p.cbk = chash & T.mac_mask;
        p.ctab = reinterpret_cast<const uint32_t*>(tm);
    } else if (k.key == kIp4) {
        p.cbk = emurx_ip4_hash(tk, k.kw[0]) & T.ip4_mask;
        p.ctab = reinterpret_cast<const uint32_t*>(t4);
    } else if (k.key == kIp6) {
        p.cbk = chash & T.ip6_mask;
        p.ctab = reinterpret_cast<const uint32_t*>(t6);
    }
    Bucket ce{};
    if (p.ctab) ce = ld_bucket(p.ctab, p.cbk);
    if (lk_ip6key(k.key)) {  // the address from the tail
        k.kw[0] = kw6.x; k.kw[1] = kw6.y; k.kw[2] = kw6.z; k.kw[3] = kw6.w;
        if (k.key == kEui) {
            const uint2 m = eui_mac(kw6.z, kw6.w);
            p.mlo = m.x;
            p.mhi = m.y;
        }
    }
    resolve_done(T, r, k, p, ce, flow);
}
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(EMURX_LOOKUP_WPE))) void k_lookup(const uint8_t* __restrict__ recv,
                                                   const uint32_t* __restrict__ recv_count, uint32_t n_parts,
                                                   uint32_t cap, uint32_t tcap, emurx_dev_tables T,
                                                   emurx_route_rec* __restrict__ out, uint32_t* __restrict__ flow) {
    // the wave's 64 heads are contiguous: 2 KiB copied into LDS by two fully coalesced LDS-DMA
    // loads; the rows then hold the wave's 40-byte outputs (2.5 KiB)
    __shared__ __attribute__((aligned(16))) uint4 s_rec[kWaves][kWave * 40 / 16];
    const uint32_t lane = threadIdx.x % kWave, wv = threadIdx.x / kWave;
    const uint32_t src = blockIdx.y, idx0 = blockIdx.x * kBlock + wv * kWave, idx = idx0 + lane;
    const uint32_t cnt = min(recv_count[2 * src], cap);
    if (idx0 >= cnt) return;  // wave-uniform
    const uint64_t j = (uint64_t)src * cap + idx;
    const uint8_t* region = recv + (uint64_t)src * (cap + 32ull * tcap) * 32;
    const uint4* base = reinterpret_cast<const uint4*>(region) + (uint64_t)idx0 * 2;
    const uint32_t nvec = min(kWave, cnt - idx0) * 2;  // never past the region's valid heads
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k)
        if (k * kWave + lane < nvec)
            __builtin_amdgcn_global_load_lds(base + k * kWave + lane,
                                             (__attribute__((address_space(3))) void*)&s_rec[wv][k * kWave], 16, 0,
                                             EMURX_LOOKUP_NT ? 2 : 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool live = idx < cnt;
    const uint4 q0 = s_rec[wv][lane * 2], q1 = s_rec[wv][lane * 2 + 1];
    const uint32_t w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    Rec r;
    uint32_t chash;
    const LKey k = unpack_lookup(w, r, chash);
    // the tail: issued ahead of the table probes (an index past the shards, EMURX_TAIL_NONE
    // included, is not read: the source reported that overflow and must route the batch again)
    const uint32_t tun = live ? lk_tail_units(w[4]) : 0u;
    uint4 t0 = make_uint4(0, 0, 0, 0), t1 = t0, t2 = t0;
    const bool tail_ok = tun && w[7] < EMURX_TAIL_SHARDS * tcap && w[7] + tun <= EMURX_TAIL_SHARDS * tcap;
    // a tcp / udp head without its c5tuplekey (the source's handle saw no TransportCtx when it
    // routed, or the tuple's tail did not fit its shard) cannot take the flow decision here: its
    // flow is EMURX_FLOW_UNKNOWN instead of a probe with a zero tuple
    const bool has_tuple = (w[4] >> 31) && tail_ok;
    if (tail_ok) {
        const uint4* tl = reinterpret_cast<const uint4*>(region + (uint64_t)cap * 32) + w[7];
        t0 = tl[0];
        if (tun == 3) {
            t1 = tl[1];
            t2 = tl[2];
        }
    }
    // frames that reached no callback travel too (their owner keeps their record): no lookup
    if (live && r.status == EMURX_ST_OK)
        resolve_owner(T, r, k, chash, t0, [&](uint32_t cid) {
            return has_tuple ? flow_probe(T, tail_tuple(w, t0, t1, t2), cid) : EMURX_FLOW_UNKNOWN;
        });
    // The wave's outputs are contiguous: its 40-B records are parked in its (now read) LDS rows
    // and written back as five 8-B pieces per lane, 512 contiguous bytes per store instruction,
    // instead of five 8-B stores per lane 40 B apart
    uint2* park = reinterpret_cast<uint2*>(s_rec[wv]);
    if (live) {
        park[lane * 5 + 0] = make_uint2(r.ns, r.cl);
        park[lane * 5 + 1] = make_uint2(r.vlan0, r.vlan1);
        park[lane * 5 + 2] = make_uint2(r.vport | (r.l3 << 16), r.l4 | (r.l7 << 16));
        park[lane * 5 + 3] = make_uint2(r.l7len | (r.nh << 16) | (r.proto << 24), r.status | (r.flags << 8));
        park[lane * 5 + 4] = make_uint2(w[0], src);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint2* o = reinterpret_cast<uint2*>(out + (uint64_t)src * cap + idx0);  // 8-B aligned
    const uint32_t npieces = min(kWave, cnt - idx0) * 5;
#pragma unroll
    for (uint32_t k5 = 0; k5 < 5; ++k5)
        if (k5 * kWave + lane < npieces) {
#if EMURX_LOOKUP_NT
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(o) + k5 * kWave + lane,
                               reinterpret_cast<const unsigned long long*>(park)[k5 * kWave + lane], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);  // sc1: the line leaves this XCD's L2
#else
            o[k5 * kWave + lane] = park[k5 * kWave + lane];
#endif
        }
    if (flow && live) flow[j] = r.flow;
}

}  // namespace emurx

int emurx_launch_owner_count(const uint8_t* frames, const emurx_desc* desc, uint32_t n, uint32_t n_parts,
                             uint32_t* send_count, uint32_t* tile_cnt, uint32_t* grp, uint32_t* grp_off,
                             uint32_t* tcur, hipStream_t st) {
    using namespace emurx;
    const uint32_t ntiles = (n + kBlock - 1) / kBlock, ngroups = (ntiles + kGroup - 1) / kGroup;
    if (n == 0) return EMURX_HIP_OK(hipMemsetAsync(send_count, 0, 2 * n_parts * sizeof(uint32_t), st)) ? 0 : -1;
    if (ngroups > kScanThreads) return -1;
    if (!EMURX_HIP_OK(emurx_launch(k_owner_count, dim3((ntiles + kOcTpw - 1) / kOcTpw), dim3(kBlock), 0, st, frames,
                                   desc, n, n_parts, tile_cnt, grp)))
        return -1;
    return EMURX_HIP_OK(emurx_launch(k_route_scan, dim3(1), dim3(kScanThreads), 0, st, grp, ngroups, n_parts, grp_off,
                                     send_count, tcur, 2u))
               ? 0
               : -1;
}

int emurx_launch_desc_keys(const uint8_t* frames, emurx_desc* desc, uint32_t n, hipStream_t st) {
    using namespace emurx;
    if (!n) return 0;
    return EMURX_HIP_OK(emurx_launch(k_desc_keys, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, frames, desc, n))
               ? 0
               : -1;
}

int emurx_launch_lookup(const emurx_lookup_rec* recv, const uint32_t* recv_count, uint32_t n_parts, uint32_t cap,
                        uint32_t tcap, const emurx_dev_tables& T, emurx_route_rec* out, uint32_t* flow,
                        hipStream_t st) {
    using namespace emurx;
    if (!n_parts || !cap) return 0;
    if (n_parts > 65535) return -1;
// k_lookup's occupancy is capped at 4 workgroups (16 waves) per CU by unused LDS: its 10 KiB of
// record rows + 30 KiB = 40 KiB of the CU's 160 KiB.  Its probes are random table lines; more
// waves in flight only queue more of them, and beside the next batch's k_rx<2> on the other
// stream the freed slots serve that kernel (6 workgroups 98.4 us per 2M records,
// 4: 96.9 us, the pipelined partitioned step +3-4.5 %; at an owner of 8, 74.3 -> 72.3 us)
#ifndef EMURX_LOOKUP_LDS_PAD
#define EMURX_LOOKUP_LDS_PAD (30 * 1024)
#endif
    return EMURX_HIP_OK(emurx_launch(k_lookup, dim3((cap + kBlock - 1) / kBlock, n_parts), dim3(kBlock), EMURX_LOOKUP_LDS_PAD, st,
                                     reinterpret_cast<const uint8_t*>(recv), recv_count, n_parts, cap, tcap, T, out, flow))
               ? 0
               : -1;
}

int emurx_launch_route(const emurx_rec* rec, uint32_t n, uint32_t n_parts, uint32_t my_rank, uint32_t cap,
                       emurx_route_rec* send, uint32_t* send_count, uint32_t* tile_cnt, uint32_t* grp,
                       uint32_t* grp_off, hipStream_t st, bool counted) {
    using namespace emurx;
    const uint32_t ntiles = (n + kBlock - 1) / kBlock, ngroups = (ntiles + kGroup - 1) / kGroup;
    if (n == 0) return EMURX_HIP_OK(hipMemsetAsync(send_count, 0, n_parts * sizeof(uint32_t), st)) ? 0 : -1;
    if (ngroups > kScanThreads) return -1;
    if (!counted &&  // else k_rx counted the owners of this batch (emurx_classify_route_dev)
        !EMURX_HIP_OK(emurx_launch(k_route<false>, dim3(ntiles), dim3(kBlock), 0, st, rec, n, n_parts, my_rank,
                                   tile_cnt, grp, (const uint32_t*)nullptr, send, cap)))
        return -1;
    if (!EMURX_HIP_OK(emurx_launch(k_route_scan, dim3(1), dim3(kScanThreads), 0, st, grp, ngroups, n_parts, grp_off,
                                   send_count, (uint32_t*)nullptr, 1u)))
        return -1;
    return EMURX_HIP_OK(emurx_launch(k_route<true>, dim3(ntiles), dim3(kBlock), 0, st, rec, n, n_parts, my_rank,
                                     tile_cnt, grp, grp_off, send, cap))
               ? 0
               : -1;
}
