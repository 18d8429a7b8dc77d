// emurx_txzmq.hip — tx ZMQ framing on the device (gfx950): VethIFZmq.Send / FlushTx,
// src/emu/core/veth_zmq.go:149-200, SURVEY.md §8f row 1.
//
// Send closes the open message before a frame whose length would bring the message's frame
// bytes to ZMQ_TX_MAX_BUFFER_SIZE or more, and after its ZMQ_TX_PKT_BURST_SIZE-th frame.
// The message boundaries are therefore a greedy chain: the message that starts at frame i
// ends at end(i) = min(i + 64, n, first j > i whose frames i..j reach 32 KiB), and the
// messages start at 0, end(0), end(end(0)), ...  Each message spans at most 64 frames, so
// the chain crosses every 64-frame tile at an entry offset in [0, 64):
//   k_txz_leaf     per tile and per possible entry e (one lane each): the exit offset into
//                  the next tile and the messages started inside; the tile's frame bytes.
//   k_txz_compose  the same functions for 64 consecutive units at once (LDS tables), one
//                  level up, until one unit is left (a scan of the chain's transfer
//                  functions; levels: n / 64, n / 4096, ...).
//   k_txz_descend  from the root down: each unit's actual entry, message base and byte base.
//   k_txz_write    per tile: the message starts (a scalar walk from the entry), each frame's
//                  output offset = 4 (msg + 1) + 4 i + bytes before i, the headers, and the
//                  frame bytes copied by the whole wave frame after frame.
// end(i) needs only the 64 frames after i: a wave holds the prefix sums of its tile and the
// next one in LDS and finds the 32 KiB crossing by binary search.
#include <hip/hip_runtime.h>

#include "../../include/emu_rx.h"
#include "emurx_kernels.h"
#include "emurx_parse.h"

namespace emurx {

constexpr uint32_t kTxTile = 64;  // frames per wave; == EMURX_ZMQ_TX_BURST
static_assert(kTxTile == EMURX_ZMQ_TX_BURST && kTxTile == kWave, "one burst per wave");

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (uint32_t d = 1; d < kWave; d <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)v, d);
        if (lane >= d) v += u;
    }
    return v;
}

// end(i) - i for lane i of the tile at `base` (1..64; 0 past n).  q: this wave's 128 LDS words.
__device__ __forceinline__ uint32_t tx_endrel(const emurx_desc* __restrict__ d, uint32_t n, uint32_t base,
                                              uint32_t* q, uint32_t& len) {
    const uint32_t lane = lane_id();
    len = base + lane < n ? d[base + lane].len : 0u;
    const uint32_t lb = base + kTxTile + lane < n ? d[base + kTxTile + lane].len : 0u;
    const uint32_t qa = wave_incl_scan_u32(len);
    const uint32_t qb = wave_incl_scan_u32(lb) + (uint32_t)__shfl((int)qa, kWave - 1);
    q[lane] = qa;
    q[kWave + lane] = qb;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // first j in (i, i + 64) with Q[j] - Q[i - 1] >= MAX, else i + 64 (6 fixed steps)
    const uint32_t thr = qa - len + EMURX_ZMQ_TX_MAX_BUFFER;
    uint32_t lo = lane + 1, hi = lane + kTxTile;
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        const uint32_t mid = (lo + hi) >> 1;
        const bool ge = lo < hi && q[mid] >= thr;
        hi = ge ? mid : hi;
        lo = (lo < hi && !ge) ? mid + 1 : lo;
    }
    const uint32_t lim = n - base;  // frames of this tile and after
    const uint32_t end = min(lo, lim);
    return lane < lim ? end - lane : 0u;
}

// per tile: X[t][e], M[t][e] for entry e (lane e), B[t] = the tile's frame bytes
__global__ __launch_bounds__(256) void k_txz_leaf(const emurx_desc* __restrict__ d, uint32_t n, uint32_t ntiles,
                                                  uint32_t* __restrict__ X, uint32_t* __restrict__ M,
                                                  unsigned long long* __restrict__ B) {
    __shared__ uint32_t s_q[4][2 * kWave];
    __shared__ uint32_t s_er[4][kWave];
    const uint32_t wv = threadIdx.x / kWave, lane = lane_id();
    const uint32_t t = blockIdx.x * 4 + wv;
    if (t >= ntiles) return;  // wave-uniform
    const uint32_t base = t * kTxTile;
    uint32_t len;
    const uint32_t er = tx_endrel(d, n, base, s_q[wv], len);
    s_er[wv][lane] = er;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t lim = min(n - base, kTxTile);
    uint32_t s = lane, m = 0;
    while (s < lim) {  // <= 64 steps; each message advances by >= 1 frame
        s += s_er[wv][s];
        ++m;
    }
    X[(size_t)t * kWave + lane] = s >= kTxTile ? s - kTxTile : 0u;
    M[(size_t)t * kWave + lane] = m;
    const uint32_t tot = (uint32_t)__shfl((int)wave_incl_scan_u32(len), kWave - 1);
    if (lane == 0) B[t] = tot;
}

// One wave's LDS for a compose / descend step: the 64 children's X / M tables, B, and the
// descend's outputs
struct TxUnitLds {
    uint32_t sx[64][kWave], sm[64][kWave];
    unsigned long long sb[64];
    uint32_t se[64], smb[64];
    unsigned long long sbb[64];
};
__device__ __forceinline__ void tx_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t tx_load_children(const uint32_t* __restrict__ Xc, const uint32_t* __restrict__ Mc,
                                                     const unsigned long long* __restrict__ Bc, uint32_t nc, uint32_t p,
                                                     TxUnitLds& S) {
    // the children's rows straight into LDS by LDS-DMA (one 256-byte row per instruction, all
    // in flight before one wait) instead of a load and a store per row and lane
    const uint32_t lane = lane_id(), c0 = p * 64, cn = min(nc - c0, 64u);
    for (uint32_t c = 0; c < cn; ++c) {
        __builtin_amdgcn_global_load_lds(Xc + (size_t)(c0 + c) * kWave + lane,
                                         (__attribute__((address_space(3))) void*)&S.sx[c][0], 4, 0, 0);
        __builtin_amdgcn_global_load_lds(Mc + (size_t)(c0 + c) * kWave + lane,
                                         (__attribute__((address_space(3))) void*)&S.sm[c][0], 4, 0, 0);
    }
    S.sb[lane] = lane < cn ? Bc[c0 + lane] : 0ull;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the rows landed
    tx_wave_sync();
    return cn;
}
// 64 children -> parent p (one wave): X/M composed along the chain for every entry, B summed
__device__ __forceinline__ void tx_compose(const uint32_t* __restrict__ Xc, const uint32_t* __restrict__ Mc,
                                           const unsigned long long* __restrict__ Bc, uint32_t nc, uint32_t p,
                                           uint32_t* __restrict__ Xp, uint32_t* __restrict__ Mp,
                                           unsigned long long* __restrict__ Bp, TxUnitLds& S) {
    const uint32_t lane = lane_id(), cn = tx_load_children(Xc, Mc, Bc, nc, p, S);
    uint32_t e = lane, m = 0;
    for (uint32_t c = 0; c < cn; ++c) {
        m += S.sm[c][e];
        e = S.sx[c][e];
    }
    Xp[(size_t)p * kWave + lane] = e;
    Mp[(size_t)p * kWave + lane] = m;
    if (lane == 0) {
        unsigned long long b = 0;
        for (uint32_t c = 0; c < cn; ++c) b += S.sb[c];
        Bp[p] = b;
    }
}
// parent p -> its 64 children (one wave): actual entry, message base, byte base of each child.
// info != nullptr: p is the root (entry 0, bases 0), and its message count and total size go to
// info and msg_off[n_msgs]
__device__ __forceinline__ void tx_descend(const uint32_t* __restrict__ Xc, const uint32_t* __restrict__ Mc,
                                           const unsigned long long* __restrict__ Bc, uint32_t nc, uint32_t p,
                                           const uint32_t* __restrict__ Ep, const uint32_t* __restrict__ MBp,
                                           const unsigned long long* __restrict__ BBp, uint32_t* __restrict__ Ec,
                                           uint32_t* __restrict__ MBc, unsigned long long* __restrict__ BBc,
                                           uint32_t n, unsigned long long* __restrict__ msg_off,
                                           unsigned long long* __restrict__ info, TxUnitLds& S) {
    const uint32_t lane = lane_id(), c0 = p * 64, cn = tx_load_children(Xc, Mc, Bc, nc, p, S);
    if (info && lane == 0) {
        const unsigned long long nm = S.sm[0][0];
        const unsigned long long total = 4ull * nm + 4ull * n + S.sb[0];
        info[0] = nm;
        info[1] = total;
        msg_off[nm] = total;
    }
    if (lane == 0) {
        uint32_t e = Ep ? Ep[p] : 0u, mb = MBp ? MBp[p] : 0u;
        unsigned long long bb = BBp ? BBp[p] : 0ull;
        for (uint32_t c = 0; c < cn; ++c) {
            S.se[c] = e;
            S.smb[c] = mb;
            S.sbb[c] = bb;
            mb += S.sm[c][e];
            e = S.sx[c][e];
            bb += S.sb[c];
        }
    }
    tx_wave_sync();
    if (lane < cn) {
        Ec[c0 + lane] = S.se[lane];
        MBc[c0 + lane] = S.smb[lane];
        BBc[c0 + lane] = S.sbb[lane];
    }
}

__global__ __launch_bounds__(64) void k_txz_compose(const uint32_t* __restrict__ Xc, const uint32_t* __restrict__ Mc,
                                                    const unsigned long long* __restrict__ Bc, uint32_t nc,
                                                    uint32_t* __restrict__ Xp, uint32_t* __restrict__ Mp,
                                                    unsigned long long* __restrict__ Bp) {
    __shared__ TxUnitLds S;
    tx_compose(Xc, Mc, Bc, nc, blockIdx.x, Xp, Mp, Bp, S);
}
__global__ __launch_bounds__(64) void k_txz_descend(const uint32_t* __restrict__ Xc, const uint32_t* __restrict__ Mc,
                                                    const unsigned long long* __restrict__ Bc, uint32_t nc,
                                                    const uint32_t* __restrict__ Ep, const uint32_t* __restrict__ MBp,
                                                    const unsigned long long* __restrict__ BBp,
                                                    uint32_t* __restrict__ Ec, uint32_t* __restrict__ MBc,
                                                    unsigned long long* __restrict__ BBc) {
    __shared__ TxUnitLds S;
    tx_descend(Xc, Mc, Bc, nc, blockIdx.x, Ep, MBp, BBp, Ec, MBc, BBc, 0u, nullptr, nullptr, S);
}

// The top of the chain scan in one workgroup of kTxTopWaves waves (a launch per level would
// cost more than the levels' work): the compose levels from k0 (<= kTxTopWaves parents) to the
// root, the root itself (message count, total size), and the descends back down to level k0
constexpr uint32_t kTxTopWaves = 4, kTxMaxLevels = 8;
struct TxLevels {
    uint32_t L, k0, n;
    uint32_t units[kTxMaxLevels];
    uint32_t *X[kTxMaxLevels], *M[kTxMaxLevels], *E[kTxMaxLevels], *MB[kTxMaxLevels];
    unsigned long long *B[kTxMaxLevels], *BB[kTxMaxLevels];
    unsigned long long *msg_off, *info;
};
__global__ __launch_bounds__(kTxTopWaves * kWave) void k_txz_top(const TxLevels t) {
    __shared__ TxUnitLds S[kTxTopWaves];
    const uint32_t wv = threadIdx.x / kWave;
    for (uint32_t k = t.k0; k < t.L; ++k) {
        if (wv < t.units[k])
            tx_compose(t.X[k - 1], t.M[k - 1], t.B[k - 1], t.units[k - 1], wv, t.X[k], t.M[k], t.B[k], S[wv]);
        __threadfence();
        __syncthreads();
    }
    const uint32_t r = t.L - 1;  // the root: entry 0, bases 0
    if (wv == 0)
        tx_descend(t.X[r], t.M[r], t.B[r], 1u, 0u, nullptr, nullptr, nullptr, t.E[r], t.MB[r], t.BB[r], t.n,
                   t.msg_off, t.info, S[0]);
    __threadfence();
    __syncthreads();
    for (uint32_t k = t.L - 1; k >= t.k0 && k >= 1; --k) {
        if (wv < t.units[k])
            tx_descend(t.X[k - 1], t.M[k - 1], t.B[k - 1], t.units[k - 1], wv, t.E[k], t.MB[k], t.BB[k], t.E[k - 1],
                       t.MB[k - 1], t.BB[k - 1], t.n, nullptr, nullptr, S[wv]);
        __threadfence();
        __syncthreads();
    }
}

// the root unit (entry 0): message count and total size; msg_off[n_msgs] = total
__global__ void k_txz_finish(const uint32_t* __restrict__ Mroot, const unsigned long long* __restrict__ Broot,
                             uint32_t n, unsigned long long* __restrict__ msg_off,
                             unsigned long long* __restrict__ info) {
    if (threadIdx.x != 0) return;
    const unsigned long long nm = n ? Mroot[0] : 0u;
    const unsigned long long total = 4ull * nm + 4ull * n + (n ? Broot[0] : 0ull);
    info[0] = nm;
    info[1] = total;
    msg_off[nm] = total;
}

// LDS budget of the staged write path, per wave: the source blocks of the tile's frames and the
// tile's output bytes (headers + frames), both as 16-byte rows
constexpr uint32_t kTxSrc = 6144, kTxOut = 6144 + 32;
constexpr uint32_t kTxSlow = 512;  // long-frame tiles: rows assembled byte by byte, listed per wave
static_assert(kTxSrc % (16 * kWave) == 0, "whole 1 KiB LDS-DMA rows");

// OR a little-endian word v into LDS bytes [p, p + 4) (dwords at p >> 2 and the next one)
__device__ __forceinline__ void lds_or4(uint32_t* o32, uint32_t p, uint32_t v) {
    const uint32_t sh = 8 * (p & 3);
    atomicOr(&o32[p >> 2], v << sh);
    if (sh) atomicOr(&o32[(p >> 2) + 1], v >> (32 - sh));
}

// kStaged: the tiles whose source blocks and output fit the LDS budget (above), else the rest:
// two launches, so that the long-frame tiles keep the occupancy of a kernel without the LDS
template <bool kStaged>
__global__ __launch_bounds__(256) void k_txz_write(const uint8_t* __restrict__ frames,
                                                   const emurx_desc* __restrict__ d, uint32_t n, uint32_t ntiles,
                                                   const uint32_t* __restrict__ E, const uint32_t* __restrict__ MB,
                                                   const unsigned long long* __restrict__ BB,
                                                   uint8_t* __restrict__ out, unsigned long long cap,
                                                   unsigned long long* __restrict__ msg_off,
                                                   uint32_t* __restrict__ done) {
    __shared__ uint32_t s_q[4][2 * kWave];
    const uint32_t wv = threadIdx.x / kWave, lane = lane_id();
    const uint32_t t = blockIdx.x * 4 + wv;
    if (t >= ntiles) return;  // wave-uniform
    if (!kStaged && done[t]) return;  // the staged launch wrote this tile
    const uint32_t base = t * kTxTile;
    if constexpr (kStaged) {  // decided from the descriptors alone, before the chain work:
        // the output range is at most the frame bytes + 8 per frame (its header and, at most,
        // a message header), so this bound implies the image fits
        const uint32_t lim0 = min(n - base, kTxTile);
        const bool v0 = lane < lim0;
        const emurx_desc d0 = v0 ? d[base + lane] : emurx_desc{0, 0, 0, 0};
        const uint32_t slo = wave_min_u32(v0 ? d0.off : 0xffffffffu);
        const uint32_t shi = wave_max_u32(v0 ? d0.off + d0.len : 0u);
        const uint32_t nsv = shi > slo ? (shi - (slo & ~15u) + 15) >> 4 : 0u;
        const uint32_t tot = wave_reduce((uint32_t)d0.len, [](uint32_t x, uint32_t y) { return x + y; });
        const bool fits = nsv * 16 <= kTxSrc && tot + 8 * lim0 + 32 <= kTxOut;  // wave-uniform
        if (lane == 0) done[t] = fits;
        if (!fits) return;  // the long-frame launch's tile
    }
    uint32_t len;
    const uint32_t er = tx_endrel(d, n, base, s_q[wv], len);
    const uint32_t lim = min(n - base, kTxTile);
    // the chain's starts inside this tile: a scalar walk from the tile's entry
    uint64_t starts = 0;
    for (uint32_t s = (uint32_t)__builtin_amdgcn_readfirstlane((int)E[t]); s < lim;
         s += (uint32_t)__builtin_amdgcn_readlane((int)er, (int)s))
        starts |= 1ull << s;
    const bool valid = lane < lim;
    const uint32_t upto = (uint32_t)__popcll(starts & ((lane == 63) ? ~0ull : ((2ull << lane) - 1)));
    const uint32_t msg = MB[t] + upto - 1;  // upto == 0: the previous tile's last message
    const uint32_t pre = wave_incl_scan_u32(len) - len;
    const unsigned long long fo = 4ull * (msg + 1ull) + 4ull * (base + lane) + BB[t] + pre;
    const emurx_desc dl = valid ? d[base + lane] : emurx_desc{0, 0, 0, 0};
    const bool st = valid && ((starts >> lane) & 1);  // this frame opens a message
    // ---- staged path: the tile's output is one contiguous range [o0, o1): built in LDS (the
    // source blocks by coalesced LDS-DMA, headers and frame bytes OR-ed into a zeroed image at
    // their offsets, funnel-shifted a dword at a time), then written as aligned 16-byte rows;
    // only the partial rows at both ends go out byte by byte (they share lines with the
    // neighbouring tiles' output)
    {
        const uint32_t slo = wave_min_u32(valid ? dl.off : 0xffffffffu);
        const uint32_t shi = wave_max_u32(valid ? dl.off + len : 0u);
        const unsigned long long o0 =
            ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(fo >> 32)) << 32 |
             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)fo)) - ((starts & 1) ? 4 : 0);
        const uint32_t last = lim - 1;
        const unsigned long long o1 =
            ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(fo >> 32), (int)last) << 32 |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)fo, (int)last)) + 4 +
            (uint32_t)__builtin_amdgcn_readlane((int)len, (int)last);
        const uint32_t sbase = slo & ~15u, nsv = shi > slo ? (shi - sbase + 15) >> 4 : 0u;
        const unsigned long long obase = o0 & ~15ull;
        const uint32_t nrow = (uint32_t)(((o1 + 15) & ~15ull) - obase) >> 4;
        if constexpr (kStaged) {  // nsv, nrow within the budget (the test above)
            // 16 B of lead (below) + the budget + 16 B of tail: a frame ending at the budget's
            // last byte reads the dword after it (masked out, but inside the array)
            __shared__ __attribute__((aligned(16))) uint32_t s_src[4][(kTxSrc + 32) / 4];
            __shared__ __attribute__((aligned(16))) uint32_t s_out[4][kTxOut / 4];
            uint32_t* src = s_src[wv];
            uint32_t* o32 = s_out[wv];
            // source blocks land 16 bytes into the slab: a frame's first dword read may start
            // up to 3 bytes before it
            const uint4* gs = reinterpret_cast<const uint4*>(frames + sbase);
#pragma unroll
            for (uint32_t k = 0; k < kTxSrc / 16 / kWave; ++k)
                if (k * kWave < nsv)
                    __builtin_amdgcn_global_load_lds(gs + min(lane + k * kWave, nsv - 1),
                                                     (__attribute__((address_space(3))) void*)(src + 4 + k * kWave * 4),
                                                     16, 0, 0);
            for (uint32_t r = lane; r < kTxOut / 16; r += kWave) reinterpret_cast<uint4*>(o32)[r] = make_uint4(0, 0, 0, 0);
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (valid) {
                const uint32_t p = (uint32_t)(fo - obase);  // the frame header in the image
                if (st) lds_or4(o32, p - 4, __builtin_bswap32(((uint32_t)EMURX_ZMQ_MAGIC << 16) + er));
                lds_or4(o32, p, __builtin_bswap32(((uint32_t)EMURX_ZMQ_PKT_MAGIC << 24) + ((uint32_t)dl.vport << 16) + dl.len));
                // frame bytes: image dword j gets source bytes [4j - p4 + q, + 4), masked to the frame
                const uint32_t p4 = p + 4, q = dl.off - sbase + 16, e = p4 + len;
                if (len) {
                    for (uint32_t j = p4 >> 2; j <= (e - 1) >> 2; ++j) {
                        const uint32_t sb = 4 * j + q - p4;  // >= 13: the 16-byte lead
                        const uint32_t v = __builtin_amdgcn_alignbyte(src[(sb >> 2) + 1], src[sb >> 2], sb & 3);
                        const uint32_t m0 = 4 * j < p4 ? 0xffffffffu << (8 * (p4 & 3)) : 0xffffffffu;
                        const uint32_t m1 = 4 * j + 4 > e ? 0xffffffffu >> (8 * (4 * j + 4 - e)) : 0xffffffffu;
                        const uint32_t m = m0 & m1;
                        if (m == 0xffffffffu) o32[j] = v;  // no other lane writes this dword
                        else atomicOr(&o32[j], v & m);
                    }
                }
                if (st) msg_off[msg] = fo - 4;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            typedef unsigned v4u __attribute__((ext_vector_type(4)));
            for (uint32_t r = lane; r < nrow; r += kWave) {
                const unsigned long long x = obase + 16ull * r;
                const uint4 v = reinterpret_cast<const uint4*>(o32)[r];
                if (x >= o0 && x + 16 <= o1 && x + 16 <= cap) {
                    __builtin_nontemporal_store(v4u{v.x, v.y, v.z, v.w}, reinterpret_cast<v4u*>(out + x));
                } else {
                    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (uint32_t j = 0; j < 16; ++j)
                        if (x + j >= o0 && x + j < o1 && x + j < cap) out[x + j] = (uint8_t)(w4[j >> 2] >> (8 * (j & 3)));
                }
            }
            return;
        }
    }
    // ---- long-frame tiles: the tile's output rows [o0 & ~15, o1) dealt over the lanes, each
    // row's source found from the frames' segments in LDS (a forward walk: a lane's rows
    // ascend), so that a wave keeps one load per lane in flight instead of copying its frames
    // one after another.  A row inside one frame's bytes is two aligned 16-byte loads
    // funnel-shifted into one aligned 16-byte store; rows holding headers or frame ends are
    // assembled byte by byte.
    if constexpr (!kStaged) {
    __shared__ uint32_t s_seg[4][6][kWave];  // segment start, data start, source, length, header, message header
    __shared__ uint32_t s_slow[4][kTxSlow];  // pass 2's rows: row << 6 | the frame its walk starts from
    const unsigned long long o0 =
        ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(fo >> 32)) << 32 |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)fo)) - ((starts & 1) ? 4 : 0);
    const uint32_t last = lim - 1;
    const uint32_t R = (uint32_t)(((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(fo >> 32), (int)last) << 32 |
                                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)fo, (int)last)) + 4 - o0) +
                       (uint32_t)__builtin_amdgcn_readlane((int)len, (int)last);  // output bytes of the tile
    uint32_t(*sg)[kWave] = s_seg[wv];
    if (valid) {
        const uint32_t fr = (uint32_t)(fo - o0);  // the frame header, relative to o0
        sg[0][lane] = st ? fr - 4 : fr;
        sg[1][lane] = fr + 4;
        sg[2][lane] = dl.off;
        sg[3][lane] = len;
        sg[4][lane] = ((uint32_t)EMURX_ZMQ_PKT_MAGIC << 24) + ((uint32_t)dl.vport << 16) + dl.len;
        sg[5][lane] = st ? ((uint32_t)EMURX_ZMQ_MAGIC << 16) + er : 0u;
        if (st) msg_off[msg] = fo - 4;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t head = (uint32_t)(o0 & 15), nrow = (head + R + 15) >> 4;
    const unsigned long long xb = o0 - head;  // 16-byte aligned (d_out is)
    // byte j of row r (relative y): its segment walked forward from k, then the byte
    auto row_byte = [&](uint32_t r, uint32_t j, uint32_t kk) {
        const int y = (int)(16 * r + j) - (int)head;
        const unsigned long long x = xb + 16ull * r + j;
        if (y < 0 || (uint32_t)y >= R || x >= cap) return;
        while (kk < last && sg[0][kk + 1] <= (uint32_t)y) ++kk;
        uint32_t rel = (uint32_t)y - sg[0][kk], v;
        const uint32_t mh = sg[5][kk];
        if (mh && rel < 4) {
            v = (mh >> (24 - 8 * rel)) & 0xff;
        } else {
            if (mh) rel -= 4;
            v = rel < 4 ? (sg[4][kk] >> (24 - 8 * rel)) & 0xff : frames[sg[2][kk] + rel - 4];
        }
        out[x] = (uint8_t)v;
    };
    // pass 1: rows inside one frame's bytes; the others (headers, frame ends, the tile's edge
    // rows, rows past the capacity) listed in LDS for pass 2
    uint32_t* slow = s_slow[wv];
    uint32_t nslow = 0, k = 0;
    constexpr uint32_t kU = 4;  // rows per lane per round, their loads in flight together
    for (uint32_t r0 = 0; r0 < nrow; r0 += kU * kWave) {  // wave-uniform trip count
        uint4 cur[kU], nxt[kU];
        uint32_t sh[kU], kk[kU];
        bool fast[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t r = r0 + u * kWave + lane;
            fast[u] = false;
            kk[u] = k;
            cur[u] = nxt[u] = make_uint4(0, 0, 0, 0);
            sh[u] = 0;
            if (r < nrow) {
                const int y0 = (int)(16 * r) - (int)head;  // the row's first byte, relative to o0
                const uint32_t yc = y0 < 0 ? 0u : (uint32_t)y0;
                while (k < last && sg[0][k + 1] <= yc) ++k;
                kk[u] = k;
                const uint32_t ds = sg[1][k], fl = sg[3][k];
                if (y0 >= (int)ds && (uint32_t)y0 + 16 <= ds + fl && xb + 16ull * r + 16 <= cap) {
                    const uintptr_t sa = (uintptr_t)(frames + sg[2][k] + ((uint32_t)y0 - ds));
                    const uint4* sv = reinterpret_cast<const uint4*>(sa & ~(uintptr_t)15);
                    sh[u] = (uint32_t)(sa & 15);
                    cur[u] = sv[0];
                    if (sh[u]) nxt[u] = sv[1];
                    fast[u] = true;
                }
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t r = r0 + u * kWave + lane;
            if (fast[u]) {
                const uint32_t q = sh[u] >> 2, b = sh[u] & 3;
                const uint32_t w[8] = {cur[u].x, cur[u].y, cur[u].z, cur[u].w, nxt[u].x, nxt[u].y, nxt[u].z, nxt[u].w};
                uint32_t o[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t lo = q == 0 ? w[i] : q == 1 ? w[i + 1] : q == 2 ? w[i + 2] : w[i + 3];
                    const uint32_t hi = q == 0 ? w[i + 1] : q == 1 ? w[i + 2] : q == 2 ? w[i + 3] : w[i + 4];
                    o[i] = __builtin_amdgcn_alignbyte(hi, lo, b);
                }
                *reinterpret_cast<uint4*>(out + xb + 16ull * r) = make_uint4(o[0], o[1], o[2], o[3]);
            }
            const bool slw = r < nrow && !fast[u];
            const uint64_t m = __ballot(slw);
            const uint32_t at = nslow + mbcnt(m);
            if (slw) {
                if (at < kTxSlow) slow[at] = r << 6 | kk[u];
                else for (uint32_t j = 0; j < 16; ++j) row_byte(r, j, kk[u]);  // list full: in place
            }
            nslow += (uint32_t)__popcll(m);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // pass 2: the listed rows a byte per lane, four rows per round (independent loads)
    const uint32_t nb = min(nslow, kTxSlow) * 16;
    for (uint32_t i = lane; i < nb; i += kWave) {
        const uint32_t e = slow[i >> 4];
        row_byte(e >> 6, i & 15, e & 63);
    }
    }
}

}  // namespace emurx

// ---------------------------------------------------------------------------------------
// launcher: scratch holds, per level, X/M [units][64] u32, B [units] u64 and the descend
// outputs E/MB [units] u32, BB [units] u64 (emurx_txz_scratch_bytes sizes it)
// ---------------------------------------------------------------------------------------
size_t emurx_txz_scratch_bytes(uint32_t n) {
    size_t bytes = 0;
    for (uint32_t u = (n + 63) / 64; u; u = u > 1 ? (u + 63) / 64 : 0) bytes += (size_t)u * (64 * 8 + 8 + 8 + 8) + 16;
    return bytes + (size_t)((n + 63) / 64) * 4 + 256;  // + the staged write's tile flags
}

int emurx_launch_tx_zmq(const uint8_t* frames, const emurx_desc* desc, uint32_t n, uint8_t* out, uint64_t cap,
                        uint64_t* msg_off, uint64_t* info, void* scratch, hipStream_t st) {
    using namespace emurx;
    unsigned long long* mo = reinterpret_cast<unsigned long long*>(msg_off);
    unsigned long long* inf = reinterpret_cast<unsigned long long*>(info);
    if (n == 0)
        return EMURX_HIP_OK(emurx_launch(k_txz_finish, dim3(1), dim3(64), 0, st, nullptr, nullptr, 0u, mo, inf)) ? 0
                                                                                                               : -1;
    struct Level {
        uint32_t units;
        uint32_t *X, *M, *E, *MB;
        unsigned long long *B, *BB;
    } lv[8];
    int L = 0;
    uint8_t* p = static_cast<uint8_t*>(scratch);
    for (uint32_t u = (n + 63) / 64;; u = (u + 63) / 64) {
        if (L == 8) return -1;
        Level& l = lv[L++];
        l.units = u;
        l.B = reinterpret_cast<unsigned long long*>(p); p += (size_t)u * 8;
        l.BB = reinterpret_cast<unsigned long long*>(p); p += (size_t)u * 8;
        l.X = reinterpret_cast<uint32_t*>(p); p += (size_t)u * 64 * 4;
        l.M = reinterpret_cast<uint32_t*>(p); p += (size_t)u * 64 * 4;
        l.E = reinterpret_cast<uint32_t*>(p); p += (size_t)u * 4;
        l.MB = reinterpret_cast<uint32_t*>(p); p += (size_t)u * 4;
        p = reinterpret_cast<uint8_t*>(((uintptr_t)p + 15) & ~(uintptr_t)15);
        if (u == 1) break;
    }
    const uint32_t nt = lv[0].units;
    uint32_t* done = reinterpret_cast<uint32_t*>(p);  // [nt] tiles the staged write took
    TxLevels tl{};
    tl.L = (uint32_t)L;
    tl.n = n;
    tl.msg_off = mo;
    tl.info = inf;
    tl.k0 = (uint32_t)L;  // the first level with at most kTxTopWaves units (its parents in the top kernel)
    for (int k = L - 1; k >= 1 && lv[k].units <= kTxTopWaves; --k) tl.k0 = (uint32_t)k;
    for (int k = 0; k < L; ++k) {
        tl.units[k] = lv[k].units;
        tl.X[k] = lv[k].X; tl.M[k] = lv[k].M; tl.E[k] = lv[k].E; tl.MB[k] = lv[k].MB;
        tl.B[k] = lv[k].B; tl.BB[k] = lv[k].BB;
    }
    hipError_t e = emurx_launch(k_txz_leaf, dim3((nt + 3) / 4), dim3(256), 0, st, desc, n, nt, lv[0].X, lv[0].M,
                                lv[0].B);
    for (uint32_t k = 1; k < tl.k0 && e == hipSuccess; ++k)
        e = emurx_launch(k_txz_compose, dim3(lv[k].units), dim3(64), 0, st, lv[k - 1].X, lv[k - 1].M, lv[k - 1].B,
                         lv[k - 1].units, lv[k].X, lv[k].M, lv[k].B);
    if (e == hipSuccess) e = emurx_launch(k_txz_top, dim3(1), dim3(kTxTopWaves * kWave), 0, st, tl);
    for (int k = (int)tl.k0 - 1; k >= 1 && e == hipSuccess; --k)
        e = emurx_launch(k_txz_descend, dim3(lv[k].units), dim3(64), 0, st, lv[k - 1].X, lv[k - 1].M, lv[k - 1].B,
                         lv[k - 1].units, lv[k].E, lv[k].MB, lv[k].BB, lv[k - 1].E, lv[k - 1].MB, lv[k - 1].BB);
    if (e == hipSuccess)
        e = emurx_launch(k_txz_write<true>, dim3((nt + 3) / 4), dim3(256), 0, st, frames, desc, n, nt, lv[0].E,
                         lv[0].MB, lv[0].BB, out, (unsigned long long)cap, mo, done);
    if (e == hipSuccess)
        e = emurx_launch(k_txz_write<false>, dim3((nt + 3) / 4), dim3(256), 0, st, frames, desc, n, nt, lv[0].E,
                         lv[0].MB, lv[0].BB, out, (unsigned long long)cap, mo, done);
    return EMURX_HIP_OK(e) ? 0 : -1;
}
