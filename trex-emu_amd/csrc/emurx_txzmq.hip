// emurx_txzmq.hip — tx ZMQ framing on the device (gfx950): VethIFZmq.Send / FlushTx,
// src/emu/core/veth_zmq.go:149-200, SURVEY.md §8f row 1.
//
// Send closes the open message before a frame whose length would bring the message's frame
// bytes to ZMQ_TX_MAX_BUFFER_SIZE or more, and after its ZMQ_TX_PKT_BURST_SIZE-th frame.
// The message boundaries are therefore a greedy chain: the message that starts at frame i
// ends at end(i) = min(i + 64, n, first j > i whose frames i..j reach 32 KiB), and the
// messages start at 0, end(0), end(end(0)), ...  Each message spans at most 64 frames, so
// the chain crosses every 64-frame tile at an entry offset in [0, 64):
//   k_txz_chain    one workgroup per 64 tiles: per tile and per possible entry e (one lane
//                  each) the exit offset into the next tile and the messages started inside
//                  (the tile's transfer function), kept in LDS; the 64 tiles' functions composed
//                  into the unit's, with the running state entering every tile; then, level by
//                  level, the workgroup that finishes a parent's last child composes the parent
//                  (levels: n / 4096, n / 262144, ... units, up to one root entered at 0).
//   k_txz_emit     per tile: its entry, message base and byte base by one running-table lookup
//                  per level from the root down; the message starts (a scalar walk from the
//                  entry); each frame's output offset = 4 (msg + 1) + 4 i + bytes before i; the
//                  tile's output assembled in LDS and written as aligned 16-byte rows.
// end(i) needs only the 64 frames after i: prefix sums of the frame lengths in LDS and a
// binary search for the 32 KiB crossing.
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

#ifndef EMURX_TXC_NOUP
#define EMURX_TXC_NOUP 0
#endif
// end(i) - i for lane i of the tile at `base`, from this tile's and the next tile's lengths
__device__ __forceinline__ uint32_t tx_endrel_v(uint32_t len, uint32_t lb, uint32_t n, uint32_t base, uint32_t* q) {
    const uint32_t lane = lane_id();
    const uint32_t qa = wave_incl_scan_u32(len);
    const uint32_t qb = wave_incl_scan_u32(lb) + (uint32_t)__shfl((int)qa, kWave - 1);
    q[lane] = qa;
    q[kWave + lane] = qb;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t thr = qa - len + EMURX_ZMQ_TX_MAX_BUFFER;
    uint32_t lo = lane + 1, hi = lane + kTxTile;
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        const uint32_t mid = (lo + hi) >> 1;
        const bool ge = lo < hi && q[mid] >= thr;
        hi = ge ? mid : hi;
        lo = (lo < hi && !ge) ? mid + 1 : lo;
    }
    const uint32_t lim = n - base;
    const uint32_t end = min(lo, lim);
    return lane < lim ? end - lane : 0u;
}
// ---- the chain scan: one launch (k_txz_chain) ------------------------------------------
// Level 0 is the 64-frame tiles, level k >= 1 units of 64 level-(k-1) units, up to one root.
// A unit's transfer table T[e] (e = the chain's entry offset into its first tile) packs the
// exit offset into the tile after it and the messages started inside: exit | msgs << 6.  A
// level-k unit also keeps its running table R[c][e] = the state entering child c (entry into
// c | messages before c), and RB[c] = the frame bytes before child c, so that the write
// kernel finds any tile's entry, message base and byte base by one lookup per level from the
// root down (the root's entry is 0) -- no descend pass.  Messages per unit fit 26 bits
// (n < 2^26 frames, checked by the host).
constexpr uint32_t kTxMaxLevels = 6;
// The arrival counters sit at the start of the scratch, at the same place for every n: each
// call's last arrival resets the counters it used, so they are all zero between calls even
// when a call of another size lays the tables out differently (n < 2^26: at most 256 level-2
// units, 4 at level 3, 1 above)
constexpr uint32_t kTxCntPerLevel = 256;
constexpr size_t kTxCntBytes = (size_t)kTxMaxLevels * kTxCntPerLevel * 4;
constexpr uint32_t kTxUnitWaves = 16;  // a level-1 unit (64 tiles, 4096 frames) per workgroup
constexpr uint32_t kTxTilesPerWave = 64 / kTxUnitWaves;
constexpr uint32_t kTxBlocks = 8, kTxBlock = 64 / kTxBlocks;  // compose: 8 blocks of 8 children
struct TxChain {
    uint32_t L, n, ntiles;
    uint32_t units[kTxMaxLevels];
    uint32_t* T[kTxMaxLevels];               // [units][64]; level 0 unused (tables stay in LDS)
    unsigned long long* B[kTxMaxLevels];     // [units] frame bytes; level 0 unused
    uint32_t* R[kTxMaxLevels];               // k >= 1: [units][64][64]
    unsigned long long* RB[kTxMaxLevels];    // k >= 1: [units][64]
    uint32_t* cnt[kTxMaxLevels];             // k >= 2: [units] children finished (reset by the last)
    unsigned long long *msg_off, *info;
    uint32_t* fb;  // non-null: the largest bound of a tile's output rows and ~ the smallest, atomicMax
};
struct TxChainLds {
    uint32_t t[64][64];         // the children's tables
    unsigned long long b[64];   // the children's bytes
    union {
        struct {                // the leaf: per wave, prefix sums of 320 frames and end(i) - i of 256
            uint32_t q[kTxUnitWaves][64 * (kTxTilesPerWave + 1)];
            uint32_t er[kTxUnitWaves][64 * kTxTilesPerWave];
        } leaf;
        struct {                // the compose: running tables per block, block tables, block prefixes
            uint32_t q[64][64];
            uint32_t blk[kTxBlocks][64];
            uint32_t p[kTxBlocks + 1][64];
        } up;
    } u;
    uint32_t fbw[kTxUnitWaves][2];  // the size feedback's per-wave bounds
    uint32_t last;
};
__device__ __forceinline__ void tx_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// The hand-off between the workgroup that composes a unit and the one that composes its parent
// (MI355X_MICROARCH.md's hand-off table, row 1): T and B stored write-through (sc1), every
// storing wave waits for its stores, a workgroup barrier, one agent-scope atomic add per
// workgroup; the workgroup whose add came last reads them with sc1 loads after a barrier.
// No __threadfence: its L2 write-back and invalidate, on every wave, cost more than the chain
__device__ __forceinline__ void tx_st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void tx_block_sync() {
    __syncthreads();
}

// Compose unit p of level k from the children's tables in S.t / S.b (cn of them), in two parts:
// tx_compose_table -- 8 blocks of 8 children walked by waves 0-7 (8 dependent LDS steps, the
// running state kept in LDS), the block prefixes by wave 0 (8 steps): the unit's table T and
// bytes B (write-through: the parent's composer reads them) and RB; tx_compose_rows -- the
// running rows R by a gather (read by the write kernel only, so they are stored while the
// unit's arrival is in flight), and the root's message count and total size.
__device__ void tx_compose_table(const TxChain& c, uint32_t k, uint32_t p, uint32_t cn, TxChainLds& S) {
    const uint32_t wv = threadIdx.x / kWave, lane = lane_id();
    if (wv < kTxBlocks) {  // running state within the block, from every entry
        uint32_t x = lane, m = 0;
        for (uint32_t i = 0; i < kTxBlock; ++i) {
            const uint32_t ch = wv * kTxBlock + i;
            S.u.up.q[ch][lane] = x | m << 6;
            if (ch < cn) {
                const uint32_t v = S.t[ch][x];
                x = v & 63u;
                m += v >> 6;
            }
        }
        S.u.up.blk[wv][lane] = x | m << 6;
    }
    tx_block_sync();
    if (wv == 0) {
        uint32_t x = lane, m = 0;
        for (uint32_t w = 0; w < kTxBlocks; ++w) {
            S.u.up.p[w][lane] = x | m << 6;
            const uint32_t v = S.u.up.blk[w][x];
            x = v & 63u;
            m += v >> 6;
        }
        S.u.up.p[kTxBlocks][lane] = x | m << 6;
        tx_st_agent(&c.T[k][(size_t)p * 64 + lane], x | m << 6);
    } else if (wv == 1) {  // bytes before each child, the unit's bytes
        const unsigned long long b = lane < cn ? S.b[lane] : 0ull;
        unsigned long long s = b;
#pragma unroll
        for (uint32_t d = 1; d < kWave; d <<= 1) {
            const unsigned long long u = __shfl_up(s, d);
            if (lane >= d) s += u;
        }
        c.RB[k][(size_t)p * 64 + lane] = s - b;
        if (lane == kWave - 1) __hip_atomic_store(&c.B[k][p], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    tx_block_sync();
}
__device__ void tx_compose_rows(const TxChain& c, uint32_t k, uint32_t p, uint32_t cn, TxChainLds& S) {
    const uint32_t wv = threadIdx.x / kWave, lane = lane_id();
    if (wv < kTxBlocks) {  // R[ch][e] = the block's running state from the block's entry
        const uint32_t pe = S.u.up.p[wv][lane], x0 = pe & 63u, m0 = pe >> 6;
        uint32_t* R = c.R[k] + (size_t)p * 4096;
        for (uint32_t i = 0; i < kTxBlock; ++i) {
            const uint32_t ch = wv * kTxBlock + i;
            const uint32_t v = S.u.up.q[ch][x0];
            R[ch * 64 + lane] = (v & 63u) | ((v >> 6) + m0) << 6;
        }
    }
    if (k == c.L - 1 && threadIdx.x == 0) {  // the root, entered at 0
        const uint32_t r = S.u.up.p[kTxBlocks][0];
        unsigned long long tot = 0;
        for (uint32_t i = 0; i < cn; ++i) tot += S.b[i];
        const unsigned long long nm = r >> 6, total = 4ull * nm + 4ull * c.n + tot;
        c.info[0] = nm;
        c.info[1] = total;
        c.msg_off[nm] = total;
    }
}

// One workgroup per level-1 unit: the 64 tiles' tables (4 tiles per wave, their descriptor
// rows all in flight at once) straight into LDS, the unit composed; then, for each level up,
// the workgroup that finishes a parent's last child composes the parent (arrival count; no
// workgroup ever waits on another).
__global__ __launch_bounds__(kTxUnitWaves * kWave) void k_txz_chain(const emurx_desc* __restrict__ d, const TxChain c) {
    __shared__ TxChainLds S;
    const uint32_t wv = threadIdx.x / kWave, lane = lane_id();
    const uint32_t p = blockIdx.x, n = c.n;
    const uint32_t t0 = p * 64 + wv * kTxTilesPerWave;  // this wave's first tile
    const uint32_t wbase = t0 * kTxTile;
    // ---- leaf: lens of 5 rows (4 tiles + the next one), all loads issued before use
    uint32_t len[kTxTilesPerWave + 1];
#pragma unroll
    for (uint32_t j = 0; j <= kTxTilesPerWave; ++j) {
        const uint32_t i = wbase + j * kWave + lane;
        len[j] = i < n ? d[i].len : 0u;
    }
    uint32_t* q = S.u.leaf.q[wv];
    uint32_t carry = 0;
#pragma unroll
    for (uint32_t j = 0; j <= kTxTilesPerWave; ++j) {
        const uint32_t s = wave_incl_scan_u32(len[j]) + carry;
        q[j * kWave + lane] = s;
        carry = (uint32_t)__shfl((int)s, kWave - 1);
    }
    tx_wave_sync();
    const uint32_t limw = n > wbase ? n - wbase : 0u;  // frames from this wave's base on
    uint32_t* er = S.u.leaf.er[wv];
#pragma unroll
    for (uint32_t j = 0; j < kTxTilesPerWave; ++j) {  // end(i) - i: first g' in (g, g + 64) with
        const uint32_t g = j * kWave + lane;          // Q[g'] - Q[g - 1] >= MAX, else g + 64
        const uint32_t thr = q[g] - len[j] + EMURX_ZMQ_TX_MAX_BUFFER;
        uint32_t lo = g + 1, hi = g + kTxTile;
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            const uint32_t mid = (lo + hi) >> 1;
            const bool ge = lo < hi && q[mid] >= thr;
            hi = ge ? mid : hi;
            lo = (lo < hi && !ge) ? mid + 1 : lo;
        }
        er[g] = g < limw ? min(lo, limw) - g : 0u;
    }
    tx_wave_sync();
    // per tile and entry e (lane): the messages started inside and the exit offset
    uint32_t s[kTxTilesPerWave], m[kTxTilesPerWave], lim[kTxTilesPerWave];
#pragma unroll
    for (uint32_t j = 0; j < kTxTilesPerWave; ++j) {
        const uint32_t tb = j * kWave;
        lim[j] = limw > tb ? min(limw - tb, kTxTile) : 0u;
        s[j] = lane;
        m[j] = 0;
    }
    for (bool any = true; any;) {  // <= 64 rounds: every step advances by >= 1 frame
        any = false;
#pragma unroll
        for (uint32_t j = 0; j < kTxTilesPerWave; ++j)
            if (s[j] < lim[j]) {
                s[j] += er[j * kWave + s[j]];
                ++m[j];
                any = true;
            }
    }
#pragma unroll
    for (uint32_t j = 0; j < kTxTilesPerWave; ++j) {
        const uint32_t ch = wv * kTxTilesPerWave + j;
        S.t[ch][lane] = (s[j] >= kTxTile ? s[j] - kTxTile : 0u) | m[j] << 6;
        const uint32_t tot = q[j * kWave + kWave - 1] - (j ? q[j * kWave - 1] : 0u);
        if (lane == 0) S.b[ch] = tot;
    }
    if (c.fb) {  // the write's variant feedback (emurx_launch_tx_zmq): bounds of the tiles' output rows
        uint32_t hi = 0, lo = 0xffffffffu;
#pragma unroll
        for (uint32_t j = 0; j < kTxTilesPerWave; ++j) {
            const uint32_t tot = q[j * kWave + kWave - 1] - (j ? q[j * kWave - 1] : 0u);
            const uint32_t mm = wave_max_u32(m[j]);  // messages started inside, the most over the entries
            if (lim[j]) {
                hi = max(hi, (tot + 4 * lim[j] + 4 * mm + 30) / 16 + 1);
                lo = min(lo, (tot + 4 * lim[j]) / 16);
            }
        }
        if (lane == 0) {
            S.fbw[wv][0] = hi;
            S.fbw[wv][1] = lo;
        }
    }
    tx_block_sync();
    if (c.fb && threadIdx.x == 0) {
        uint32_t hi = 0, lo = 0xffffffffu;
        for (uint32_t w = 0; w < kTxUnitWaves; ++w) {
            hi = max(hi, S.fbw[w][0]);
            lo = min(lo, S.fbw[w][1]);
        }
        atomicMax(&c.fb[0], hi);
        atomicMax(&c.fb[1], ~lo);  // the smallest lower bound, as the largest complement
    }
    uint32_t cn = min(c.ntiles - p * 64, 64u);
    tx_compose_table(c, 1, p, cn, S);
    // ---- up the levels: the workgroup that completes a parent's last child composes it; a
    // unit's running rows are stored while its arrival's atomic is in flight
    uint32_t up = p;
    for (uint32_t k = 1;; ++k) {
        const bool top = k == c.L - 1;
#if EMURX_TXC_NOUP
        if (!top) {  // timing of the leaf + level-1 compose alone (wrong results past one level)
            tx_compose_rows(c, k, up, cn, S);
            return;
        }
#endif
        const uint32_t par = up >> 6, kids = top ? 0u : min(c.units[k] - par * 64, 64u);
        if (!top) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores of T / B
            tx_block_sync();
            if (threadIdx.x == 0) {
                const uint32_t old =
                    __hip_atomic_fetch_add(&c.cnt[k + 1][par], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                S.last = old == kids - 1;
                if (S.last) tx_st_agent(&c.cnt[k + 1][par], 0u);  // all arrived: ready for the next call
            }
        }
        tx_compose_rows(c, k, up, cn, S);
        if (top) return;
        tx_block_sync();      // S.last, and the rows are done with the LDS the parent's compose reuses
        if (!S.last) return;  // workgroup-uniform
        // the children's tables into LDS (sc1 vector loads: written in this launch, write-through)
        for (uint32_t r = wv; r < kids; r += kTxUnitWaves)
            S.t[r][lane] = __hip_atomic_load(&c.T[k][((size_t)par * 64 + r) * 64 + lane], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        if (threadIdx.x < 64)
            S.b[threadIdx.x] = threadIdx.x < kids ? __hip_atomic_load(&c.B[k][(size_t)par * 64 + threadIdx.x],
                                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                  : 0ull;
        tx_block_sync();
        up = par;
        cn = kids;
        tx_compose_table(c, k + 1, up, cn, S);
    }
}

// Tile t's entry, message base and byte base: one running-table lookup per level, root down
__device__ __forceinline__ void tx_tile_base(const TxChain& c, uint32_t t, uint32_t& e, uint32_t& mb,
                                             unsigned long long& bb) {
    e = 0;
    mb = 0;
    bb = 0;
    for (uint32_t k = c.L - 1; k >= 1; --k) {
        const uint32_t pu = t >> (6 * k), ch = (t >> (6 * (k - 1))) & 63u;
        const uint32_t v = c.R[k][(size_t)pu * 4096 + ch * 64 + e];
        bb += c.RB[k][(size_t)pu * 64 + ch];
        e = v & 63u;
        mb += v >> 6;
    }
}

constexpr uint32_t kTxSlow = 512;  // long-frame tiles: rows assembled byte by byte, listed per wave
// Waves per tile of the long variant (EMURX_TXZ_LONG), A/B knob: split, every wave makes the
// tile's segments itself and copies a contiguous part of its rows.  Measured on config E (1M
// IMIX frames): 1 wave 263 us per call, 2 waves 262-268, 4 waves 288:
// the launch's tail is not what E's write pays for.  1 (one wave per tile) kept.
#ifndef EMURX_TX_SPLIT
#define EMURX_TX_SPLIT 1
#endif
constexpr uint32_t kTxSplit = EMURX_TX_SPLIT;

// OR a little-endian word v into LDS bytes [p, p + 4) (dwords at p >> 2 and the next one)
__device__ __forceinline__ void lds_or4(uint32_t* o32, uint32_t p, uint32_t v) {
    const uint32_t sh = 8 * (p & 3);
    atomicOr(&o32[p >> 2], v << sh);
    if (sh) atomicOr(&o32[(p >> 2) + 1], v >> (32 - sh));
}

// ---- the write, one launch (round 5): the tile's output image in LDS (6 KiB per wave, no source
// slab), each lane's frame bytes loaded straight into registers -- aligned 16-byte loads of the
// blocks that hold the frame, funnel-shifted into the image's dwords -- so that twice as many
// waves are resident as with the staged source; tiles whose output does not fit the image take
// the long-frame path in the same launch, its arrays carved from the same LDS
// kTxImg: output bytes per wave (headers + frames, 16-B rows) of the image path, chosen per launch
// from the tile sizes earlier calls saw (emurx_launch_tx_zmq): 6 KiB (6 waves per SIMD), 4.5 KiB
// (8), or none (every tile takes the long path; its arrays alone, 8 waves).  Every variant
// writes every tile correctly: a tile that does not fit the image takes the long path.
constexpr uint32_t kTxImgWide = 6144, kTxImgNarrow = 4608, kTxLongLds = 6 * kWave * 4 + 512 * 4;
template <uint32_t kTxImg>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kTxImg == kTxImgWide ? 6 : 8))) void k_txz_emit(const uint8_t* __restrict__ frames, const emurx_desc* __restrict__ d,
                                                  uint32_t n, uint32_t ntiles, const TxChain c,
                                                  uint8_t* __restrict__ out, unsigned long long cap,
                                                  unsigned long long* __restrict__ msg_off) {
    constexpr uint32_t kLds = kTxImg > kTxLongLds ? kTxImg : kTxLongLds;
    __shared__ __attribute__((aligned(16))) uint32_t s_img[4][kLds / 4];
    __shared__ uint32_t s_q[4][2 * kWave];
    const uint32_t wv = threadIdx.x / kWave, lane = lane_id();
    // the long variant (no image): kTxSplit waves per tile, each making the tile's segments itself
    // and copying its share of the tile's rows
    constexpr uint32_t kSplit = kTxImg == 0 ? kTxSplit : 1u;
    const uint32_t gw = blockIdx.x * 4 + wv, t = gw / kSplit, part = gw % kSplit;
    if (t >= ntiles) return;  // wave-uniform
    const uint32_t base = t * kTxTile;
    // loads that wait on nothing first: this and the next tile's descriptors, the tile base
    const uint32_t lim = min(n - base, kTxTile);
    const bool valid = lane < lim;
    const emurx_desc dl = valid ? d[base + lane] : emurx_desc{0, 0, 0, 0};
    const uint32_t lnext = base + kTxTile + lane < n ? d[base + kTxTile + lane].len : 0u;
    uint32_t te, tmb;
    unsigned long long tbb;
    tx_tile_base(c, t, te, tmb, tbb);
    const uint32_t len = dl.len;
    const uint32_t er = tx_endrel_v(len, lnext, n, base, s_q[wv]);
    uint64_t starts = 0;  // the chain's starts inside this tile: a scalar walk from the tile's entry
    for (uint32_t s = (uint32_t)__builtin_amdgcn_readfirstlane((int)te); s < lim;
         s += (uint32_t)__builtin_amdgcn_readlane((int)er, (int)s))
        starts |= 1ull << s;
    const uint32_t upto = (uint32_t)__popcll(starts & ((lane == 63) ? ~0ull : ((2ull << lane) - 1)));
    const uint32_t msg = tmb + upto - 1;  // upto == 0: the previous tile's last message
    const uint32_t pre = wave_incl_scan_u32(len) - len;
    const unsigned long long fo = 4ull * (msg + 1ull) + 4ull * (base + lane) + tbb + pre;
    const bool st = valid && ((starts >> lane) & 1);  // this frame opens a message
    if (st) msg_off[msg] = fo - 4;
    const unsigned long long o0 =
        ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(fo >> 32)) << 32 |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)fo)) - ((starts & 1) ? 4 : 0);
    const uint32_t last = lim - 1;
    const unsigned long long o1 =
        ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(fo >> 32), (int)last) << 32 |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)fo, (int)last)) + 4 +
        (uint32_t)__builtin_amdgcn_readlane((int)len, (int)last);
    uint32_t* o32 = s_img[wv];
    const unsigned long long obase = o0 & ~15ull;
    const uint32_t nrow = (uint32_t)(((o1 + 15) & ~15ull) - obase) >> 4;
    if (kTxImg && nrow * 16 <= kTxImg) {  // wave-uniform: the tile's output rows fit the image

        for (uint32_t r = lane; r < nrow; r += kWave) reinterpret_cast<uint4*>(o32)[r] = make_uint4(0, 0, 0, 0);
        tx_wave_sync();
        if (valid) {
            const uint32_t p = (uint32_t)(fo - obase);  // the frame header in the image
            if (st) lds_or4(o32, p - 4, __builtin_bswap32(((uint32_t)EMURX_ZMQ_MAGIC << 16) + er));
            lds_or4(o32, p, __builtin_bswap32(((uint32_t)EMURX_ZMQ_PKT_MAGIC << 24) + ((uint32_t)dl.vport << 16) + len));
            if (len) {
                // image dwords j0 .. j1 take source bytes G0 + 4 i .. + 4 (i = j - j0), G0 = the
                // frame's address - (p4 & 3); they come from the aligned 16-byte blocks from A on
                const uint32_t p4 = p + 4, e = p4 + len, j0 = p4 >> 2, nd = ((e - 1) >> 2) - j0 + 1;
                const uintptr_t F = (uintptr_t)(frames + dl.off), G0 = F - (p4 & 3), A = G0 & ~(uintptr_t)15;
                const uintptr_t Fend = F + len;
                const uint32_t qd = (uint32_t)(G0 & 15) >> 2, sb = (uint32_t)(G0 & 3);
                for (uint32_t i0 = 0; i0 < nd; i0 += 16) {  // 16 image dwords per round, 5 blocks in flight
                    uint32_t W[20];
#pragma unroll
                    for (uint32_t v = 0; v < 5; ++v) {
                        const uintptr_t a = A + 4 * i0 + 16 * v;  // 4 * i0: i0 is a multiple of 16
                        uint4 x = make_uint4(0, 0, 0, 0);
                        // only blocks that hold a frame byte are read (the first may lie wholly
                        // before the frame: G0 is up to 3 bytes before it; those bytes are masked)
                        if (a < Fend && a + 16 > F) x = *reinterpret_cast<const uint4*>(a);
                        W[4 * v] = x.x; W[4 * v + 1] = x.y; W[4 * v + 2] = x.z; W[4 * v + 3] = x.w;
                    }
#pragma unroll
                    for (uint32_t ii = 0; ii < 16; ++ii) {
                        const uint32_t i = i0 + ii;
                        if (i < nd) {
                            const uint32_t lo = qd == 0 ? W[ii] : qd == 1 ? W[ii + 1] : qd == 2 ? W[ii + 2] : W[ii + 3];
                            const uint32_t hi = qd == 0 ? W[ii + 1] : qd == 1 ? W[ii + 2] : qd == 2 ? W[ii + 3] : W[ii + 4];
                            const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, sb);
                            const uint32_t j = j0 + i;
                            const uint32_t m0 = 4 * j < p4 ? 0xffffffffu << (8 * (p4 & 3)) : 0xffffffffu;
                            const uint32_t m1 = 4 * j + 4 > e ? 0xffffffffu >> (8 * (4 * j + 4 - e)) : 0xffffffffu;
                            const uint32_t m = m0 & m1;
                            if (m == 0xffffffffu) o32[j] = v;  // no other lane writes this dword
                            else atomicOr(&o32[j], v & m);
                        }
                    }
                }
            }
        }
        tx_wave_sync();
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
    // ---- long-frame tiles: the tile's output rows [o0 & ~15, o1) dealt over the lanes, each
    // row's source found from the frames' segments (a forward walk: a lane's rows ascend), so
    // that a wave keeps one load per lane in flight instead of copying its frames one after
    // another.  A row inside one frame's bytes is two aligned 16-byte loads funnel-shifted into
    // one aligned 16-byte store; rows holding headers or frame ends are assembled byte by byte.
    // The segment table and the slow-row list live in this wave's image space
    uint32_t(*sg)[kWave] = reinterpret_cast<uint32_t(*)[kWave]>(o32);  // [6][64]
    uint32_t* slow = o32 + 6 * kWave;                                   // [kTxSlow]
    static_assert(6 * kWave * 4 + kTxSlow * 4 <= kLds, "long path's arrays in the image space");
    const uint32_t R = (uint32_t)(o1 - o0);  // output bytes of the tile
    if (valid) {
        const uint32_t fr = (uint32_t)(fo - o0);  // the frame header, relative to o0
        sg[0][lane] = st ? fr - 4 : fr;
        sg[1][lane] = fr + 4;
        sg[2][lane] = dl.off;
        sg[3][lane] = len;
        sg[4][lane] = ((uint32_t)EMURX_ZMQ_PKT_MAGIC << 24) + ((uint32_t)dl.vport << 16) + dl.len;
        sg[5][lane] = st ? ((uint32_t)EMURX_ZMQ_MAGIC << 16) + er : 0u;
    }
    tx_wave_sync();
    const uint32_t head = (uint32_t)(o0 & 15);  // nrow (above) = (head + R + 15) / 16
    const unsigned long long xb = o0 - head;  // 16-byte aligned (d_out is)
    auto byte_at = [&](uint32_t y, uint32_t kk) {  // output byte y of the tile (y < R), segment >= kk
        while (kk < last && sg[0][kk + 1] <= y) ++kk;
        uint32_t rel = y - sg[0][kk], v;
        const uint32_t mh = sg[5][kk];
        if (mh && rel < 4) {
            v = (mh >> (24 - 8 * rel)) & 0xff;
        } else {
            if (mh) rel -= 4;
            v = rel < 4 ? (sg[4][kk] >> (24 - 8 * rel)) & 0xff : frames[sg[2][kk] + rel - 4];
        }
        return v;
    };
    auto row_byte = [&](uint32_t r, uint32_t j, uint32_t kk) {
        const int y = (int)(16 * r + j) - (int)head;
        const unsigned long long x = xb + 16ull * r + j;
        if (y < 0 || (uint32_t)y >= R || x >= cap) return;
        out[x] = (uint8_t)byte_at((uint32_t)y, kk);
    };
    uint32_t nslow = 0, k = 0;
#ifndef EMURX_TX_P2ROUND  // 0: the slow rows after the tile's last round (rounds 1-4)
#define EMURX_TX_P2ROUND 1
#endif
#if EMURX_TX_P2ROUND
    uint32_t p2done = 0;
#endif
#ifndef EMURX_TX_KU
#define EMURX_TX_KU 4
#endif
    constexpr uint32_t kU = EMURX_TX_KU;  // rows per lane per round, their loads in flight together
    // this wave's share of the rows: kSplit contiguous parts, whole 64-row groups each
    const uint32_t per = kSplit == 1 ? nrow : ((nrow + kSplit - 1) / kSplit + kWave - 1) & ~(kWave - 1);
    const uint32_t rbeg = min(nrow, part * per), rend = min(nrow, rbeg + per);
    for (uint32_t r0 = rbeg; r0 < rend; r0 += kU * kWave) {  // wave-uniform trip count
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
#ifdef EMURX_TX_PURECOPY  // timing only: every row a copy from the frames buffer's first 256 MiB
            if (r < rend && xb + 16ull * r + 16 <= cap) {
#ifndef EMURX_TX_PC_OFF
#define EMURX_TX_PC_OFF 5
#endif
                const uintptr_t sa = (uintptr_t)(frames + (((uint32_t)xb + 16 * r) & 0x0ffffff0u) + EMURX_TX_PC_OFF);
                const uint4* sv = reinterpret_cast<const uint4*>(sa & ~(uintptr_t)15);
                sh[u] = EMURX_TX_PC_OFF;
                cur[u] = sv[0];
                if (EMURX_TX_PC_OFF) nxt[u] = sv[1];
                fast[u] = true;
            }
            if (false) {
#else
            if (r < rend) {
#endif
                const int y0 = (int)(16 * r) - (int)head;
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
            const bool slw = r < rend && !fast[u];
            const uint64_t m = __ballot(slw);
            const uint32_t at = nslow + mbcnt(m);
            if (slw) {
                if (at < kTxSlow) slow[at] = r << 6 | kk[u];
                else for (uint32_t j = 0; j < 16; ++j) row_byte(r, j, kk[u]);  // list full: in place
            }
            nslow += (uint32_t)__popcll(m);
        }
#if EMURX_TX_P2ROUND && !defined(EMURX_TX_NOPASS2)
        // this round's byte-by-byte rows now, while the lines its full rows wrote are in L2 (a
        // line left partly written costs its write-back a read-modify-write)
        tx_wave_sync();
        const uint32_t nl = min(nslow, kTxSlow);
        for (uint32_t i = p2done * 16 + lane; i < nl * 16; i += kWave) {
            const uint32_t e = slow[i >> 4];
            row_byte(e >> 6, i & 15, e & 63);
        }
        p2done = nl;
#endif
    }
    tx_wave_sync();
#ifdef EMURX_TX_NOPASS2  // timing only: the long path without its byte-by-byte rows (wrong output)
    const uint32_t nb = 0;
#else
    const uint32_t nb = min(nslow, kTxSlow) * 16;
#endif
#if EMURX_TX_P2ROUND
    for (uint32_t i = p2done * 16 + lane; i < nb; i += kWave) {
#else
    for (uint32_t i = lane; i < nb; i += kWave) {
#endif
        const uint32_t e = slow[i >> 4];
        row_byte(e >> 6, i & 15, e & 63);
    }
}

}  // namespace emurx

// ---------------------------------------------------------------------------------------
// launcher: scratch holds, per level, X/M [units][64] u32, B [units] u64 and the descend
// outputs E/MB [units] u32, BB [units] u64 (emurx_txz_scratch_bytes sizes it)
// ---------------------------------------------------------------------------------------
size_t emurx_txz_scratch_bytes(uint32_t n) {
    // per level k >= 1: T [units][64] u32, B [units] u64, R [units][64][64] u32, RB [units][64] u64,
    // after the arrival counters (kTxCntBytes)
    size_t bytes = emurx::kTxCntBytes;
    const uint32_t nt = (n + 63) / 64;
    for (uint32_t u = (nt + 63) / 64;; u = (u + 63) / 64) {
        bytes += (size_t)u * (256 + 16384 + 512) + (((size_t)u * 8 + 511) & ~(size_t)511) + 512;
        if (u <= 1) break;
    }
    return bytes;
}

int emurx_launch_tx_zmq(const uint8_t* frames, const emurx_desc* desc, uint32_t n, uint8_t* out, uint64_t cap,
                        uint64_t* msg_off, uint64_t* info, void* scratch, hipStream_t st, int variant, bool feedback) {
    using namespace emurx;
    unsigned long long* mo = reinterpret_cast<unsigned long long*>(msg_off);
    unsigned long long* inf = reinterpret_cast<unsigned long long*>(info);
    if (n >= EMURX_TX_ZMQ_MAX_FRAMES) return -1;
    if (n == 0)
        return EMURX_HIP_OK(hipMemsetAsync(inf, 0, 16, st)) && EMURX_HIP_OK(hipMemsetAsync(mo, 0, 8, st)) ? 0 : -1;
    TxChain c{};
    c.n = n;
    c.ntiles = (n + 63) / 64;
    c.units[0] = c.ntiles;
    c.msg_off = mo;
    c.info = inf;
    c.fb = feedback ? static_cast<uint32_t*>(scratch) : nullptr;  // level 0's counter words (unused)
    uint8_t* p = static_cast<uint8_t*>(scratch) + kTxCntBytes;
    uint32_t L = 1;
    for (uint32_t u = (c.ntiles + 63) / 64;; u = (u + 63) / 64) {
        if (L == kTxMaxLevels) return -1;
        c.units[L] = u;
        // every array 512-byte aligned: a parent's 64 children's T rows and B words sit on lines
        // of their own (its hand-off reads them once, after every child stored them)
        c.R[L] = reinterpret_cast<uint32_t*>(p); p += (size_t)u * 16384;
        c.T[L] = reinterpret_cast<uint32_t*>(p); p += (size_t)u * 256;
        c.RB[L] = reinterpret_cast<unsigned long long*>(p); p += (size_t)u * 512;
        c.B[L] = reinterpret_cast<unsigned long long*>(p); p += ((size_t)u * 8 + 511) & ~(size_t)511;
        c.cnt[L] = static_cast<uint32_t*>(scratch) + L * kTxCntPerLevel;  // fixed: see kTxCntBytes
        p = reinterpret_cast<uint8_t*>(((uintptr_t)p + 511) & ~(uintptr_t)511);
        ++L;
        if (u <= 1) break;
    }
    c.L = L;
    const uint32_t nt = c.ntiles;
    hipError_t e = emurx_launch(k_txz_chain, dim3(c.units[1]), dim3(kTxUnitWaves * kWave), 0, st, desc, c);
    if (e == hipSuccess) {
        const uint32_t waves = variant == EMURX_TXZ_LONG ? nt * kTxSplit : nt;  // the long variant: kTxSplit waves per tile
        e = emurx_launch(variant == EMURX_TXZ_NARROW ? k_txz_emit<kTxImgNarrow>
                         : variant == EMURX_TXZ_LONG ? k_txz_emit<0>
                                                     : k_txz_emit<kTxImgWide>,
                         dim3((waves + 3) / 4), dim3(256), 0, st, frames, desc, n, nt, c, out, (unsigned long long)cap, mo);
    }
    return EMURX_HIP_OK(e) ? 0 : -1;
}
