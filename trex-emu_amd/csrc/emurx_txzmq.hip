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

// 64 children -> one parent: X/M composed along the chain for every entry, B summed
__global__ __launch_bounds__(64) void k_txz_compose(const uint32_t* __restrict__ Xc, const uint32_t* __restrict__ Mc,
                                                    const unsigned long long* __restrict__ Bc, uint32_t nc,
                                                    uint32_t* __restrict__ Xp, uint32_t* __restrict__ Mp,
                                                    unsigned long long* __restrict__ Bp) {
    __shared__ uint32_t sx[64][kWave], sm[64][kWave];
    __shared__ unsigned long long sb[64];
    const uint32_t p = blockIdx.x, lane = lane_id();
    const uint32_t c0 = p * 64, cn = min(nc - c0, 64u);
    for (uint32_t c = 0; c < cn; ++c) {
        sx[c][lane] = Xc[(size_t)(c0 + c) * kWave + lane];
        sm[c][lane] = Mc[(size_t)(c0 + c) * kWave + lane];
    }
    sb[lane] = lane < cn ? Bc[c0 + lane] : 0ull;
    __syncthreads();
    uint32_t e = lane, m = 0;
    for (uint32_t c = 0; c < cn; ++c) {
        m += sm[c][e];
        e = sx[c][e];
    }
    Xp[(size_t)p * kWave + lane] = e;
    Mp[(size_t)p * kWave + lane] = m;
    if (lane == 0) {
        unsigned long long b = 0;
        for (uint32_t c = 0; c < cn; ++c) b += sb[c];
        Bp[p] = b;
    }
}

// one parent -> its 64 children: actual entry, message base, byte base of each child
__global__ __launch_bounds__(64) void k_txz_descend(const uint32_t* __restrict__ Xc, const uint32_t* __restrict__ Mc,
                                                    const unsigned long long* __restrict__ Bc, uint32_t nc,
                                                    const uint32_t* __restrict__ Ep, const uint32_t* __restrict__ MBp,
                                                    const unsigned long long* __restrict__ BBp,
                                                    uint32_t* __restrict__ Ec, uint32_t* __restrict__ MBc,
                                                    unsigned long long* __restrict__ BBc) {
    __shared__ uint32_t sx[64][kWave], sm[64][kWave];
    __shared__ unsigned long long sb[64];
    __shared__ uint32_t se[64], smb[64];
    __shared__ unsigned long long sbb[64];
    const uint32_t p = blockIdx.x, lane = lane_id();
    const uint32_t c0 = p * 64, cn = min(nc - c0, 64u);
    for (uint32_t c = 0; c < cn; ++c) {
        sx[c][lane] = Xc[(size_t)(c0 + c) * kWave + lane];
        sm[c][lane] = Mc[(size_t)(c0 + c) * kWave + lane];
    }
    sb[lane] = lane < cn ? Bc[c0 + lane] : 0ull;
    __syncthreads();
    if (lane == 0) {
        uint32_t e = Ep ? Ep[p] : 0u, mb = MBp ? MBp[p] : 0u;
        unsigned long long bb = BBp ? BBp[p] : 0ull;
        for (uint32_t c = 0; c < cn; ++c) {
            se[c] = e;
            smb[c] = mb;
            sbb[c] = bb;
            mb += sm[c][e];
            e = sx[c][e];
            bb += sb[c];
        }
    }
    __syncthreads();
    if (lane < cn) {
        Ec[c0 + lane] = se[lane];
        MBc[c0 + lane] = smb[lane];
        BBc[c0 + lane] = sbb[lane];
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

__device__ __forceinline__ void put_be32(uint8_t* out, unsigned long long at, unsigned long long cap, uint32_t v) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (at + k < cap) out[at + k] = (uint8_t)(v >> (24 - 8 * k));
}

__global__ __launch_bounds__(256) void k_txz_write(const uint8_t* __restrict__ frames,
                                                   const emurx_desc* __restrict__ d, uint32_t n, uint32_t ntiles,
                                                   const uint32_t* __restrict__ E, const uint32_t* __restrict__ MB,
                                                   const unsigned long long* __restrict__ BB,
                                                   uint8_t* __restrict__ out, unsigned long long cap,
                                                   unsigned long long* __restrict__ msg_off) {
    __shared__ uint32_t s_q[4][2 * kWave];
    const uint32_t wv = threadIdx.x / kWave, lane = lane_id();
    const uint32_t t = blockIdx.x * 4 + wv;
    if (t >= ntiles) return;  // wave-uniform
    const uint32_t base = t * kTxTile;
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
    if (valid) {
        if ((starts >> lane) & 1) {
            msg_off[msg] = fo - 4;
            put_be32(out, fo - 4, cap, ((uint32_t)EMURX_ZMQ_MAGIC << 16) + er);
        }
        put_be32(out, fo, cap, ((uint32_t)EMURX_ZMQ_PKT_MAGIC << 24) + ((uint32_t)dl.vport << 16) + dl.len);
    }
    // the bytes, one frame at a time by the whole wave (coalesced).  Short frames: one byte
    // per lane.  Longer ones: aligned 16-byte output stores, each funnel-shifted out of two
    // aligned 16-byte source vectors, with the head and tail bytes (up to the 16-byte
    // boundaries) stored singly by lanes 0-15 and 16-31.
    for (uint32_t f = 0; f < lim; ++f) {
        const uint32_t fl = (uint32_t)__builtin_amdgcn_readlane((int)len, (int)f);
        const uint8_t* s = frames + (uint32_t)__builtin_amdgcn_readlane((int)dl.off, (int)f);
        const unsigned long long D =
            ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(fo >> 32), (int)f) << 32 |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)fo, (int)f)) + 4;
        if (fl < 128) {
            for (uint32_t k = lane; k < fl; k += kWave)
                if (D + k < cap) out[D + k] = s[k];
            continue;
        }
        const unsigned long long Ee = D + fl, a0 = (D + 15) & ~15ull, a1 = Ee & ~15ull;  // a0 < a1
        const unsigned long long hb = lane < 16 ? D + lane : a1 + (lane - 16);
        if (lane < 32 && hb < (lane < 16 ? a0 : Ee) && hb < cap) out[hb] = s[hb - D];
        const uintptr_t sa = (uintptr_t)(s + (a0 - D));
        const uint4* sv = reinterpret_cast<const uint4*>(sa & ~(uintptr_t)15);
        const uint32_t r = (uint32_t)(sa & 15), q = r >> 2, b = r & 3;
        const uint32_t nch = (uint32_t)((a1 - a0) >> 4);
        for (uint32_t c = lane; c < nch; c += kWave) {
            const uint4 cur = sv[c];
            const uint4 nxt = r ? sv[c + 1] : make_uint4(0, 0, 0, 0);  // r > 0: this chunk's tail
            const uint32_t w[8] = {cur.x, cur.y, cur.z, cur.w, nxt.x, nxt.y, nxt.z, nxt.w};
            uint32_t o[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t lo = q == 0 ? w[i] : q == 1 ? w[i + 1] : q == 2 ? w[i + 2] : w[i + 3];
                const uint32_t hi = q == 0 ? w[i + 1] : q == 1 ? w[i + 2] : q == 2 ? w[i + 3] : w[i + 4];
                o[i] = __builtin_amdgcn_alignbyte(hi, lo, b);
            }
            const unsigned long long x = a0 + 16ull * c;
            if (x + 16 <= cap) {
                *reinterpret_cast<uint4*>(out + x) = make_uint4(o[0], o[1], o[2], o[3]);
            } else {
                for (uint32_t j = 0; j < 16; ++j)
                    if (x + j < cap) out[x + j] = (uint8_t)(o[j >> 2] >> (8 * (j & 3)));
            }
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
    for (uint32_t u = (n + 63) / 64; u; u = u > 1 ? (u + 63) / 64 : 0) bytes += (size_t)u * (64 * 8 + 8 + 8 + 8);
    return bytes + 256;
}

int emurx_launch_tx_zmq(const uint8_t* frames, const emurx_desc* desc, uint32_t n, uint8_t* out, uint64_t cap,
                        uint64_t* msg_off, uint64_t* info, void* scratch, hipStream_t st) {
    (void)hipGetLastError();  // a status left by the caller's own failed HIP call is not this launch's
    using namespace emurx;
    unsigned long long* mo = reinterpret_cast<unsigned long long*>(msg_off);
    unsigned long long* inf = reinterpret_cast<unsigned long long*>(info);
    if (n == 0) {
        hipLaunchKernelGGL(k_txz_finish, dim3(1), dim3(64), 0, st, nullptr, nullptr, 0u, mo, inf);
        return EMURX_HIP_OK(hipGetLastError()) ? 0 : -1;
    }
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
    hipLaunchKernelGGL(k_txz_leaf, dim3((nt + 3) / 4), dim3(256), 0, st, desc, n, nt, lv[0].X, lv[0].M, lv[0].B);
    for (int k = 1; k < L; ++k)
        hipLaunchKernelGGL(k_txz_compose, dim3(lv[k].units), dim3(64), 0, st, lv[k - 1].X, lv[k - 1].M, lv[k - 1].B,
                           lv[k - 1].units, lv[k].X, lv[k].M, lv[k].B);
    hipLaunchKernelGGL(k_txz_finish, dim3(1), dim3(64), 0, st, lv[L - 1].M, lv[L - 1].B, n, mo, inf);
    // the root (one unit) has entry 0, base 0: its own descend writes E/MB/BB of level L-1
    hipLaunchKernelGGL(k_txz_descend, dim3(1), dim3(64), 0, st, lv[L - 1].X, lv[L - 1].M, lv[L - 1].B, 1u,
                       nullptr, nullptr, nullptr, lv[L - 1].E, lv[L - 1].MB, lv[L - 1].BB);
    for (int k = L - 1; k >= 1; --k)
        hipLaunchKernelGGL(k_txz_descend, dim3(lv[k].units), dim3(64), 0, st, lv[k - 1].X, lv[k - 1].M,
                           lv[k - 1].B, lv[k - 1].units, lv[k].E, lv[k].MB, lv[k].BB, lv[k - 1].E, lv[k - 1].MB,
                           lv[k - 1].BB);
    hipLaunchKernelGGL(k_txz_write, dim3((nt + 3) / 4), dim3(256), 0, st, frames, desc, n, nt, lv[0].E, lv[0].MB,
                       lv[0].BB, out, (unsigned long long)cap, mo);
    return EMURX_HIP_OK(hipGetLastError()) ? 0 : -1;
}
