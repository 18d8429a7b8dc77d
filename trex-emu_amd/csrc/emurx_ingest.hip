// emurx_ingest.hip — device side of the batched ZMQ ingest (gfx950).
//
// The host path (emurx_ingest_* / emurx_rx_stream) hands the GPU many ZMQ messages per
// launch (src/emu/core/veth_zmq.go:8-22 wire format) and gets back records, packed
// per-callback queues and folded counters.  Around k_rx (emurx_kernels.hip) run:
//   k_zmq_walk  one lane per message: the offset walk of VethIFZmq.OnRxStream
//               (veth_zmq.go:277-320, uint16 running offset, abort on a header error) ->
//               descriptors in the message's slot range, each with its frame's owner key
//               (EMURX_DESC_KEYED: bytes 12..19 of the frame, loaded with its header);
//               slots past the decoded frames are marked EMURX_DESC_HOLE (k_rx skips them);
//               one status word per message
//   k_qscan     one workgroup: exclusive offset of every (queue, tile) segment of k_rx's
//               per-tile queue output in the packed queue-major order, qoff[14], and the
//               histogram shards folded into one copy (shards left zero for the next batch)
//   k_qpack     one workgroup per tile: copies its segments to their packed positions
// Messages are independent, so the walk needs no cross-lane communication; it is a chain of
// dependent loads per message, latency bound and far off the HBM roofline (the host batch
// is PCIe bound).
#include <hip/hip_runtime.h>

#include "../../include/emu_rx.h"
#include "emurx_kernels.h"
#include "emurx_parse.h"

namespace emurx {

constexpr uint32_t kScanLanes = 512;  // 1024 capped VGPRs at 128 and spilled

// 4 bytes at any address as a big-endian word (two aligned dword loads + funnel shift; the
// staging buffer is padded, so the second dword is always readable)
__device__ __forceinline__ uint32_t ld_be32(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
    const uint32_t lo = gld4(w), hi = gld4(w + 1);
    return __builtin_bswap32(__builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(a & 3)));
}

// kKeys: derive each frame's Namespace-owner key (EMURX_DESC_KEYED) on the way; false only in
// the measurement of what that costs (emurx_zmq_walk_dev, EMURX_WALK_NO_KEYS)
template <bool kKeys>
__global__ __launch_bounds__(kBlock) void k_zmq_walk(const uint8_t* __restrict__ buf,
                                                     const uint32_t* __restrict__ ctl, uint32_t nmsg,
                                                     emurx_desc* __restrict__ desc,
                                                     uint32_t* __restrict__ msg_stat) {
    const uint32_t m = blockIdx.x * kBlock + threadIdx.x;
    if (m >= nmsg) return;
    // ctl: emurx_msg[nmsg] {off, len}, then slot_base[nmsg + 1]
    const uint2 M = reinterpret_cast<const uint2*>(ctl)[m];
    const uint32_t* slot_base = ctl + 2 * nmsg;
    const uint32_t base = slot_base[m], slots = slot_base[m + 1] - base;
    const uint8_t* s = buf + M.x;
    const uint32_t blen = M.y;
    uint32_t found = 0, err = 0;
    if (blen < 4) {
        err = EMURX_MSG_PARSE_ERR;
    } else {
        uint32_t header = ld_be32(s);
        if ((header >> 16) != EMURX_ZMQ_MAGIC) {
            err = EMURX_MSG_PARSE_ERR;
        } else {
            const uint32_t pkts = header & 0xffff;
            uint32_t of = 4;  // uint16 in Go; every accepted frame keeps it below 2^16
            for (uint32_t i = 0; i < pkts; ++i) {
                const uint32_t h4 = (of + 4) & 0xffff;
                if (blen < h4) { err = EMURX_MSG_PARSE_ERR; break; }
                if (h4 < of) { err = EMURX_MSG_PANIC; break; }  // stream[of:of+4] out of range
                // the frame's bytes 12..19 for its owner key come with its header: 32 bytes from
                // the header's aligned dword in two 16-byte loads (one memory round trip per
                // frame, and two load instructions instead of six: each one touches 64 lines, one
                // per message of the wave); read before the header's checks, so up to 28 bytes
                // past a message's end may be read, never used.  (A wave per message guessing 64
                // equal strides per round, and 512-byte LDS windows of each message, both
                // measured slower on config D's mixed sizes: DESIGN.md §6 round 5)
                uint32_t w12 = 0, w16 = 0;
                const uintptr_t a = (uintptr_t)(s + of);
                const uint32_t sh = (uint32_t)(a & 3);
                const uint32_t* wa = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
                if constexpr (kKeys) {
                    const uint4 x = gld16(wa), y = gld16(wa + 4);
                    header = __builtin_bswap32(__builtin_amdgcn_alignbyte(x.y, x.x, sh));
                    w12 = __builtin_bswap32(__builtin_amdgcn_alignbyte(y.y, y.x, sh));  // bytes of+16 .. of+19
                    w16 = __builtin_bswap32(__builtin_amdgcn_alignbyte(y.z, y.y, sh));  // bytes of+20 .. of+23
                } else {  // the header's two dwords in one load
                    typedef unsigned v2u __attribute__((ext_vector_type(2)));
                    const v2u x = *(const __attribute__((address_space(1))) v2u*)wa;
                    header = __builtin_bswap32(__builtin_amdgcn_alignbyte(x.y, x.x, sh));
                }
                if ((header & 0xff000000u) != 0xAA000000u) { err = EMURX_MSG_PARSE_ERR; break; }
                const uint32_t vport = (header >> 16) & 0xff, plen = header & 0xffff;
                const uint32_t e = (of + 4 + plen) & 0xffff;
                if (blen < e) { err = EMURX_MSG_PARSE_ERR; break; }
                if (plen > EMURX_MAX_FRAME) { err = EMURX_MSG_PANIC; break; }  // MbufPoll.Alloc
                if (e < h4) { err = EMURX_MSG_PANIC; break; }
                if (found >= slots) { err = EMURX_MSG_PANIC; break; }  // unreachable: slots bound the walk
                // the owner key from the CTunnelKey the parse will leave (l2_vlans: the frame's
                // bytes 12..19 and its length); bytes past the frame are masked by the length
                uint32_t key = 0;
                if constexpr (kKeys) {
                    uint32_t v0, v1;
                    l2_vlans(plen, w12, w16, v0, v1);
                    key = emurx_owner_key(emurx_tk_hash(vport, v0, v1));
                }
                reinterpret_cast<uint2*>(desc)[base + found] = make_uint2(M.x + h4, plen | (vport << 16) | (key << 24));
                ++found;
                of = e;
            }
        }
    }
    for (uint32_t k = found; k < slots; ++k)
        reinterpret_cast<uint2*>(desc)[base + k] = make_uint2(0, EMURX_DESC_HOLE << 24);
    msg_stat[m] = found | (err << 24);
}

// inclusive wave64 prefix sum
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (uint32_t o = 1; o < kWave; o <<= 1) {
        const uint32_t up = (uint32_t)__shfl_up((int)v, o);
        if (lane >= o) v += up;
    }
    return v;
}

__device__ __forceinline__ void tile_row(const uint32_t* tile_cnt, uint32_t t, uint32_t r[EMURX_NUM_QUEUES]) {
    const uint4* row = reinterpret_cast<const uint4*>(tile_cnt + (size_t)t * 16);
    const uint4 a = row[0], b = row[1], c = row[2], d = row[3];
    r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
    r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
    r[8] = c.x; r[9] = c.y; r[10] = c.z; r[11] = c.w;
    r[12] = d.x;
}

__global__ __launch_bounds__(kScanLanes) void k_qscan(const uint32_t* __restrict__ tile_cnt, uint32_t nt,
                                                      uint32_t* __restrict__ seg_off,
                                                      uint32_t* __restrict__ qoff,
                                                      unsigned long long* __restrict__ hist,
                                                      unsigned long long* __restrict__ hist_out) {
    constexpr uint32_t kW = kScanLanes / kWave;
    __shared__ uint32_t s_w[kW][EMURX_NUM_QUEUES];
    __shared__ uint32_t s_base[EMURX_NUM_QUEUES + 1];
    const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid / kWave;
    const uint32_t per = (nt + kScanLanes - 1) / kScanLanes;
    const uint32_t t0 = min(tid * per, nt), t1 = min(t0 + per, nt);
    uint32_t v[EMURX_NUM_QUEUES], r[EMURX_NUM_QUEUES];
#pragma unroll
    for (int q = 0; q < EMURX_NUM_QUEUES; ++q) v[q] = 0;
    for (uint32_t t = t0; t < t1; ++t) {
        tile_row(tile_cnt, t, r);
#pragma unroll
        for (int q = 0; q < EMURX_NUM_QUEUES; ++q) v[q] += r[q];
    }
    uint32_t ex[EMURX_NUM_QUEUES];
#pragma unroll
    for (int q = 0; q < EMURX_NUM_QUEUES; ++q) {
        const uint32_t incl = wave_incl_scan(v[q]);
        ex[q] = incl - v[q];
        if (lane == kWave - 1) s_w[wv][q] = incl;
    }
    __syncthreads();
    if (tid == 0) {  // queue bases of the queue-major concatenation
        uint32_t at = 0;
        for (int q = 0; q < EMURX_NUM_QUEUES; ++q) {
            s_base[q] = at;
            for (uint32_t w = 0; w < kW; ++w) at += s_w[w][q];
        }
        s_base[EMURX_NUM_QUEUES] = at;
    }
    __syncthreads();
    if (tid <= EMURX_NUM_QUEUES) qoff[tid] = s_base[tid];
#pragma unroll
    for (int q = 0; q < EMURX_NUM_QUEUES; ++q) {
        uint32_t before = 0;
        for (uint32_t w = 0; w < wv; ++w) before += s_w[w][q];
        ex[q] += before + s_base[q];
    }
    for (uint32_t t = t0; t < t1; ++t) {
        tile_row(tile_cnt, t, r);
        uint4* o = reinterpret_cast<uint4*>(seg_off + (size_t)t * 16);
        o[0] = make_uint4(ex[0], ex[1], ex[2], ex[3]);
        o[1] = make_uint4(ex[4], ex[5], ex[6], ex[7]);
        o[2] = make_uint4(ex[8], ex[9], ex[10], ex[11]);
        o[3] = make_uint4(ex[12], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < EMURX_NUM_QUEUES; ++q) ex[q] += r[q];
    }
    // fold the histogram shards (k_rx accumulates into them) and clear them
    if (tid < 2 * EMURX_HIST_BINS) {
        unsigned long long acc = 0;
        for (uint32_t s = 0; s < EMURX_HIST_SHARDS; ++s) {
            unsigned long long* p = hist + (size_t)s * 2 * EMURX_HIST_BINS + tid;
            acc += *p;
            *p = 0;
        }
        hist_out[tid] = acc;
    }
}

__global__ __launch_bounds__(kBlock) void k_qpack(const uint32_t* __restrict__ qlist, uint32_t qcap,
                                                  const uint32_t* __restrict__ tile_cnt,
                                                  const uint32_t* __restrict__ seg_off,
                                                  uint32_t* __restrict__ packed) {
    const uint32_t t = blockIdx.x, tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < EMURX_NUM_QUEUES; ++q) {
        const uint32_t c = tile_cnt[(size_t)t * 16 + q];
        if (tid < c)
            packed[seg_off[(size_t)t * 16 + q] + tid] =
                qlist[(size_t)q * qcap + (size_t)t * EMURX_QUEUE_TILE + tid];
    }
}

// ---- small batches: the whole ingest in ONE launch (emurx_ingest_submit's latency path) --------
// For a batch of at most kSmallTiles tiles whose every tile's messages fit kSmallLds bytes of
// LDS, one launch replaces the two H2D copies, the four kernels and the six D2H copies of the
// pipeline above: the kernel reads the control words and the messages straight from the slot's
// pinned host buffers and writes every result straight into the slot's pinned result buffers.
// Workgroup t owns descriptor slots [256 t, 256 t + 256):
//   1. the messages with slots in the tile (and those whose status word the tile writes) are
//      copied host -> LDS (16-byte loads, all in flight), each at an LDS offset congruent to
//      its buffer offset mod 16;
//   2. one lane per message walks it in LDS exactly as k_zmq_walk does (owner keys included),
//      keeping the descriptors of the tile's slots;
//   3. one lane per slot parses + classifies its frame from LDS (parse_flat / classify, as
//      k_rx's staged path), writes its record and descriptor, ranks it in its queue (ballots);
//      the tile's queue segments and counts go to device scratch with write-through stores;
//   4. the workgroup that arrives last (one agent-scope atomic per workgroup, after a release
//      fence; MI355X_MICROARCH.md's hand-off table, row 1) packs the queues in queue-major
//      order, writes qoff and the folded histogram, and clears the scratch for the next batch.
// The results are the pipeline's, slot for slot (tests/test_gpu_parity.py runs both paths).
constexpr uint32_t kSmallLds = EMURX_SMALL_LDS;        // staged message bytes per tile
constexpr uint32_t kSmallMsgs = EMURX_SMALL_MSGS;      // messages per batch
struct SmallArgs {
    const uint8_t* buf;          // pinned host: the slot's messages
    const uint32_t* ctl;         // pinned host: emurx_msg[nmsg], slot_base[nmsg + 1]
    uint32_t nmsg, n, nt;        // messages, descriptor slots, tiles
    emurx_dev_tables T;
    emurx_rec* rec;              // pinned host results
    emurx_desc* desc;
    uint32_t* qlist;
    uint32_t* stat;
    uint32_t* qoff;
    unsigned long long* hist_out;
    uint32_t* qseg;              // device scratch: [EMURX_SMALL_TILES][EMURX_NUM_QUEUES][256]
    uint32_t* tcnt;              // [EMURX_SMALL_TILES][16]
    unsigned long long* hist;    // [2 * EMURX_HIST_BINS], zero between batches
    uint32_t* ticket;            // zero between batches
    uint32_t* done;              // pinned host: the batch's sequence number, written last
    uint32_t seq;                // < 2^31: bit 31 of the completion word says "degraded"
    uint32_t spin_ticks;         // wall-clock ticks a workgroup waits for every tile to arrive
                                 // (0: none, the degraded pack at once: tests of that path)
    uint32_t trange[EMURX_SMALL_TILES];  // per tile: its first message | message count << 16
};

// EMURX_SMALL_STAMP=1 (diagnostic build, tools/lat_probe.py): the wall clock (100 MHz) at the
// phases of k_ingest_small, per workgroup, read back by emurx_debug_small_stamps
#ifndef EMURX_SMALL_STAMP
#define EMURX_SMALL_STAMP 0
#endif
#if EMURX_SMALL_STAMP
__device__ unsigned long long g_small_stamp[EMURX_SMALL_TILES * 10 + 16];  // + the last workgroup's pack phases
#define SSTAMP(k)                                                 \
    do {                                                          \
        if (tid == 0) g_small_stamp[t * 10 + (k)] = wall_clock64(); \
    } while (0)
#define PSTAMP(k)                                                                 \
    do {                                                                          \
        if (tid == 0) g_small_stamp[EMURX_SMALL_TILES * 10 + (k)] = wall_clock64(); \
    } while (0)
#else
#define PSTAMP(k) \
    do {          \
    } while (0)
#define SSTAMP(k) \
    do {          \
    } while (0)
#endif

__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // write-through (sc1)
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 4 bytes at an LDS byte index as a big-endian word (the staged message has 32 bytes of slack)
__device__ __forceinline__ uint32_t lds_be32(const uint32_t* w, uint32_t a) {
    return __builtin_bswap32(__builtin_amdgcn_alignbyte(w[(a >> 2) + 1], w[a >> 2], a & 3));
}

__global__ __launch_bounds__(kBlock) void k_ingest_small(const SmallArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t s_msg[kSmallLds / 4];
    __shared__ uint32_t s_vec[kSmallMsgs + 1];  // 16-byte vectors before each staged message (prefix)
    __shared__ uint2 s_desc[kBlock];            // the tile's descriptors: LDS frame offset, len | vport | key
    __shared__ uint32_t s_fpos[kBlock + 1];     // the walk: LDS byte of each slot's frame header (0: none)
    __shared__ uint32_t s_hoff[kBlock + 1];     // and its offset in the host buffer (+ a spare entry)
    __shared__ uint32_t s_wcnt[kWaves][16];
    __shared__ uint32_t s_hp[EMURX_HIST_BINS], s_hb[EMURX_HIST_BINS];
    __shared__ uint32_t s_last;
    __shared__ uint2 s_mk[kSmallMsgs];          // the tile's messages {offset, length}, read from the host once
    __shared__ uint32_t s_base[kSmallMsgs + 1];  // and their first descriptor slots
    const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid / kWave, t = blockIdx.x;
    // 1. this tile's messages (the host's trange: slots overlapping [s0, s1), or the message's
    //    status word is ours, tile min(base / 256, nt - 1); a contiguous range, base being
    //    monotonic): their control words in one bus round trip
    const uint32_t m0 = a.trange[t] & 0xffffu, nm = a.trange[t] >> 16;
    for (uint32_t k = tid; k < 2 * nm + 1; k += kBlock) {
        if (k < 2 * nm) reinterpret_cast<uint32_t*>(s_mk)[k] = a.ctl[2 * m0 + k];
        if (k <= nm) s_base[k] = a.ctl[2 * a.nmsg + m0 + k];
    }
    SSTAMP(0);
    const uint32_t s0 = t * kBlock;
    if (tid < 16) for (uint32_t w = 0; w < kWaves; ++w) s_wcnt[w][tid] = 0;
    if (tid < EMURX_HIST_BINS) { s_hp[tid] = 0; s_hb[tid] = 0; }
    s_fpos[tid] = 0;
    __syncthreads();
    SSTAMP(1);
    // staged layout: message k of the range at LDS byte s_lo[k] (+ its offset mod 16), its
    // vectors [s_vec[k], s_vec[k + 1]) of the range's flat vector list
    if (wv == 0) {
        uint32_t vb = 0, nv = 0;
        for (uint32_t c = 0; c < nm; c += kWave) {  // exclusive prefix over the range, 64 at a time
            const uint32_t k = c + lane;
            uint32_t v = 0;
            if (k < nm) {
                const uint2 mk = s_mk[k];
                v = mk.y ? (((mk.x & 15u) + mk.y + 15u) >> 4) + 2u : 0u;  // + 32 B of slack
            }
            uint32_t incl = v;
#pragma unroll
            for (uint32_t o = 1; o < kWave; o <<= 1) {
                const uint32_t up = (uint32_t)__shfl_up((int)incl, o);
                if (lane >= o) incl += up;
            }
            if (k < nm) s_vec[k] = vb + incl - v;
            vb += (uint32_t)__shfl((int)incl, kWave - 1);
            nv = vb;
        }
        if (lane == 0) s_vec[nm] = nv;
    }
    __syncthreads();
    SSTAMP(2);
    // host -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR round trip, every row of every
    // wave in flight before one wait): a wave per 64-vector row of the flat list, a lane's
    // message found by a binary search over s_vec.  The vectors past a message's end (its 32
    // bytes of slack) hold the host buffer's next bytes (the slot keeps 64 bytes of padding
    // past the last message): the parse reads no byte past a frame's length
    const uint32_t nvec = min(s_vec[nm], kSmallLds / 16);  // the host admits only batches that fit
    static_assert(kSmallLds % (16 * kWave) == 0, "whole 1 KiB DMA rows");
    for (uint32_t c = wv * kWave; c < nvec; c += kBlock) {
        const uint32_t v = min(c + lane, nvec - 1);  // the row's tail repeats its last vector
        uint32_t lo = 0, hi = nm;  // last k with s_vec[k] <= v
        while (hi - lo > 1) {
            const uint32_t md = (lo + hi) >> 1;
            if (s_vec[md] <= v) lo = md; else hi = md;
        }
        const uint32_t off = s_mk[lo].x;
        const uint8_t* src = a.buf + (off & ~15u) + 16u * (v - s_vec[lo]);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(src),
                                         (__attribute__((address_space(3))) void*)(reinterpret_cast<uint4*>(s_msg) + c),
                                         16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's rows landed
    __syncthreads();
    SSTAMP(3);
    // 2. the walk of OnRxStream (veth_zmq.go:277-320), in LDS.  A frame's step notes only its
    //    header position (LDS and host offset); owner keys and descriptors come after, one lane
    //    per slot.  A step continues while every check of OnRxStream passes, which with the
    //    message inside the LDS budget (< 64 KiB, so no 16-bit wrap of an accepted step) is
    //    magic && plen <= MAX && of + 4 + plen <= blen && a slot is left; the first failing
    //    step's error is then decided once with the checks in their Go order (go_error).
    //    Few messages (the latency case): a wave per message, 64 steps speculated per round
    //    (lane j guesses the header at P + j * s, s the stride of the frame at P) and the prefix
    //    whose guesses chain up accepted, so a message of equal-sized frames takes one round
    //    and any message at least one frame per round.  Many messages: one lane per message
    //    follows its chain serially, every message in parallel.
    auto go_error = [&](uint32_t L0, uint32_t blen, uint32_t of) {  // the failing step at of
        const uint32_t h4 = (of + 4) & 0xffff;
        const uint32_t hd = lds_be32(s_msg, L0 + min(of, blen));
        const uint32_t plen = hd & 0xffff, e = (of + 4 + plen) & 0xffff;
        return blen < h4                             ? (uint32_t)EMURX_MSG_PARSE_ERR
               : h4 < of                             ? (uint32_t)EMURX_MSG_PANIC
               : (hd & 0xff000000u) != 0xAA000000u   ? (uint32_t)EMURX_MSG_PARSE_ERR
               : blen < e                            ? (uint32_t)EMURX_MSG_PARSE_ERR
               : plen > EMURX_MAX_FRAME              ? (uint32_t)EMURX_MSG_PANIC
               : e < h4                              ? (uint32_t)EMURX_MSG_PANIC
                                                     : (uint32_t)EMURX_MSG_PANIC;  // no slot left
    };
    auto note = [&](uint32_t sl, uint32_t pos, uint32_t host) {  // a frame of slot sl; other tiles': the spare
        const uint32_t d = sl - s0, k = d < (uint32_t)kBlock ? d : (uint32_t)kBlock;
        s_fpos[k] = pos;
        s_hoff[k] = host;
    };
    if (nm <= 2 * kWaves) {
        for (uint32_t mi = wv; mi < nm; mi += kWaves) {  // wave-uniform
            const uint32_t m = m0 + mi;
            const uint2 mk = s_mk[mi];
            const uint32_t bm = s_base[mi], slots = s_base[mi + 1] - bm;
            const uint32_t L0 = s_vec[mi] * 16 + (mk.x & 15u), blen = mk.y;
            uint32_t f = 0, err = 0;
            if (blen < 4) {
                err = EMURX_MSG_PARSE_ERR;
            } else if ((lds_be32(s_msg, L0) >> 16) != EMURX_ZMQ_MAGIC) {
                err = EMURX_MSG_PARSE_ERR;
            } else {
                const uint32_t pkts = lds_be32(s_msg, L0) & 0xffff;
                uint32_t P = 4;
                while (f < pkts) {
                    const uint32_t st = 4 + (lds_be32(s_msg, L0 + min(P, blen)) & 0xffff);
                    const uint32_t g = P + lane * st;
                    const uint32_t hd = lds_be32(s_msg, L0 + min(g, blen));
                    const uint32_t plen = hd & 0xffff, e = g + 4 + plen;
                    const bool ok = (hd >> 24) == 0xAAu && plen <= EMURX_MAX_FRAME && e <= blen && f + lane < slots;
                    const uint64_t brk = __ballot(!(ok && e == g + st));
                    const uint32_t first = brk ? (uint32_t)__ffsll((long long)brk) - 1 : kWave;
                    const uint32_t fl = first < kWave ? first : kWave - 1;
                    const bool okf = first == kWave || __builtin_amdgcn_readlane((int)ok, (int)fl) != 0;
                    const uint32_t acc = min(first + (okf && first < kWave ? 1u : 0u), pkts - f);
                    if (lane < acc) note(bm + f + lane, L0 + g, mk.x + g);
                    if (!okf && f + first < pkts) {
                        err = go_error(L0, blen, (uint32_t)__builtin_amdgcn_readlane((int)g, (int)first));
                        f += acc;
                        break;
                    }
                    f += acc;
                    P = (uint32_t)__builtin_amdgcn_readlane((int)e, (int)fl);
                }
            }
            if (lane == 0 && min(bm / kBlock, a.nt - 1) == t) a.stat[m] = f | (err << 24);
        }
    } else {
        for (uint32_t mi = tid; mi < nm; mi += kBlock) {  // more messages than lanes: in turns
            const uint32_t m = m0 + mi;
            const uint2 mk = s_mk[mi];
            const uint32_t bm = s_base[mi], slots = s_base[mi + 1] - bm;
            const uint32_t L0 = s_vec[mi] * 16 + (mk.x & 15u);  // LDS byte of message byte 0
            const uint32_t blen = mk.y;
            uint32_t found = 0, err = 0;
            if (blen < 4) {
                err = EMURX_MSG_PARSE_ERR;
            } else {
                uint32_t header = lds_be32(s_msg, L0);
                if ((header >> 16) != EMURX_ZMQ_MAGIC) {
                    err = EMURX_MSG_PARSE_ERR;
                } else {
                    const uint32_t pkts = header & 0xffff;
                    uint32_t of = 4;
                    for (; found < pkts; ++found) {
                        header = lds_be32(s_msg, L0 + of);  // of <= blen: inside the staged message
                        const uint32_t plen = header & 0xffff, e = of + 4 + plen;
                        if (!((header >> 24) == 0xAAu && plen <= EMURX_MAX_FRAME && e <= blen && found < slots)) break;
                        note(bm + found, L0 + of, mk.x + of);
                        of = e;
                    }
                    if (found < pkts) err = go_error(L0, blen, of);
                }
            }
            if (min(bm / kBlock, a.nt - 1) == t) a.stat[m] = found | (err << 24);
        }
    }
    __syncthreads();
    SSTAMP(4);
    {  // one lane per slot of the tile: the frame's header word, owner key, descriptor (holes stay holes)
        const uint32_t sl = s0 + tid, fp = s_fpos[tid];
        uint2 dd = make_uint2(0, EMURX_DESC_HOLE << 24);
        if (fp) {  // a header is never at LDS byte 0 (it follows the message's own 4-byte header)
            const uint32_t hd = lds_be32(s_msg, fp), plen = hd & 0xffff, vport = (hd >> 16) & 0xff;
            uint32_t v0, v1;
            l2_vlans(plen, lds_be32(s_msg, fp + 16), lds_be32(s_msg, fp + 20), v0, v1);
            dd = make_uint2(fp + 4, plen | (vport << 16) | (emurx_owner_key(emurx_tk_hash(vport, v0, v1)) << 24));
        }
        s_desc[tid] = dd;
        if (sl < a.n)
            reinterpret_cast<uint2*>(a.desc)[sl] = fp ? make_uint2(s_hoff[tid] + 4, dd.y) : make_uint2(0, EMURX_DESC_HOLE << 24);
    }
    __syncthreads();
    SSTAMP(5);
    // 3. one lane per slot: parse + classify from LDS, record, queue rank, histogram
    const uint32_t sl = s0 + tid;
    const uint2 dd = s_desc[tid];
    const bool valid = sl < a.n && (dd.y >> 24) != EMURX_DESC_HOLE;
    const uint32_t len = dd.y & 0xffff, vport = (dd.y >> 16) & 0xff;
    Rec r;
    r.dlen = 0;
    if (valid) {
        LdsSrc src{reinterpret_cast<const uint8_t*>(s_msg), s_msg, dd.x};
        parse_flat(src, len, vport, a.T.cb_mask, r);
        classify(src, len, a.T, r);
    }
    SSTAMP(6);
    if (sl < a.n) {
        uint4* o = reinterpret_cast<uint4*>(a.rec + sl);
        o[0] = valid ? make_uint4(r.ns, r.cl, r.vlan0, r.vlan1) : make_uint4(EMURX_ID_NONE, EMURX_ID_NONE, 0, 0);
        o[1] = valid ? make_uint4(r.vport | (r.l3 << 16), r.l4 | (r.l7 << 16), r.l7len | (r.nh << 16) | (r.proto << 24),
                                  r.status | (r.flags << 8))
                     : make_uint4(0, 0, (uint32_t)EMURX_CB_NONE << 24, EMURX_ST_HOLE);
    }
    const uint32_t q = valid ? (r.status == EMURX_ST_OK ? r.proto : EMURX_Q_DROP) : 0xffu;
    if (valid) {
        const uint32_t bin = EMURX_HIST_BIN(r.status, r.proto);
        atomicAdd(&s_hp[bin], 1u);
        atomicAdd(&s_hb[bin], len);
    }
    uint32_t rank = 0;
    uint64_t left = __ballot(q != 0xffu);
    while (left) {
        const uint32_t lead = (uint32_t)__ffsll((long long)left) - 1;
        const uint32_t qq = (uint32_t)__builtin_amdgcn_readlane((int)q, (int)lead);
        const uint64_t m = __ballot(q == qq);
        if (q == qq) rank = mbcnt(m);
        if (lane == lead) s_wcnt[wv][qq] = (uint32_t)__popcll(m);
        left &= ~m;
    }
    __syncthreads();
    if (a.nt == 1) {
        // one tile: queues, qoff and the histogram straight from LDS into the host buffers, no
        // device scratch and no ticket; then the completion word after every store and a
        // system-scope release
        __shared__ uint32_t s_qo[EMURX_NUM_QUEUES];
        if (tid == 0) {
            uint32_t at = 0;
            for (uint32_t k = 0; k < EMURX_NUM_QUEUES; ++k) {
                s_qo[k] = at;
                a.qoff[k] = at;
                at += s_wcnt[0][k] + s_wcnt[1][k] + s_wcnt[2][k] + s_wcnt[3][k];
            }
            a.qoff[EMURX_NUM_QUEUES] = at;
        }
        __syncthreads();
        if (q != 0xffu) {
            uint32_t pos = s_qo[q] + rank;
            for (uint32_t w = 0; w < wv; ++w) pos += s_wcnt[w][q];
            a.qlist[pos] = sl;
        }
        if (tid < EMURX_HIST_BINS) {
            a.hist_out[2 * tid] = s_hp[tid];
            a.hist_out[2 * tid + 1] = s_hb[tid];
        }
        SSTAMP(7);
        SSTAMP(8);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __atomic_thread_fence(__ATOMIC_RELEASE);
            __hip_atomic_store(a.done, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        SSTAMP(9);
        return;
    }
    if (q != 0xffu) {
        uint32_t pos = rank;
        for (uint32_t w = 0; w < wv; ++w) pos += s_wcnt[w][q];
        st_agent(a.qseg + ((size_t)t * EMURX_NUM_QUEUES + q) * kBlock + pos, sl);
    }
    if (tid < 16) st_agent(a.tcnt + t * 16 + tid, s_wcnt[0][tid] + s_wcnt[1][tid] + s_wcnt[2][tid] + s_wcnt[3][tid]);
    if (tid < EMURX_HIST_BINS && s_hp[tid]) {
        atomicAdd(&a.hist[2 * tid], (unsigned long long)s_hp[tid]);
        atomicAdd(&a.hist[2 * tid + 1], (unsigned long long)s_hb[tid]);
    }
    // queue-major offsets of every (queue, tile) segment from the tiles' published counts:
    // s_off[q * nt + t], s_off[nseg] = the total; qoff written by the caller's choice
    __shared__ uint32_t s_off[EMURX_SMALL_TILES * EMURX_NUM_QUEUES + 1];
    const uint32_t nseg = a.nt * EMURX_NUM_QUEUES;  // segment k = (q = k / nt, t = k % nt)
    auto segment_offsets = [&](bool write_qoff) {
        // exclusive prefix, the whole workgroup: kPer consecutive segments per lane, their counts
        // loaded straight into registers (all in flight), then the lanes' sums by a wave scan and
        // the waves' totals (one lane walking 832 segments serially spent ~40 us of a 16K-frame
        // batch in dependent LDS reads)
        constexpr uint32_t kPer = (EMURX_SMALL_TILES * EMURX_NUM_QUEUES + kBlock - 1) / kBlock;  // segments per lane
        __shared__ uint32_t s_wsum[kWaves];
        uint32_t c4[kPer], sum = 0;
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) {
            const uint32_t k = kPer * tid + j;
            c4[j] = k < nseg ? ld_agent(a.tcnt + (k % a.nt) * 16 + k / a.nt) : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) sum += c4[j];
        const uint32_t incl = wave_incl_scan(sum);
        if (lane == kWave - 1) s_wsum[wv] = incl;
        __syncthreads();
        uint32_t at = incl - sum, total = 0;
        for (uint32_t w2 = 0; w2 < kWaves; ++w2) {
            at += w2 < wv ? s_wsum[w2] : 0u;
            total += s_wsum[w2];
        }
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) {
            const uint32_t k = kPer * tid + j;
            if (k < nseg) {
                s_off[k] = at;
                if (write_qoff && k % a.nt == 0) a.qoff[k / a.nt] = at;
            }
            at += c4[j];
        }
        if (tid == 0) {
            s_off[nseg] = total;
            if (write_qoff) a.qoff[EMURX_NUM_QUEUES] = total;
        }
        __syncthreads();
    };
    // 4. the tiles meet: every workgroup publishes its queue counts (write-through stores, then a
    // release and an arrival count), waits until every tile has arrived, derives the segment
    // offsets from all the counts and writes its own queue entries straight to their packed
    // places in the host's qlist (the PCIe writes spread over every workgroup: one workgroup
    // writing a 16K-frame batch's 64 KiB took 20 us at its outstanding-write limit).  The wait
    // is bounded in time (spin_ticks of the 100 MHz wall clock, the host's EMURX_INGEST_SPIN_US):
    // a workgroup that gives up (its tiles were not all resident, e.g. beside other kernels)
    // marks the batch degraded, and the last workgroup then packs the queues from the device
    // scratch every tile also wrote (qseg) as before.  The host caps the grid at the workgroups
    // the GPU holds at once (emurx_ingest_small_capacity), so the wait ends early but for
    // co-tenancy; its worst case is spin_ticks per batch.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ uint32_t s_direct;
    if (tid == 0) {
        __atomic_thread_fence(__ATOMIC_RELEASE);  // every wave's stores are behind the barrier
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        atomicAdd(a.ticket + 1, 1u);
        uint32_t seen = 0;
        const uint64_t t_0 = (uint64_t)wall_clock64();
        while (a.spin_ticks && (seen = ld_agent(a.ticket + 1)) < a.nt &&
               (uint64_t)wall_clock64() - t_0 < a.spin_ticks)
            __builtin_amdgcn_s_sleep(2);
        s_direct = a.spin_ticks && seen >= a.nt;
        if (!s_direct) atomicOr(a.ticket + 2, 1u);  // before this workgroup's ticket (release below)
    }
    __syncthreads();
    SSTAMP(7);
    if (s_direct) {
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        segment_offsets(t == 0);
        if (q != 0xffu) {
            uint32_t pos = s_off[q * a.nt + t] + rank;
            for (uint32_t w = 0; w < wv; ++w) pos += s_wcnt[w][q];
            a.qlist[pos] = sl;
        }
    }
    // the ticket: every wave's stores (host qlist entries included) have completed first; the
    // workgroup that takes the last ticket folds the histogram, packs the queues if the batch
    // was degraded, resets the scratch words and writes the completion word
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __atomic_thread_fence(__ATOMIC_RELEASE);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_last = atomicAdd(a.ticket, 1u) == a.nt - 1;
    }
    __syncthreads();
    if (!s_last) return;
    PSTAMP(0);
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    PSTAMP(1);
    const bool degraded = ld_agent(a.ticket + 2) != 0;
    if (degraded) segment_offsets(true);
    PSTAMP(2);
    PSTAMP(3);
    // The packed queues, entry p by lane p mod 256 in round p / 256: every store instruction
    // writes 1 KiB of contiguous host memory (PCIe writes of whole lines), and a lane issues
    // kPackBatch rounds' loads before their stores.  Its segment advances monotonically with p.
    // (Round 4 copied a segment per wave, 64 entries per step: a batch of one-queue traffic
    // took one device round trip per 64 entries, 21 us for 16 tiles)
    if (degraded) {
        constexpr uint32_t kPackBatch = 16;
        const uint32_t total = s_off[nseg];
        uint32_t k = 0;  // the segment of this lane's current entry
        if (tid < total) {  // its first: the last segment starting at or before it (empty ones skipped)
            uint32_t lo = 0, hi = nseg;
            while (hi - lo > 1) {
                const uint32_t md = (lo + hi) >> 1;
                if (s_off[md] <= tid) lo = md; else hi = md;
            }
            k = lo;
        }
        for (uint32_t p0 = 0; p0 < total; p0 += kPackBatch * kBlock) {
            uint32_t v[kPackBatch];
#pragma unroll
            for (uint32_t u = 0; u < kPackBatch; ++u) {
                const uint32_t p = p0 + u * kBlock + tid;
                v[u] = 0;
                if (p < total) {
                    while (s_off[k + 1] <= p) ++k;  // s_off[nseg] = total > p: stops inside
                    const uint32_t qq = k / a.nt, tt = k % a.nt;
                    v[u] = ld_agent(a.qseg + ((size_t)tt * EMURX_NUM_QUEUES + qq) * kBlock + (p - s_off[k]));
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < kPackBatch; ++u) {
                const uint32_t p = p0 + u * kBlock + tid;
                if (p < total) a.qlist[p] = v[u];
            }
        }
    }
    PSTAMP(4);
    if (tid < 2 * EMURX_HIST_BINS) {
        unsigned long long* hp = a.hist + tid;
        a.hist_out[tid] = __hip_atomic_load(hp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hp, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid < 3) __hip_atomic_store(a.ticket + tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    SSTAMP(8);
    // 5. the host's completion word, after every result store of this workgroup has completed
    // and a system-scope release (the other workgroups' results are ordered before their
    // tickets, which this one acquired): emurx_ingest_wait spins on it instead of waiting for
    // the kernel's end-of-dispatch signal
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    PSTAMP(5);
    if (tid == 0) {
        __atomic_thread_fence(__ATOMIC_RELEASE);
        __hip_atomic_store(a.done, a.seq | (degraded ? 0x80000000u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    SSTAMP(9);
}

}  // namespace emurx

int emurx_launch_zmq_walk(const uint8_t* buf, const uint32_t* ctl, uint32_t nmsg, emurx_desc* desc,
                          uint32_t* msg_stat, hipStream_t st, bool keys) {
    using namespace emurx;
    if (!nmsg) return 0;
    return EMURX_HIP_OK(emurx_launch(keys ? k_zmq_walk<true> : k_zmq_walk<false>, dim3((nmsg + kBlock - 1) / kBlock),
                                     dim3(kBlock), 0, st, buf, ctl, nmsg, desc, msg_stat))
               ? 0
               : -1;
}

int emurx_launch_ingest_small(const uint8_t* h_buf, const uint32_t* h_ctl, uint32_t nmsg, uint32_t n,
                              const emurx_dev_tables& T, emurx_rec* h_rec, emurx_desc* h_desc, uint32_t* h_qlist,
                              uint32_t* h_stat, uint32_t* h_qoff, uint64_t* h_hist, uint32_t* d_qseg, uint32_t* d_tcnt,
                              uint64_t* d_hist, uint32_t* d_ticket, uint32_t* h_done, uint32_t seq,
                              uint32_t spin_ticks, const uint32_t* trange, hipStream_t st) {
    using namespace emurx;
    const uint32_t nt = std::max<uint32_t>((n + kBlock - 1) / kBlock, 1);
    if (nt > EMURX_SMALL_TILES || nmsg > kSmallMsgs || (seq >> 31)) return -1;
    SmallArgs args{h_buf, h_ctl, nmsg, n, nt, T, h_rec, h_desc, h_qlist, h_stat, h_qoff,
                   reinterpret_cast<unsigned long long*>(h_hist), d_qseg, d_tcnt,
                   reinterpret_cast<unsigned long long*>(d_hist), d_ticket, h_done, seq, spin_ticks, {}};
    for (uint32_t t = 0; t < nt; ++t) args.trange[t] = trange[t];
    return EMURX_HIP_OK(emurx_launch(k_ingest_small, dim3(nt), dim3(kBlock), 0, st, args)) ? 0 : -1;
}

// Workgroups of k_ingest_small the device holds at once (occupancy x compute units): the
// one-launch path's tiles must all be resident for its direct queue pack.
uint32_t emurx_ingest_small_capacity(int device) {
    using namespace emurx;
    int per_cu = 0, cus = 0;
    if (!EMURX_HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_ingest_small, kBlock, 0)) ||
        !EMURX_HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device)))
        return 0;
    return (uint32_t)std::max(per_cu, 0) * (uint32_t)std::max(cus, 0);
}

#if EMURX_SMALL_STAMP
extern "C" int emurx_debug_small_stamps(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(emurx::g_small_stamp), sizeof(emurx::g_small_stamp)) == hipSuccess ? 0 : -1;
}
#endif

int emurx_launch_queue_pack(const uint32_t* qlist, uint32_t qcap, const uint32_t* tile_cnt, uint32_t n,
                            uint32_t* seg_off, uint32_t* packed, uint32_t* qoff, uint64_t* hist,
                            uint64_t* hist_out, hipStream_t st) {
    using namespace emurx;
    const uint32_t nt = (n + EMURX_QUEUE_TILE - 1) / EMURX_QUEUE_TILE;
    if (!EMURX_HIP_OK(emurx_launch(k_qscan, dim3(1), dim3(kScanLanes), 0, st, tile_cnt, nt, seg_off, qoff,
                                   reinterpret_cast<unsigned long long*>(hist),
                                   reinterpret_cast<unsigned long long*>(hist_out))))
        return -1;
    if (!nt) return 0;
    return EMURX_HIP_OK(emurx_launch(k_qpack, dim3(nt), dim3(kBlock), 0, st, qlist, qcap, tile_cnt, seg_off, packed))
               ? 0
               : -1;
}
