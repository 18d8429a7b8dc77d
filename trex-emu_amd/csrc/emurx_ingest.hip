// emurx_ingest.hip — device side of the batched ZMQ ingest (gfx950).
//
// The host path (emurx_ingest_* / emurx_rx_stream) hands the GPU many ZMQ messages per
// launch (src/emu/core/veth_zmq.go:8-22 wire format) and gets back records, packed
// per-callback queues and folded counters.  Around k_rx (emurx_kernels.hip) run:
//   k_zmq_walk  one lane per message: the offset walk of VethIFZmq.OnRxStream
//               (veth_zmq.go:277-320, uint16 running offset, abort on a header error) ->
//               descriptors in the message's slot range, each with its frame's owner key
//               (EMURX_DESC_KEYED: bytes 12..19 of the frame, loaded beside its header);
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
                header = ld_be32(s + of);
                if ((header & 0xff000000u) != 0xAA000000u) { err = EMURX_MSG_PARSE_ERR; break; }
                const uint32_t vport = (header >> 16) & 0xff, plen = header & 0xffff;
                const uint32_t e = (of + 4 + plen) & 0xffff;
                if (blen < e) { err = EMURX_MSG_PARSE_ERR; break; }
                if (plen > EMURX_MAX_FRAME) { err = EMURX_MSG_PANIC; break; }  // MbufPoll.Alloc
                if (e < h4) { err = EMURX_MSG_PANIC; break; }
                if (found >= slots) { err = EMURX_MSG_PANIC; break; }  // unreachable: slots bound the walk
                // the owner key from the CTunnelKey the parse will leave (l2_vlans: the frame's
                // bytes 12..19 and its length); bytes past the frame are masked by the length
                uint32_t v0, v1;
                l2_vlans(plen, ld_be32(s + h4 + 12), ld_be32(s + h4 + 16), v0, v1);
                const uint32_t key = emurx_owner_key(emurx_tk_hash(vport, v0, v1));
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

}  // namespace emurx

int emurx_launch_zmq_walk(const uint8_t* buf, const uint32_t* ctl, uint32_t nmsg, emurx_desc* desc,
                          uint32_t* msg_stat, hipStream_t st) {
    using namespace emurx;
    if (!nmsg) return 0;
    return EMURX_HIP_OK(emurx_launch(k_zmq_walk, dim3((nmsg + kBlock - 1) / kBlock), dim3(kBlock), 0, st, buf, ctl,
                                     nmsg, desc, msg_stat))
               ? 0
               : -1;
}

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
