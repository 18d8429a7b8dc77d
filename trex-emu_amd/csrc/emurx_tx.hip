// emurx_tx.hip — tx-side checksum generation (gfx950), SURVEY.md §8f row 4.
//
// k_tx_csum: one frame per lane, in place, the wave's frames staged in LDS when they fit.  The
// sums are the rx path's dword form (v_sad_u16 over 16-byte loads, emurx_parse.h): every region is summed as it is in memory and the
// bytes Go would already have rewritten (the checksum fields) are corrected in the exact
// 16-bit-half sum, so nothing is written before the values are known and the only stores
// are the two bytes of each field.
//   IPv4Header.UpdateChecksum            ip4.go:132-136 (header of IHL*4 bytes)
//   PktChecksumTcpUdp + IPv4 GetPhCs     tcpip.go:38-40, ip4.go:49-58
//   FixL4ChecksumOffset + IPv6 GetPhCs   ip6.go:40-56, 127-134; PktChecksumTcpUdpV6 tcpip.go:34-36
//   ICMPv4Header.UpdateChecksum          icmp4.go:252-256
// Go's tcpipChecksum returns ^fold(sum): 0xffff only for an all-zero sum, 0 for any other sum
// that is 0 mod 0xffff; both cases are kept apart with an exact zero test.
#include <hip/hip_runtime.h>

#include "../../include/emu_rx.h"
#include "emurx_kernels.h"
#include "emurx_parse.h"

namespace emurx {

// exact 16-bit-half contribution of the byte at address a (weight 256^(a & 1))
__device__ __forceinline__ uint32_t byte_weight(uint32_t b, uint32_t a) { return (a & 1) ? b << 8 : b; }

// tcpipChecksum(span, pcs) from T = the exact 16-bit-half sum of the span as the Go code sees
// it (span_at: the span's address, for its parity), pz = pcs is exactly zero, pm = pcs mod 0xffff
__device__ __forceinline__ uint32_t tx_value(uint32_t T, uint32_t span_at, uint32_t pm, bool pz) {
    if (T == 0 && pz) return 0xffffu;
    const uint32_t x = fold16(be_domain(T, span_at) + pm);
    return (x == 0 || x == 0xffffu) ? 0u : (~x & 0xffffu);
}

__device__ __forceinline__ void put_be16(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

// the bytes of one frame: global memory (a lane's own frame, the wide path) or the wave's LDS
// slab (the wave's frames staged by LDS-DMA; an LDS byte index is the global address mod 16
// plus a multiple of 16, so every parity the sums depend on is the same)
// a wide wave's frame: its first bytes in the lane's LDS window (the rx window path's WinSrc:
// headers read there, the rest from global memory), the L4 span's sum taken beforehand by
// the wave's rows (coop_span_sum)
struct TxWinPre {
    WinSrc w;
    uint32_t s0, n, pre;  // sum(s0, n) == pre
    __device__ __forceinline__ uint32_t u8(uint32_t a) const { return w.u8(a); }
    __device__ __forceinline__ uint32_t sum(uint32_t a, uint32_t m) const { return a == s0 && m == n ? pre : w.sum(a, m); }
    __device__ __forceinline__ uint32_t at(uint32_t a) const { return w.at(a); }
};
struct TxLds {
    const uint8_t* b8;
    const uint32_t* b32;
    uint32_t base;  // LDS byte of frame byte 0
    __device__ __forceinline__ uint32_t u8(uint32_t a) const { return b8[base + a]; }
    __device__ __forceinline__ uint32_t sum(uint32_t a, uint32_t n) const { return dword_sum(b32, base + a, n); }
    __device__ __forceinline__ uint32_t at(uint32_t a) const { return base + a; }
};

// the two checksum values of one frame (hcs: IPv4 header, lcs: L4) as the Go send path
// computes them; false when a slice it takes leaves the frame
template <class S>
__device__ __forceinline__ bool tx_sums(const S& s, uint32_t len, uint32_t l3, uint32_t l4, uint32_t osize,
                                        uint32_t ops, uint32_t nhx, uint32_t& hcs, uint32_t& lcs, uint32_t& fo) {
    const uint32_t kind = ops >> EMURX_TX_L4_SHIFT;
    const uint32_t field = kind == EMURX_TX_L4_TCP4 || kind == EMURX_TX_L4_TCP6 ? 16
                         : kind == EMURX_TX_L4_UDP4 || kind == EMURX_TX_L4_UDP6 ? 6 : 2;
    const bool v4l4 = kind == EMURX_TX_L4_TCP4 || kind == EMURX_TX_L4_UDP4;
    const bool v6l4 = kind >= EMURX_TX_L4_TCP6 && kind <= EMURX_TX_L4_ICMP6;
    // every slice the Go code takes must lie inside the frame
    bool ok = kind <= EMURX_TX_L4_ICMP4;
    uint32_t hlen = 20;
    if (ok && (ops & EMURX_TX_IPV4_HDR)) {
        ok = l3 + 20 <= len;
        if (ok) {
            const uint32_t ihl = s.u8(l3) & 0xf;
            hlen = ihl > 5 ? ihl << 2 : 20;
            ok = l3 + hlen <= len;
        }
    }
    if (ok && v4l4) ok = l3 + 20 <= len;
    if (ok && v6l4) ok = l3 + 40 <= len;
    if (ok && kind) ok = l4 + field + 2 <= len;
    if (!ok) return false;

    // Go runs UpdateChecksum on the header first, then clears the L4 field, then reads the
    // pseudo header and the span: the L4 phase sees the new header checksum and a zero field
    // wherever those bytes fall.  Sums are taken as stored and corrected at those 4 bytes.
    const bool hdr = ops & EMURX_TX_IPV4_HDR;
    fo = l4 + field;
    hcs = 0;
    lcs = 0;
    if (hdr) {  // the header with its own field cleared, the L4 field still as stored
        const uint32_t h0 = s.u8(l3 + 10), h1 = s.u8(l3 + 11);
        const uint32_t T = s.sum(l3, hlen) - byte_weight(h0, s.at(l3 + 10)) - byte_weight(h1, s.at(l3 + 11));
        hcs = tx_value(T, s.at(l3), 0, true);
    }
    if (kind) {
        // the byte the L4 phase reads at frame offset a (stored value b)
        auto seen = [&](uint32_t a, uint32_t b) -> uint32_t {
            if (a == fo || a == fo + 1) return 0;
            if (hdr && a == l3 + 10) return hcs >> 8;
            if (hdr && a == l3 + 11) return hcs & 0xff;
            return b;
        };
        auto vb = [&](uint32_t a) { return seen(a, s.u8(a)); };
        // half-sum of [r0, r1) as stored -> as the L4 phase sees it
        auto fix = [&](uint32_t T, uint32_t r0, uint32_t r1) {
            const uint32_t c[4] = {fo, fo + 1, hdr ? l3 + 10 : fo, hdr ? l3 + 11 : fo};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t a = c[k];
                bool dup = false;
                for (int j = 0; j < k; ++j) dup |= c[j] == a;
                if (dup || a < r0 || a >= r1) continue;
                const uint32_t b = s.u8(a);
                T += byte_weight(seen(a, b), s.at(a)) - byte_weight(b, s.at(a));
            }
            return T;
        };
        uint32_t pm = 0;
        bool pz = true;
        if (v4l4) {  // GetPhCs: src, dst, 0, proto, totlen - IHL*4 (uint16)
            const uint32_t Ta = fix(s.sum(l3 + 12, 8), l3 + 12, l3 + 20);
            const uint32_t proto = vb(l3 + 9);
            const uint32_t tl = (vb(l3 + 2) << 8) | vb(l3 + 3);
            const uint32_t l = (tl - ((vb(l3) & 0xf) << 2)) & 0xffff;
            pm = be_domain(Ta, s.at(l3 + 12)) + proto + l;
            pz = Ta == 0 && proto == 0 && l == 0;
        } else if (v6l4) {  // GetPhCs(osize, nextH): src, dst, uint32(plen - osize), nextH
            const uint32_t Ta = fix(s.sum(l3 + 8, 32), l3 + 8, l3 + 40);
            const uint32_t pl = (vb(l3 + 4) << 8) | vb(l3 + 5);
            const uint32_t l = (pl - osize) & 0xffff;
            const uint32_t nh = (ops & EMURX_TX_V6_NH) ? nhx : vb(l3 + 6);
            pm = be_domain(Ta, s.at(l3 + 8)) + l + nh;
            pz = Ta == 0 && l == 0 && nh == 0;
        }
        lcs = tx_value(fix(s.sum(l4, len - l4), l4, len), s.at(l4), fold16(pm), pz);
    }
    return true;
}

// One frame per lane.  A wave whose frames' byte range fits its 6 KiB LDS slab copies the
// range in by LDS-DMA (1 KiB rows, coalesced, as k_rx stages) and sums from LDS; a wider wave
// stages a header window per lane and sums its L4 spans cooperatively (coop_span_sum, the rx
// window path's rows).  The only stores are the checksum fields.
constexpr uint32_t kTxSlab = 6144;
__global__ __launch_bounds__(kBlock) void k_tx_csum(uint8_t* __restrict__ frames,
                                                    const emurx_tx_desc* __restrict__ desc, uint32_t n,
                                                    uint8_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint32_t s_slab[kWaves][(kTxSlab + 32) / 4];
    __shared__ uint32_t s_wsum[kWaves][kWave];  // coop_span_sum's per-span sums
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x, lane = lane_id(), wv = threadIdx.x / kWave;
    const bool live = i < n;
    const uint4 d = live ? gld16(desc + i) : make_uint4(0, 0, 0, 0);  // {off} {len | l3} {l4 | osize} {ops | nh}
    const uint32_t len = d.y & 0xffff, l3 = d.y >> 16, l4 = d.z & 0xffff, osize = d.z >> 16;
    const uint32_t ops = d.w & 0xff, nhx = (d.w >> 8) & 0xff;
    const uint32_t lo = wave_min_u32(live ? d.x : 0xffffffffu);
    const uint32_t hi = wave_max_u32(live ? d.x + len : 0u);
    // the staged rows start at the 16-byte boundary of the ABSOLUTE address (d_frames need not
    // be 16-aligned): a frame byte's slab index is then its address mod 16 plus a multiple of 16
    // (built from the absolute address: lo - skew in frame offsets would wrap below d_frames
    // when the wave's first frame sits within its first 16 bytes)
    const uintptr_t abs_lo = (uintptr_t)frames + lo;
    const uint32_t skew = (uint32_t)(abs_lo & 15u);  // lo's offset in its aligned vector
    const uint32_t nvec = hi > lo ? (hi - lo + skew + 15) >> 4 : 0;
    const bool staged = nvec > 0 && nvec <= kTxSlab / 16;  // wave-uniform
    uint32_t hcs = 0, lcs = 0, fo = 0;
    bool ok;
    if (staged) {
        static_assert(kTxSlab % (16 * kWave) == 0, "whole 1 KiB DMA rows");
        const uint4* src = reinterpret_cast<const uint4*>(abs_lo & ~(uintptr_t)15);  // 16-byte aligned
        uint4* dst = reinterpret_cast<uint4*>(s_slab[wv]);
#pragma unroll
        for (uint32_t k = 0; k < kTxSlab / 16 / kWave; ++k)
            if (k * kWave < nvec)
                __builtin_amdgcn_global_load_lds(src + min(lane + k * kWave, nvec - 1),
                                                 (__attribute__((address_space(3))) void*)(dst + k * kWave), 16, 0, 0);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the wave's rows landed
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const TxLds s{reinterpret_cast<const uint8_t*>(s_slab[wv]), s_slab[wv], d.x - lo + skew};
        ok = live && tx_sums(s, len, l3, l4, osize, ops, nhx, hcs, lcs, fo);
    } else {
        // frames too wide to stage whole (long L4 spans): each lane's first kTxWinVec vectors in
        // the slab (vector k of lane l at byte k * 1 KiB + l * 16, one DMA row per k), the L4
        // spans summed cooperatively (16 lanes per span, 1 KiB per row round)
        constexpr uint32_t kTxWinVec = kTxSlab / 16 / kWave;
        const uintptr_t fa = (uintptr_t)(frames + d.x);
        const uint4* src = reinterpret_cast<const uint4*>(fa & ~(uintptr_t)15);
        const uint32_t head = (uint32_t)(fa & 15), nv = live && len ? (head + len + 15) >> 4 : 0u;
        uint4* dst = reinterpret_cast<uint4*>(s_slab[wv]);
#pragma unroll
        for (uint32_t k = 0; k < kTxWinVec; ++k)
            if (k < nv)
                __builtin_amdgcn_global_load_lds(src + k, (__attribute__((address_space(3))) void*)(dst + k * kWave), 16, 0,
                                                 0);
        const bool want = live && (ops >> EMURX_TX_L4_SHIFT) != 0 && l4 < len;
        const uint32_t pre = coop_span_sum(frames + d.x + l4, want ? len - l4 : 0u, want, s_wsum[wv]);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the windows landed
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const WinSrc w{reinterpret_cast<const uint8_t*>(s_slab[wv]), s_slab[wv], lane * 16, head,
                       min(kTxWinVec * 16 - head, len), frames + d.x};
        ok = live && tx_sums(TxWinPre{w, l4, want ? len - l4 : 0u, pre}, len, l3, l4, osize, ops, nhx, hcs, lcs, fo);
    }
    if (!live) return;
    if (status) status[i] = ok ? EMURX_TX_OK : EMURX_TX_RANGE;
    if (!ok) return;
    uint8_t* p = frames + d.x;
    if (ops & EMURX_TX_IPV4_HDR) put_be16(p + l3 + 10, hcs);
    if (ops >> EMURX_TX_L4_SHIFT) put_be16(p + fo, lcs);
}

}  // namespace emurx

int emurx_launch_tx_csum(uint8_t* frames, const emurx_tx_desc* desc, uint32_t n, uint8_t* status,
                         hipStream_t st) {
    using namespace emurx;
    if (!n) return 0;
    return EMURX_HIP_OK(emurx_launch(k_tx_csum, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, frames, desc, n,
                                     status))
               ? 0
               : -1;
}
