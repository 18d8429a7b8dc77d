// emurx_tx.hip — tx-side checksum generation (gfx950), SURVEY.md §8f row 4.
//
// k_tx_csum: one frame per lane, in place.  The sums are the rx path's dword form (v_sad_u16
// over 16-byte loads, emurx_parse.h): every region is summed as it is in memory and the
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
__device__ __forceinline__ uint32_t byte_weight(uint32_t b, uintptr_t a) { return (a & 1) ? b << 8 : b; }

// tcpipChecksum(span, pcs) from T = the exact 16-bit-half sum of the span as the Go code sees
// it, pz = pcs is exactly zero, pm = pcs mod 0xffff
__device__ __forceinline__ uint32_t tx_value(uint32_t T, const uint8_t* span, uint32_t pm, bool pz) {
    if (T == 0 && pz) return 0xffffu;
    const uint32_t x = fold16(be_domain(T, (uint32_t)(uintptr_t)span) + pm);
    return (x == 0 || x == 0xffffu) ? 0u : (~x & 0xffffu);
}

__device__ __forceinline__ void put_be16(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

__global__ __launch_bounds__(kBlock) void k_tx_csum(uint8_t* __restrict__ frames,
                                                    const emurx_tx_desc* __restrict__ desc, uint32_t n,
                                                    uint8_t* __restrict__ status) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint4 d = gld16(desc + i);  // {off} {len | l3 << 16} {l4 | osize << 16} {ops | nh << 8}
    uint8_t* p = frames + d.x;
    const uint32_t len = d.y & 0xffff, l3 = d.y >> 16, l4 = d.z & 0xffff, osize = d.z >> 16;
    const uint32_t ops = d.w & 0xff, nhx = (d.w >> 8) & 0xff, kind = ops >> EMURX_TX_L4_SHIFT;
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
            const uint32_t ihl = gld1(p + l3) & 0xf;
            hlen = ihl > 5 ? ihl << 2 : 20;
            ok = l3 + hlen <= len;
        }
    }
    if (ok && v4l4) ok = l3 + 20 <= len;
    if (ok && v6l4) ok = l3 + 40 <= len;
    if (ok && kind) ok = l4 + field + 2 <= len;
    if (status) status[i] = ok ? EMURX_TX_OK : EMURX_TX_RANGE;
    if (!ok) return;

    // Go runs UpdateChecksum on the header first, then clears the L4 field, then reads the
    // pseudo header and the span: the L4 phase sees the new header checksum and a zero field
    // wherever those bytes fall.  Sums are taken from memory and corrected at those 4 bytes.
    const bool hdr = ops & EMURX_TX_IPV4_HDR;
    const uint32_t fo = l4 + field;
    uint32_t hcs = 0, lcs = 0;
    if (hdr) {  // the header with its own field cleared, the L4 field still as stored
        const uint32_t h0 = gld1(p + l3 + 10), h1 = gld1(p + l3 + 11);
        const uint32_t T = glb_sum(p + l3, hlen) - byte_weight(h0, (uintptr_t)(p + l3 + 10)) -
                           byte_weight(h1, (uintptr_t)(p + l3 + 11));
        hcs = tx_value(T, p + l3, 0, true);
    }
    if (kind) {
        // the byte the L4 phase reads at frame offset a (stored value b)
        auto seen = [&](uint32_t a, uint32_t b) -> uint32_t {
            if (a == fo || a == fo + 1) return 0;
            if (hdr && a == l3 + 10) return hcs >> 8;
            if (hdr && a == l3 + 11) return hcs & 0xff;
            return b;
        };
        auto vb = [&](uint32_t a) { return seen(a, gld1(p + a)); };
        // half-sum of [r0, r1) as stored -> as the L4 phase sees it
        auto fix = [&](uint32_t T, uint32_t r0, uint32_t r1) {
            const uint32_t c[4] = {fo, fo + 1, hdr ? l3 + 10 : fo, hdr ? l3 + 11 : fo};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t a = c[k];
                bool dup = false;
                for (int j = 0; j < k; ++j) dup |= c[j] == a;
                if (dup || a < r0 || a >= r1) continue;
                const uint32_t b = gld1(p + a);
                T += byte_weight(seen(a, b), (uintptr_t)(p + a)) - byte_weight(b, (uintptr_t)(p + a));
            }
            return T;
        };
        uint32_t pm = 0;
        bool pz = true;
        if (v4l4) {  // GetPhCs: src, dst, 0, proto, totlen - IHL*4 (uint16)
            const uint32_t Ta = fix(glb_sum(p + l3 + 12, 8), l3 + 12, l3 + 20);
            const uint32_t proto = vb(l3 + 9);
            const uint32_t tl = (vb(l3 + 2) << 8) | vb(l3 + 3);
            const uint32_t l = (tl - ((vb(l3) & 0xf) << 2)) & 0xffff;
            pm = be_domain(Ta, (uint32_t)(uintptr_t)(p + l3 + 12)) + proto + l;
            pz = Ta == 0 && proto == 0 && l == 0;
        } else if (v6l4) {  // GetPhCs(osize, nextH): src, dst, uint32(plen - osize), nextH
            const uint32_t Ta = fix(glb_sum(p + l3 + 8, 32), l3 + 8, l3 + 40);
            const uint32_t pl = (vb(l3 + 4) << 8) | vb(l3 + 5);
            const uint32_t l = (pl - osize) & 0xffff;
            const uint32_t nh = (ops & EMURX_TX_V6_NH) ? nhx : vb(l3 + 6);
            pm = be_domain(Ta, (uint32_t)(uintptr_t)(p + l3 + 8)) + l + nh;
            pz = Ta == 0 && l == 0 && nh == 0;
        }
        lcs = tx_value(fix(glb_sum(p + l4, len - l4), l4, len), p + l4, fold16(pm), pz);
    }
    if (ops & EMURX_TX_IPV4_HDR) put_be16(p + l3 + 10, hcs);
    if (kind) put_be16(p + fo, lcs);
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
