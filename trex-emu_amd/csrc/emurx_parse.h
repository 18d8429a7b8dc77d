// emurx_parse.h — device-side restatement of the TRex-EMU receive path (gfx950).
//
// One frame per lane.  Byte sources (wave LDS slab or global memory), the RFC 1071 sum in
// dword form, ParsePacket / parsePacketL4 / processIpv6Options (src/emu/core/parser.go:
// 583-959) and the per-callback Namespace / Client rules of src/emu/plugins/* as device
// functions; the kernels that drive them are in emurx_kernels.hip.  The CPU oracle
// (oracle/emurx_oracle.c) is the line-by-line twin the parity tests compare with.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/emu_rx.h"
#include "emurx_kernels.h"
#include "emurx_tables.h"

namespace emurx {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWaves = kBlock / kWave;
constexpr uint32_t kStage = 8192;  // LDS bytes staged per wave (64 frames)

#ifndef EMURX_ABL
#define EMURX_ABL 0  // experiment-only stage ablation (tools/ablate.sh); 0 in every real build
#endif

// ---------------------------------------------------------------------------------------
// wave helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o);
        uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

// ---------------------------------------------------------------------------------------
// RFC 1071 sum, restated for dword loads.
// Go (layers/tcpip.go:76-94) adds big-endian byte pairs of the span into a uint32 and
// folds; the span is valid iff the folded value is 0xffff.  Modulo 0xffff, 2^16 == 1 and
// 256*256 == 1, so a little-endian dword at an aligned address contributes each byte with
// weight 256^(address & 1).  Summing masked aligned dwords therefore gives
//   S_go == T * 256^(1 - (span_start & 1))   (mod 0xffff)
// and S_go + pseudo == 0 (mod 0xffff) with a non-zero total <=> Go's check passes.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t fold16(uint64_t s) {
    uint32_t x = (uint32_t)(s & 0xffff) + (uint32_t)((s >> 16) & 0xffff) +
                 (uint32_t)((s >> 32) & 0xffff) + (uint32_t)(s >> 48);
    x = (x & 0xffff) + (x >> 16);
    x = (x & 0xffff) + (x >> 16);
    return x;  // <= 0xffff, == s mod 0xffff (0xffff stands for 0)
}
__device__ __forceinline__ uint32_t byte_mask(int sb, int eb) {  // bytes [sb, eb) of a dword
    uint32_t lo = eb >= 4 ? 0xffffffffu : ((1u << (8 * max(eb, 0))) - 1u);
    uint32_t hi = sb <= 0 ? 0xffffffffu : (sb >= 4 ? 0u : (0xffffffffu << (8 * sb)));
    return lo & hi;
}
// true iff tcpipChecksum(span, pcs) == 0
__device__ __forceinline__ bool csum_ok(uint64_t sum, bool all_zero, uint32_t a_start, uint32_t pcs) {
    uint32_t t = fold16(sum);
    if ((a_start & 1u) == 0) t = ((t << 8) | (t >> 8)) & 0xffffu;
    uint32_t x = t + pcs;
    x = (x & 0xffff) + (x >> 16);
    x = (x & 0xffff) + (x >> 16);
    x = (x & 0xffff) + (x >> 16);
    return (x == 0xffffu || x == 0u) && !(all_zero && pcs == 0);
}

// ---------------------------------------------------------------------------------------
// byte sources: the wave's LDS slab (fast path) or global memory (frames that do not fit)
// ---------------------------------------------------------------------------------------
struct LdsSrc {
    const uint8_t* b8;    // block LDS
    const uint32_t* b32;  // same array, dword view
    uint32_t base;        // LDS byte index of frame byte 0 (== global address mod 16)
    __device__ __forceinline__ uint32_t u8(uint32_t i) const { return b8[base + i]; }
    __device__ __forceinline__ bool csum(uint32_t s, uint32_t n, uint32_t pcs) const {
        if (EMURX_ABL & 1) return true;
        uint32_t a = base + s, e = a + n;
        uint32_t k0 = a >> 2, k1 = (e + 3) >> 2;
        uint64_t sum = 0;
        uint32_t orv = 0;
        for (uint32_t k = k0; k < k1; ++k) {
            uint32_t w = b32[k];
            int rel = (int)(k << 2);
            w &= byte_mask((int)a - rel, (int)e - rel);
            sum += w;
            orv |= w;
        }
        return csum_ok(sum, orv == 0, a, pcs);
    }
};
struct GlbSrc {
    const uint8_t* f;  // frame byte 0 (global)
    __device__ __forceinline__ uint32_t u8(uint32_t i) const { return f[i]; }
    __device__ __forceinline__ bool csum(uint32_t s, uint32_t n, uint32_t pcs) const {
        uintptr_t a = (uintptr_t)(f + s), e = a + n;
        const uint32_t* w32 = (const uint32_t*)(a & ~(uintptr_t)3);
        uint32_t nw = (uint32_t)(((e + 3) & ~(uintptr_t)3) - (a & ~(uintptr_t)3)) >> 2;
        uint64_t sum = 0;
        uint32_t orv = 0;
        int sa = (int)(a & 3);
        int ee = (int)(e - (a & ~(uintptr_t)3));
        for (uint32_t k = 0; k < nw; ++k) {
            uint32_t w = w32[k];
            int rel = (int)(k << 2);
            w &= byte_mask(sa - rel, ee - rel);
            sum += w;
            orv |= w;
        }
        return csum_ok(sum, orv == 0, (uint32_t)a, pcs);
    }
};

template <class S>
__device__ __forceinline__ uint32_t be16(const S& s, uint32_t i) { return (s.u8(i) << 8) | s.u8(i + 1); }
template <class S>
__device__ __forceinline__ uint32_t be32(const S& s, uint32_t i) {
    return (s.u8(i) << 24) | (s.u8(i + 1) << 16) | (s.u8(i + 2) << 8) | s.u8(i + 3);
}
template <class S>  // bytes i..i+3 as a little-endian word (the table key encoding)
__device__ __forceinline__ uint32_t le32(const S& s, uint32_t i) {
    return s.u8(i) | (s.u8(i + 1) << 8) | (s.u8(i + 2) << 16) | (s.u8(i + 3) << 24);
}

// ---------------------------------------------------------------------------------------
// parse state == ParserPacketState + CTunnelData + outcome
// ---------------------------------------------------------------------------------------
struct Rec {
    uint32_t ns, cl, vlan0, vlan1;
    uint32_t vport, l3, l4, l7, l7len;
    uint32_t nh, proto, status, flags;
};

__device__ __forceinline__ void invoke(Rec& r, uint32_t cb, uint32_t cb_mask) {
    r.proto = cb;
    if (cb_mask & (1u << cb)) r.status = EMURX_ST_OK;
    else if (cb == EMURX_CB_EAPOL) r.status = EMURX_ST_PANIC_NIL_EAPOL;  // nil ParserCb :789
    else r.status = EMURX_ST_NOT_SUPPORTED;                              // parserNotSupported
}
__device__ __forceinline__ void fail(Rec& r, uint32_t st) { r.status = st; r.proto = EMURX_CB_NONE; }

__device__ __forceinline__ bool span_ok(uint32_t l4, uint32_t l4len) {
    return ((l4 + l4len) & 0xffffu) >= l4;  // Go slice p[L4:L4+l4len] with uint16 end
}

// processIpv6Options parser.go:726-746; false on Go's out-of-range p[i+1]
template <class S>
__device__ bool ipv6_options(const S& s, uint32_t p0, int size, uint32_t& flags) {
    int i = 0;
    uint32_t nh = s.u8(p0);
    for (;;) {
        if (nh == 0) {
            i++;
        } else if (nh == 5) {
            flags |= EMURX_FLAG_RTALERT;
            return true;
        } else {
            if (i + 1 >= size) return false;
            i = i + 2 + (int)s.u8(p0 + i + 1);
        }
        if (i > size - 1) return true;
        nh = s.u8(p0 + i);
    }
}

// Parser.parsePacketL4 parser.go:583-724
template <class S>
__device__ void parse_l4(const S& s, uint32_t len, Rec& r, uint32_t nextHdr, uint32_t pcs,
                         uint32_t l4len, bool v6, uint32_t cb_mask) {
    r.nh = nextHdr;
    const uint32_t L4 = r.l4;
    switch (nextHdr) {
    case 1:  // ICMPv4
        if (len < ((L4 + 8) & 0xffff)) { fail(r, EMURX_ST_ICMPV4_TOO_SHORT); return; }
        if (!span_ok(L4, l4len)) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
        if (!s.csum(L4, l4len, 0)) { fail(r, EMURX_ST_ICMPV4_CS); return; }
        r.l7 = (L4 + 8) & 0xffff;
        invoke(r, EMURX_CB_ICMP, cb_mask);
        return;
    case 2:  // IGMP (no checksum in the parser)
        if (len < ((L4 + 8) & 0xffff)) { fail(r, EMURX_ST_ICMPV4_TOO_SHORT); return; }
        invoke(r, EMURX_CB_IGMP, cb_mask);
        return;
    case 6: {  // TCP
        if (l4len < 20) { fail(r, EMURX_ST_TCP_TOO_SHORT); return; }
        if (((L4 + 12) & 0xffff) >= len) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
        uint32_t tcplen = (s.u8((L4 + 12) & 0xffff) >> 4) << 2;
        if (l4len < tcplen) { fail(r, EMURX_ST_TCP_TOO_SHORT); return; }
        r.l7 = (L4 + tcplen) & 0xffff;
        r.l7len = (l4len - tcplen) & 0xffff;
        if (!span_ok(L4, l4len)) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
        if (!s.csum(L4, l4len, pcs)) { fail(r, EMURX_ST_TCP_CS); return; }
        invoke(r, EMURX_CB_TCP, cb_mask);
        return;
    }
    case 17: {  // UDP
        if (len < ((L4 + 8) & 0xffff)) { fail(r, EMURX_ST_UDP_TOO_SHORT); return; }
        r.l7len = (l4len - 8) & 0xffff;
        if (be16(s, L4 + 6) > 0) {
            if (!span_ok(L4, l4len)) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
            if (!s.csum(L4, l4len, pcs)) { fail(r, EMURX_ST_UDP_CS); return; }
        }
        r.l7 = (L4 + 8) & 0xffff;
        uint32_t src = be16(s, L4), dst = be16(s, L4 + 2);
        uint32_t cb = EMURX_CB_UDP;
        if (dst == 5353) cb = EMURX_CB_MDNS;
        else if (v6) { if (src == 547 && dst == 546) cb = EMURX_CB_DHCPV6; }
        else if (src == 67 && dst == 68) cb = EMURX_CB_DHCP;
        else if (dst == 67 && (src == 67 || src == 68)) cb = EMURX_CB_DHCPSRV;
        invoke(r, cb, cb_mask);
        return;
    }
    case 58: {  // ICMPv6
        if (len < ((L4 + 4) & 0xffff)) { fail(r, EMURX_ST_ICMPV6_TOO_SHORT); return; }
        if (!span_ok(L4, l4len)) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
        if (!s.csum(L4, l4len, pcs)) { fail(r, EMURX_ST_ICMPV6_CS); return; }
        uint32_t t = s.u8(L4);
        bool okt = (t >= 1 && t <= 4) || (t >= 128 && t <= 136);
        if (okt) invoke(r, EMURX_CB_ICMPV6, cb_mask);
        else fail(r, EMURX_ST_ICMPV6_UNSUPPORTED);
        return;
    }
    default:
        fail(r, EMURX_ST_L4_UNSUPPORTED);
        return;
    }
}

// pseudo-header partial sums: IPv4Header.GetPhCs ip4.go:49-58, IPv6Header.GetPhCs ip6.go:126-134
template <class S>
__device__ __forceinline__ uint32_t pair_sum(const S& s, uint32_t p, int n) {
    uint32_t c = 0;
    for (int i = 0; i < n; i += 2) c += be16(s, p + i);
    return c;
}

// Parser.ParsePacket parser.go:756-959
template <class S>
__device__ void parse_packet(const S& s, uint32_t len, uint32_t vport, uint32_t cb_mask, Rec& r) {
    r.ns = EMURX_ID_NONE; r.cl = EMURX_ID_NONE;
    r.vlan0 = 0; r.vlan1 = 0; r.vport = vport;
    r.l3 = r.l4 = r.l7 = r.l7len = 0;
    r.nh = 0; r.proto = EMURX_CB_NONE; r.status = EMURX_ST_OK; r.flags = 0;
    if (len < 14) { fail(r, EMURX_ST_PACKET_TOO_SHORT); return; }
    uint32_t offset = 14;
    uint32_t nextHdr = be16(s, 12);
    int vlanIndex = 0;
    for (;;) {
        if (nextHdr == 0x8100 || nextHdr == 0x88A8) {
            if (len < offset + 4) { fail(r, EMURX_ST_DOT1Q_TOO_SHORT); return; }
            if (vlanIndex > 1) { fail(r, EMURX_ST_TOO_MANY_DOT1Q); return; }
            uint32_t val = be32(s, offset - 2) & 0xffff0fffu;
            if (vlanIndex == 0) r.vlan0 = val; else r.vlan1 = val;
            vlanIndex++;
            nextHdr = be16(s, offset + 2);
            if (nextHdr == 0x8863 || nextHdr == 0x8864) { invoke(r, EMURX_CB_PPP, cb_mask); return; }
            offset += 4;
            continue;
        }
        if (nextHdr == 0x0800) {  // IPv4
            r.l3 = offset;
            if (len < offset + 20) { fail(r, EMURX_ST_IPV4_TOO_SHORT); return; }
            uint32_t b0 = s.u8(offset);
            if ((b0 >> 4) != 4) { fail(r, EMURX_ST_IPV4_HDR_TOO_SHORT); return; }
            uint32_t frag = be16(s, offset + 6);
            if ((frag & 0x1fff) != 0 || (frag & 0x2000) != 0) { fail(r, EMURX_ST_IPV4_FRAGMENT); return; }
            uint32_t hdr = (b0 & 0xf) << 2;
            if (hdr < 20) { fail(r, EMURX_ST_IPV4_HDR_TOO_SHORT); return; }
            if (len < offset + hdr) { fail(r, EMURX_ST_IPV4_HDR_TOO_SHORT); return; }
            uint32_t totlen = be16(s, offset + 2);
            if (len < ((offset + totlen) & 0xffff)) { fail(r, EMURX_ST_IPV4_TOO_SHORT); return; }
            if (!s.csum(offset, hdr, 0)) { fail(r, EMURX_ST_IPV4_CS); return; }
            uint32_t l4len = (totlen - hdr) & 0xffff;
            r.l4 = offset + hdr;
            uint32_t proto = s.u8(offset + 9);
            uint32_t pcs = pair_sum(s, offset + 12, 8) + proto + l4len;  // src, dst, 0|proto, len
            parse_l4(s, len, r, proto, pcs, l4len, false, cb_mask);
            return;
        }
        if (nextHdr == 0x86DD) {  // IPv6
            r.l3 = offset;
            if (len < offset + 40) { fail(r, EMURX_ST_IPV6_TOO_SHORT); return; }
            if ((s.u8(offset) >> 4) != 6) { fail(r, EMURX_ST_IPV6_TOO_SHORT); return; }
            uint32_t plen = be16(s, offset + 4);
            if (len < ((offset + 40 + plen) & 0xffff)) { fail(r, EMURX_ST_IPV6_TOO_SHORT); return; }
            if (s.u8(offset + 7) == 0) { fail(r, EMURX_ST_IPV6_HOPLIMIT); return; }
            uint32_t l4 = offset + 40, l4len = plen, osize = 0;
            uint32_t nh = s.u8(offset + 6);
            for (;;) {
                bool ext = nh == 0 || nh == 60 || nh == 43 || nh == 51 || nh == 50 || nh == 135 ||
                           nh == 139 || nh == 140;
                if (!ext) break;
                if (l4len < 8) { fail(r, EMURX_ST_IPV6_TOO_SHORT); return; }
                if (l4 + 2 > len) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
                uint32_t hl = (s.u8(l4 + 1) << 3) + 8;
                if (l4len < hl) { fail(r, EMURX_ST_IPV6_TOO_SHORT); return; }
                if (l4 + hl > len) { fail(r, EMURX_ST_PANIC_L4LEN); return; }
                uint32_t nnh = s.u8(l4);
                if (!ipv6_options(s, l4 + 2, (int)hl - 2, r.flags)) { fail(r, EMURX_ST_PANIC_IPV6_OPT); return; }
                nh = nnh;
                l4len -= hl;
                osize += hl;
                l4 += hl;
            }
            if (nh == 44) { fail(r, EMURX_ST_IPV6_FRAGMENT); return; }
            if (nh == 194) { fail(r, EMURX_ST_IPV6_JUMBO); return; }
            if (nh == 59) { fail(r, EMURX_ST_IPV6_EMPTY); return; }
            r.l4 = l4;
            uint32_t pcs = pair_sum(s, offset + 8, 32) + ((plen - osize) & 0xffff) + nh;
            parse_l4(s, len, r, nh, pcs, l4len, true, cb_mask);
            return;
        }
        if (nextHdr == 0x888E) {  // EAPOL
            if (len < offset + 4) { fail(r, EMURX_ST_EAPOL_TOO_SHORT); return; }
            r.l3 = offset;
            invoke(r, EMURX_CB_EAPOL, cb_mask);
            return;
        }
        if (nextHdr == 0x0806) {  // ARP, ARPHeaderSize 28
            if (len < offset + 28) { fail(r, EMURX_ST_ARP_TOO_SHORT); return; }
            r.l3 = offset;
            invoke(r, EMURX_CB_ARP, cb_mask);
            return;
        }
        if (nextHdr == 0x8863 || nextHdr == 0x8864) { invoke(r, EMURX_CB_PPP, cb_mask); return; }
        fail(r, EMURX_ST_L3_UNSUPPORTED);
        return;
    }
}

// ---------------------------------------------------------------------------------------
// Namespace / Client lookups (GetNs thread_ctx.go:777-784, CLookupBy* ns_ctx.go:262-329)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint4 ld4(const uint32_t* p) { return *reinterpret_cast<const uint4*>(p); }

// ns slot: {vport | ns_plugins << 16, vlan0, vlan1, ns_id} -> (ns_id, ns plugin mask)
__device__ uint2 probe_ns(const emurx_dev_tables& T, uint32_t w0, uint32_t w1, uint32_t w2) {
    uint32_t i = emurx_ns_hash(w0, w1, w2) & T.ns_mask;
    for (uint32_t k = 0; k <= T.ns_mask; ++k, i = (i + 1) & T.ns_mask) {
        uint4 e = ld4(T.ns_tab + 4 * i);
        if (e.w == EMURX_EMPTY) break;
        if ((e.x & 0xffffu) == w0 && e.y == w1 && e.z == w2) return make_uint2(e.w, e.x >> 16);
    }
    return make_uint2(EMURX_ID_NONE, 0);
}
// mac slot: {ns_id, mac[0..3], mac[4..5] | client_plugins << 16, client_id}
__device__ uint2 probe_mac(const emurx_dev_tables& T, uint32_t ns, uint32_t lo, uint32_t hi) {
    if (lo == 0 && hi == 0) return make_uint2(EMURX_ID_NONE, 0);  // MACKey.IsZero
    uint32_t i = emurx_mac_hash(ns, lo, hi) & T.mac_mask;
    for (uint32_t k = 0; k <= T.mac_mask; ++k, i = (i + 1) & T.mac_mask) {
        uint4 e = ld4(T.mac_tab + 4 * i);
        if (e.w == EMURX_EMPTY) break;
        if (e.x == ns && e.y == lo && (e.z & 0xffffu) == hi) return make_uint2(e.w, e.z >> 16);
    }
    return make_uint2(EMURX_ID_NONE, 0);
}
__device__ uint32_t probe_ip4(const emurx_dev_tables& T, uint32_t ns, uint32_t ip) {
    if (ip == 0) return EMURX_ID_NONE;
    uint32_t i = emurx_ip4_hash(ns, ip) & T.ip4_mask;
    for (uint32_t k = 0; k <= T.ip4_mask; ++k, i = (i + 1) & T.ip4_mask) {
        uint4 e = ld4(T.ip4_tab + 4 * i);
        if (e.w == EMURX_EMPTY) return EMURX_ID_NONE;
        if (e.x == ns && e.y == ip) return e.w;
    }
    return EMURX_ID_NONE;
}
__device__ __forceinline__ uint32_t probe_ip6(const emurx_dev_tables& T, uint32_t ns, const uint32_t ip[4]) {
    if ((ip[0] | ip[1] | ip[2] | ip[3]) == 0) return EMURX_ID_NONE;
    uint32_t i = emurx_ip6_hash(ns, ip[0], ip[1], ip[2], ip[3]) & T.ip6_mask;
    for (uint32_t k = 0; k <= T.ip6_mask; ++k, i = (i + 1) & T.ip6_mask) {
        uint4 a = ld4(T.ip6_tab + 8 * i);
        uint4 b = ld4(T.ip6_tab + 8 * i + 4);
        if (b.w == EMURX_EMPTY) return EMURX_ID_NONE;
        if (a.x == ns && a.y == ip[0] && a.z == ip[1] && a.w == ip[2] && b.x == ip[3]) return b.w;
    }
    return EMURX_ID_NONE;
}

__device__ __forceinline__ void set_lk(Rec& r, uint32_t lk) {
    r.flags = (r.flags & ~EMURX_FLAG_LK_MASK) | (lk << EMURX_FLAG_LK_SHIFT);
}
// client found -> client.PluginCtx.Get(<plugin>) where the handler checks it
__device__ __forceinline__ void client_result(Rec& r, uint32_t cid, uint32_t cplugins, uint32_t plug,
                                              bool check) {
    if (cid == EMURX_ID_NONE) { set_lk(r, EMURX_LK_NO_CLIENT); return; }
    r.cl = cid;
    if (check && !(cplugins & (1u << plug))) { set_lk(r, EMURX_LK_CLIENT_NO_PLUGIN); return; }
    set_lk(r, EMURX_LK_CLIENT);
}
__device__ __forceinline__ uint32_t client_plugins(const emurx_dev_tables& T, uint32_t cid) {
    return cid == EMURX_ID_NONE ? 0u : T.client[8 * cid + 2];
}
// CClient.IsUnicastToMe client_ctx.go:389-398 (frames here are always > 6 bytes)
__device__ __forceinline__ bool unicast_to_me(const emurx_dev_tables& T, uint32_t cid,
                                              uint32_t dlo, uint32_t dhi) {
    return T.client[8 * cid + 0] == dlo && T.client[8 * cid + 1] == dhi;
}

// Go 1.18 net.IP.IsLinkLocalUnicast / IsGlobalUnicast for a 16-byte address (words LE)
__device__ __forceinline__ bool ip6_local_or_global(const uint32_t w[4]) {
    uint32_t b0 = w[0] & 0xff, b1 = (w[0] >> 8) & 0xff;
    bool v4in6 = w[0] == 0 && w[1] == 0 && (w[2] & 0xffff) == 0 && (w[2] >> 16) == 0xffffu;
    if (v4in6) {
        uint32_t v = w[3], c0 = v & 0xff, c1 = (v >> 8) & 0xff;
        bool ll = c0 == 169 && c1 == 254;
        if (ll) return true;
        if (v == 0xffffffffu || v == 0 || c0 == 127 || (c0 & 0xf0) == 0xe0) return false;
        return true;
    }
    bool ll = b0 == 0xfe && (b1 & 0xc0) == 0x80;
    if (ll) return true;
    if ((w[0] | w[1] | w[2] | w[3]) == 0) return false;                      // unspecified
    if (w[0] == 0 && w[1] == 0 && w[2] == 0 && w[3] == 0x01000000u) return false;  // ::1
    if (b0 == 0xff) return false;                                            // multicast
    return true;
}
// CNSCtx.CLookupByIPv6LocalGlobal ns_ctx.go:288-316
__device__ __forceinline__ uint32_t lookup_ip6_lg(const emurx_dev_tables& T, uint32_t ns, const uint32_t w[4]) {
    if (!ip6_local_or_global(w)) return EMURX_ID_NONE;
    uint32_t b11 = (w[2] >> 24) & 0xff, b12 = w[3] & 0xff;
    if (b11 == 0xff && b12 == 0xfe) {  // ExtractOnlyMac client_ctx.go:314-329
        uint32_t m0 = (w[2] & 0xff) ^ 2, m1 = (w[2] >> 8) & 0xff, m2 = (w[2] >> 16) & 0xff;
        uint32_t m3 = (w[3] >> 8) & 0xff, m4 = (w[3] >> 16) & 0xff, m5 = w[3] >> 24;
        uint32_t lo = m0 | (m1 << 8) | (m2 << 16) | (m3 << 24), hi = m4 | (m5 << 8);
        uint32_t cid = probe_mac(T, ns, lo, hi).x;
        if (cid == EMURX_ID_NONE) return cid;
        // CClient.IsValidPrefix client_ctx.go:279-295
        if (w[0] == 0x000080feu && w[1] == 0) return cid;
        const uint32_t* c = T.client + 8 * cid;
        uint32_t ra = c[3];
        if ((ra & 1u) && ((ra >> 8) & 0xff) == 64 && c[4] == w[0] && c[5] == w[1]) return cid;
        return EMURX_ID_NONE;
    }
    return probe_ip6(T, ns, w);
}
// PluginDhcpNs.GetMacFromDhcp dhcp.go:863-891 + DHCPv4.DecodeFromBytes dhcpv4.go:125-172
template <class S>
__device__ bool dhcp_chaddr(const S& s, uint32_t len, const Rec& r, uint32_t& lo, uint32_t& hi) {
    uint32_t d = r.l7, dlen = r.l7len;
    if (dlen < 240) return false;
    if (((d + dlen) & 0xffff) < d || d + dlen > len) return false;
    if (be32(s, d + 236) != 0x63825363u) return false;
    if (dlen > 240) {
        uint32_t o = d + 240;
        int stop = (int)dlen - 240, start = 0;
        while (start < stop) {
            uint32_t t = s.u8(o + start);
            if (t == 255) break;
            if (t == 0) { start++; continue; }
            if (stop - start < 2) return false;
            int l = (int)s.u8(o + start + 1);
            if (l > stop - start - 2) return false;
            start += l + 2;
        }
    }
    if (s.u8(d + 1) != 1 || s.u8(d + 2) != 6) return false;
    lo = le32(s, d + 28);
    hi = s.u8(d + 32) | (s.u8(d + 33) << 8);
    return true;
}

__constant__ uint8_t kCbPlugin[EMURX_NUM_CB] = {
    EMURX_PLUG_ARP, EMURX_PLUG_ICMP, EMURX_PLUG_IGMP, EMURX_PLUG_DHCP, EMURX_PLUG_DHCPSRV,
    EMURX_PLUG_DHCPV6, EMURX_PLUG_MDNS, EMURX_PLUG_TRANSPORT, EMURX_PLUG_TRANSPORT,
    EMURX_PLUG_IPV6, EMURX_PLUG_DOT1X, EMURX_PLUG_PPP};

template <class S>
__device__ void classify(const S& s, uint32_t len, const emurx_dev_tables& T, Rec& r) {
    if (r.status != EMURX_ST_OK) return;
    const uint2 nsr = probe_ns(T, r.vport, r.vlan0, r.vlan1);  // CTunnelKey words
    const uint32_t ns = nsr.x;
    if (ns == EMURX_ID_NONE) { set_lk(r, EMURX_LK_NO_NS); return; }
    r.ns = ns;
    uint32_t cb = r.proto, plug = kCbPlugin[cb];
    if (!(nsr.y & (1u << plug))) { set_lk(r, EMURX_LK_NS_NO_PLUGIN); return; }
    uint32_t dlo = le32(s, 0), dhi = s.u8(4) | (s.u8(5) << 8);  // p[0:6]
    bool bcast = dlo == 0xffffffffu && dhi == 0xffffu;
    switch (cb) {
    case EMURX_CB_ARP:  // arp.go:904-949
        if (be16(s, r.l3 + 6) == 1) {
            const uint32_t cid = probe_ip4(T, ns, le32(s, r.l3 + 24));
            client_result(r, cid, client_plugins(T, cid), plug, true);
        } else {
            set_lk(r, EMURX_LK_NS_LEVEL);
        }
        return;
    case EMURX_CB_ICMP: {  // icmp.go:396-427
        uint32_t cid = probe_ip4(T, ns, le32(s, r.l3 + 16));
        if (cid != EMURX_ID_NONE && !unicast_to_me(T, cid, dlo, dhi)) cid = EMURX_ID_NONE;
        client_result(r, cid, 0, plug, false);
        return;
    }
    case EMURX_CB_IGMP:
    case EMURX_CB_MDNS:
        set_lk(r, EMURX_LK_NS_LEVEL);
        return;
    case EMURX_CB_DHCP: {  // dhcp.go:893-917
        uint32_t lo = dlo, hi = dhi;
        if (bcast && !dhcp_chaddr(s, len, r, lo, hi)) { set_lk(r, EMURX_LK_NO_CLIENT); return; }
        const uint2 c = probe_mac(T, ns, lo, hi);
        client_result(r, c.x, c.y, plug, true);
        return;
    }
    case EMURX_CB_DHCPSRV:  // dhcpsrv.go:1798-1826: broadcast -> GetFirstClient
    case EMURX_CB_EAPOL: {  // dot1x.go:624-650: 01:80:c2:00:00:03 -> GetFirstClient
        const bool first = cb == EMURX_CB_DHCPSRV ? bcast : (dlo == 0x00c28001u && dhi == 0x0300u);
        if (first) {
            const uint32_t cid = T.ns_info[4 * ns + 1];
            client_result(r, cid, client_plugins(T, cid), plug, true);
        } else {
            const uint2 c = probe_mac(T, ns, dlo, dhi);
            client_result(r, c.x, c.y, plug, true);
        }
        return;
    }
    case EMURX_CB_ICMPV6: {  // ipv6.go:465-540
        if (be16(s, r.l4) != 0x8000u) { set_lk(r, EMURX_LK_NS_LEVEL); return; }
        if (r.l3 + 40 > len) { set_lk(r, EMURX_LK_NO_CLIENT); return; }
        uint32_t w[4] = {le32(s, r.l3 + 24), le32(s, r.l3 + 28), le32(s, r.l3 + 32), le32(s, r.l3 + 36)};
        uint32_t cid = lookup_ip6_lg(T, ns, w);
        if (cid != EMURX_ID_NONE && !unicast_to_me(T, cid, dlo, dhi)) cid = EMURX_ID_NONE;
        if (cid != EMURX_ID_NONE && s.u8(r.l3 + 8) == 0xff) cid = EMURX_ID_NONE;
        client_result(r, cid, 0, plug, false);
        return;
    }
    default: {  // dhcpv6, ppp, tcp, udp: client = MAC[dst] (plugin_transport.go:83-115 ...)
        const uint2 c = probe_mac(T, ns, dlo, dhi);
        client_result(r, c.x, c.y, plug, true);
        return;
    }
    }
}

}  // namespace emurx
