// emurx_tables.h — device-resident Namespace / Client tables (layout shared by the host
// builder in emurx_api.cpp and the HIP kernels in emurx_kernels.hip).
//
// They mirror the reference's Go maps:
//   MapNsT        map[CTunnelKey]*CNSCtx   src/emu/core/thread_ctx.go:139
//   MapClientMAC  map[MACKey]*CClient      src/emu/core/ns_ctx.go:110-112  (per Namespace)
//   MapClientIPv4 map[Ipv4Key]*CClient
//   MapClientIPv6 map[Ipv6Key]*CClient     (static Ipv6 and Dhcpv6 addresses, ns_ctx.go:377-383)
// as flat open-addressing arrays of 64-byte BUCKETS (one cache line; 4 slots of 16 B, IPv4 and
// IPv6: 2 slots of 32 B), load factor <= 1/2, power-of-two bucket counts, linear probing over
// buckets.  A lookup reads its home bucket with four 16-byte loads of one line and ends at
// the first bucket that holds an empty slot.  Only exact-match semantics matter for parity
// with the Go maps; the hash function is ours.
//
// The per-Namespace client maps become one global map per key kind, keyed by
// (Namespace, address) and hashed from (CTunnelKey hash, address): a frame's client bucket
// is known from its parsed tunnel key alone, so the Namespace and Client probes of one frame
// are issued together (one memory round trip) and the Namespace id is compared afterwards.
#pragma once
#include <stdint.h>

#ifndef EMURX_HD
#if defined(__HIPCC__)
#define EMURX_HD __host__ __device__ __forceinline__
#else
#define EMURX_HD static inline
#endif
#endif

#define EMURX_EMPTY 0xFFFFFFFFu
// a deleted slot: value EMURX_TOMB, every key word 0xFFFFFFFF (no probe key ever equals it:
// vport words are < 0x10000, Namespace and client ids < EMURX_ID_NONE); a probe walks past
// it and only a bucket with an EMPTY slot ends a chain
#define EMURX_TOMB 0xFFFFFFFEu
#define EMURX_BUCKET_WORDS 16u  // 64 B
#define EMURX_CPL_CTX 0x8000u   // client slot plugin half: the client has a TransportCtx

// 32-bit mix of up to five key words (murmur3 finaliser over a multiplicative combine).
EMURX_HD uint32_t emurx_fmix(uint32_t h) {
    h ^= h >> 16; h *= 0x85EBCA6Bu;
    h ^= h >> 13; h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
EMURX_HD uint32_t emurx_hash(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e) {
    uint32_t h = a * 0x9E3779B1u;
    h = (h ^ (h >> 15)) + b * 0x85EBCA77u;
    h = (h ^ (h >> 13)) + c * 0xC2B2AE3Du;
    h = (h ^ (h >> 16)) + d * 0x27D4EB2Fu;
    h = (h ^ (h >> 15)) + e * 0x165667B1u;
    return emurx_fmix(h);
}

// Slot layouts (uint32 words; the last word of a slot is the value, EMURX_EMPTY = free):
//  ns   [4]: vport | ns_plugins << 16, vlan0, vlan1, ns_id   (key = CTunnelKey as 3 LE words)
//  mac  [4]: ns_id, mac[0..3] LE, mac[4..5] LE | client_plugins << 16, client_id
//  ip4  [8]: ns_id, ipv4 bytes LE, mac[0..3], mac[4..5] | client_plugins << 16, 0, 0, 0, client_id
//  ip6  [8]: ns_id, ip[0..3], ip[4..7], ip[8..11], ip[12..15], mac[0..3], mac[4..5] | client_plugins << 16,
//            client_id
//  (the client's MAC and plugin mask in the IP slots answer IsUnicastToMe / PluginCtx.Get;
//  the mask's top bit, EMURX_CPL_CTX, is set when the client has a TransportCtx)
//  ns_info   [4]: plugin_mask, first_client, 0, 0            (dense, indexed by ns id)
//  ci   [8]: client_id, plugin_mask, ra (bit0 has_ra, bits 8..15 prefix_len), ra_prefix[0..3],
//            ra_prefix[4..7], has_transport_ctx, 0, 0      (hashed by client id, 2 per bucket)
// Home buckets: ns = tk & ns_mask; client tables = hash(tk, address) & mask, where
// tk = emurx_tk_hash(CTunnelKey words) of the client's Namespace; ci = emurx_ci_hash(id).
EMURX_HD uint32_t emurx_tk_hash(uint32_t w0, uint32_t w1, uint32_t w2) {
    return emurx_hash(w0, w1, w2, 0x6E73u, 0);
}
EMURX_HD uint32_t emurx_mac_hash(uint32_t tk, uint32_t lo, uint32_t hi) {
    return emurx_hash(tk, lo, hi, 0x6D6163u, 0);
}
EMURX_HD uint32_t emurx_ip4_hash(uint32_t tk, uint32_t ip) {
    return emurx_hash(tk, ip, 0x697034u, 0, 0);
}
EMURX_HD uint32_t emurx_ip6_hash(uint32_t tk, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return emurx_hash(tk, a ^ 0x697036u, b, c, d);
}
EMURX_HD uint32_t emurx_ci_hash(uint32_t cid) {
    return emurx_hash(cid, 0x63696eu, 0, 0, 0);
}

// Transport tables (TransportCtx.ftv4 / ftv6 / serverCb, src/emu/plugins/transport/
// client_ctx.go:490-497), one global map per kind keyed by (client id, tuple):
//  ft4  [8]: cid, src LE, dst LE, ports (4 wire bytes LE), proto, 0, 0, flow_id   (2 per bucket)
//  ft6 [16]: cid, src[4], dst[4], ports, nh, 0 x 5, flow_id                       (1 per bucket)
//  srv  [4]: cid, port | proto << 16, 0, 1                                        (4 per bucket)
// client word 6 bit 0: the client has a TransportCtx.
EMURX_HD uint32_t emurx_ft4_hash(uint32_t cid, uint32_t src, uint32_t dst, uint32_t ports, uint32_t proto) {
    return emurx_hash(cid, src, dst, ports, proto ^ 0x667434u);
}
EMURX_HD uint32_t emurx_ft6_hash(uint32_t cid, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, uint32_t d0,
                                 uint32_t d1, uint32_t d2, uint32_t d3, uint32_t ports, uint32_t nh) {
    return emurx_hash(emurx_hash(cid, s0, s1, s2, s3), d0, d1, d2, d3 ^ (ports * 0x9E3779B1u) ^ nh);
}
EMURX_HD uint32_t emurx_srv_hash(uint32_t cid, uint32_t port_proto) {
    return emurx_hash(cid, port_proto, 0x737276u, 0, 0);
}

struct emurx_dev_tables {
    const uint32_t* ns_tab;   // [ns_mask + 1] buckets of 4 slots
    const uint32_t* ns_info;  // 4 words per ns id
    const uint32_t* mac_tab;  // [mac_mask + 1] buckets of 4 slots
    const uint32_t* ip4_tab;  // [ip4_mask + 1] buckets of 2 slots
    const uint32_t* ip6_tab;  // [ip6_mask + 1] buckets of 2 slots
    const uint32_t* ci_tab;   // [ci_mask + 1] buckets of 2 client-info slots
    uint32_t ns_mask, mac_mask, ip4_mask, ip6_mask;  // bucket count - 1
    uint32_t ci_mask, max_ns;
    uint32_t cb_mask;         // registered callbacks (Parser.Register)
    uint32_t ft_on;           // any client has a TransportCtx: resolve transport flows
    const uint32_t* ft4_tab;  // [ft4_mask + 1] buckets of 2 slots
    const uint32_t* ft6_tab;  // [ft6_mask + 1] buckets of 1 slot
    const uint32_t* srv_tab;  // [srv_mask + 1] buckets of 4 slots
    uint32_t ft4_mask, ft6_mask, srv_mask, pad;
};

// Namespace partition of a tunnel-key hash among n_parts <= 8 GPUs: the top 7 bits of the
// hash, scaled (uniform for a well-mixed hash, no division).  The owner is a function of the
// frame's OWNER KEY, the descriptor byte 0x80 | min(tk >> 25, 126) that the device framing
// walk writes (emurx_desc.pad, EMURX_DESC_KEYED): 126 and 127 give the same owner for every
// n_parts <= 8, so the key never collides with EMURX_DESC_HOLE (0xFF).
EMURX_HD uint32_t emurx_owner(uint32_t tk, uint32_t n_parts) { return ((tk >> 25) * n_parts) >> 7; }
EMURX_HD uint32_t emurx_owner_key(uint32_t tk) {
    const uint32_t k = tk >> 25;
    return 0x80u | (k < 126u ? k : 126u);
}
EMURX_HD uint32_t emurx_owner_of_key(uint32_t key, uint32_t n_parts) { return ((key & 0x7fu) * n_parts) >> 7; }
