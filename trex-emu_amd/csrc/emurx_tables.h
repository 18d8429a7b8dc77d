// emurx_tables.h — device-resident Namespace / Client tables (layout shared by the host
// builder in emurx_mirror.cpp and the HIP kernels in emurx_parse.h / emurx_kernels.hip).
//
// They mirror the reference's Go maps:
//   MapNsT        map[CTunnelKey]*CNSCtx   src/emu/core/thread_ctx.go:139
//   MapClientMAC  map[MACKey]*CClient      src/emu/core/ns_ctx.go:110-112  (per Namespace)
//   MapClientIPv4 map[Ipv4Key]*CClient
//   MapClientIPv6 map[Ipv6Key]*CClient     (static Ipv6 and Dhcpv6 addresses, ns_ctx.go:377-383)
// as bucketized CUCKOO tables with two choices: every key lives in one of exactly two 32-byte
// buckets (b1, b2 below; two 16-byte slots, or one 32-byte slot, per bucket; the IPv6 flow
// table: one 64-byte slot per 64-byte bucket).  A lookup issues both bucket reads together
// and is resolved after ONE memory round trip, whatever the table's load: there are no probe
// chains, so no lane of a wave can hold the wave back for extra trips, and the tables stay
// dense (load 1/2 .. 4/5 for two-slot buckets, 1/3 .. 0.45 for one-slot buckets).  A delete
// clears its slot (no tombstones).  Only exact-match semantics matter for parity with the Go
// maps; the hash functions are ours.
//
// The per-Namespace client maps become one global map per key kind, keyed by
// (Namespace, address) and hashed from (CTunnelKey hash, address): a frame's client buckets
// are known from its parsed tunnel key alone, so the Namespace and Client probes of one frame
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
#define EMURX_BUCKET_WORDS 16u  // 64-byte shipment blocks (emurx_delta) of every table image
#define EMURX_CBUCKET_WORDS 8u  // 32-byte cuckoo buckets (the IPv6 flow table: 16 words)

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
EMURX_HD uint32_t emurx_mulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

// The two candidate buckets of a key whose table hash is h, in a table of nb buckets (any
// count >= 1, not a power of two: range reduction by multiply-high).  b2 takes the high bits
// of h times an odd constant, which depend on h's low bits, so keys sharing b1 spread over
// b2.  b1 == b2 is allowed (the key then has one bucket).
EMURX_HD uint32_t emurx_b1(uint32_t h, uint32_t nb) { return emurx_mulhi(h, nb); }
EMURX_HD uint32_t emurx_b2(uint32_t h, uint32_t nb) { return emurx_mulhi(h * 0x2C1B3C6Du, nb); }

// Slot layouts (uint32 words; the marker word is EMURX_EMPTY in a free slot):
//  ns   [4]: vport | ns_plugins << 16, vlan0, vlan1, ns_id          (marker: ns_id)
//  mac  [4]: ns_id, mac[0..3] LE, mac[4..5] LE | client_plugins << 16, client_id   (client_id)
//  ip4  [8]: ns_id, ipv4 bytes LE, mac[0..3], mac[4..5] | client_plugins << 16, 0, 0, 0,
//            client_id                                              (client_id)
//  ip6  [8]: ns_id, ip[0..3], ip[4..7], ip[8..11], ip[12..15], mac[0..3],
//            mac[4..5] | client_plugins << 16, client_id            (client_id)
//  (the client's MAC and plugin mask in the IP slots answer IsUnicastToMe / PluginCtx.Get)
//  ci   [4]: client_id, plugins & 0xffff | has_ra << 16 | has_transport_ctx << 17 |
//            ra_prefix_len << 24, ra_prefix[0..3], ra_prefix[4..7]  (client_id)
//  ns_info   [4]: plugin_mask, first_client, 0, 0            (dense, indexed by ns id)
// Table hashes (the seed of a table is chosen by the host and changed when a cuckoo insert
// fails, emurx_mirror.cpp): ns = emurx_ns_hash(tk); clients = hash(tk, address), where
// tk = emurx_tk_hash(CTunnelKey words) of the client's Namespace; ci = emurx_ci_hash(id).
EMURX_HD uint32_t emurx_tk_hash(uint32_t w0, uint32_t w1, uint32_t w2) {
    return emurx_hash(w0, w1, w2, 0x6E73u, 0);
}
EMURX_HD uint32_t emurx_ns_hash(uint32_t tk, uint32_t seed) { return emurx_fmix(tk ^ seed); }
EMURX_HD uint32_t emurx_mac_hash(uint32_t tk, uint32_t lo, uint32_t hi, uint32_t seed) {
    return emurx_hash(tk, lo, hi, 0x6D6163u, seed);
}
EMURX_HD uint32_t emurx_ip4_hash(uint32_t tk, uint32_t ip, uint32_t seed) {
    return emurx_hash(tk, ip, 0x697034u, 0, seed);
}
EMURX_HD uint32_t emurx_ip6_hash(uint32_t tk, uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t seed) {
    return emurx_hash(tk, a ^ 0x697036u ^ seed, b, c, d);
}
EMURX_HD uint32_t emurx_ci_hash(uint32_t cid, uint32_t seed) {
    return emurx_hash(cid, 0x63696eu, 0, 0, seed);
}

// Transport tables (TransportCtx.ftv4 / ftv6 / serverCb, src/emu/plugins/transport/
// client_ctx.go:490-497), one global map per kind keyed by (client id, tuple):
//  ft4  [8]: cid, src LE, dst LE, ports (4 wire bytes LE), proto, 0, 0, flow_id   (flow_id)
//  ft6 [16]: cid, src[4], dst[4], ports, nh, 0 x 4, flow_id                       (flow_id)
//  srv  [4]: cid, port | proto << 16, 0, 1                                        (word 3)
// client info bit 17: the client has a TransportCtx.
EMURX_HD uint32_t emurx_ft4_hash(uint32_t cid, uint32_t src, uint32_t dst, uint32_t ports, uint32_t proto,
                                 uint32_t seed) {
    return emurx_hash(cid, src, dst, ports, proto ^ 0x667434u ^ seed);
}
EMURX_HD uint32_t emurx_ft6_hash(uint32_t cid, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, uint32_t d0,
                                 uint32_t d1, uint32_t d2, uint32_t d3, uint32_t ports, uint32_t nh, uint32_t seed) {
    return emurx_hash(emurx_hash(cid, s0, s1, s2, s3), d0, d1, d2, d3 ^ (ports * 0x9E3779B1u) ^ nh ^ seed);
}
EMURX_HD uint32_t emurx_srv_hash(uint32_t cid, uint32_t port_proto, uint32_t seed) {
    return emurx_hash(cid, port_proto, 0x737276u, 0, seed);
}

// one table as the kernels see it: base, bucket count, hash seed
struct emurx_dev_tab {
    const uint32_t* p;
    uint32_t nb, seed;
};
struct emurx_dev_tables {
    emurx_dev_tab ns, mac, ip4, ip6, ci;  // 32-byte buckets
    const uint32_t* ns_info;              // 4 words per ns id
    uint32_t max_ns;
    uint32_t cb_mask;                     // registered callbacks (Parser.Register)
    uint32_t ft_on;                       // any client has a TransportCtx: resolve transport flows
    emurx_dev_tab ft4, srv;               // 32-byte buckets
    emurx_dev_tab ft6;                    // 64-byte buckets
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
