// emurx_api.cpp — C-ABI of the MI355X receive path (include/emu_rx.h).
//
// Owns the Namespace / Client tables (host copies with the Go maps' semantics, flattened
// into the device layout of emurx_tables.h on emurx_sync), the device scratch of a batch,
// and the host batch entry point that replaces VethIFZmq.OnRxStream's per-frame loop
// (src/emu/core/veth_zmq.go:277-320).  No exception or abort crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <unordered_map>
#include <vector>

#include "../../include/emu_rx.h"
#include "emurx_kernels.h"
#include "emurx_tables.h"

namespace {

uint32_t pow2_at_least(uint64_t v) {
    uint64_t p = 16;
    while (p < v) p <<= 1;
    return (uint32_t)p;
}
uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
bool zero(const uint8_t* p, int n) {
    for (int i = 0; i < n; ++i)
        if (p[i]) return false;
    return true;
}

// table keys: (ns_id, address words) — the per-Namespace Go maps flattened into one
struct K5 {
    uint32_t w[5];
    bool operator==(const K5& o) const { return !memcmp(w, o.w, sizeof(w)); }
};
struct K5Hash {
    size_t operator()(const K5& k) const { return emurx_hash(k.w[0], k.w[1], k.w[2], k.w[3], k.w[4]); }
};
using Map = std::unordered_map<K5, uint32_t, K5Hash>;

K5 key_ns(const uint8_t* k12) { return K5{{le32(k12), le32(k12 + 4), le32(k12 + 8), 0, 0}}; }
K5 key_mac(uint32_t ns, const uint8_t* m) {
    return K5{{ns, le32(m), (uint32_t)(m[4] | (m[5] << 8)), 0, 0}};
}
K5 key_ip4(uint32_t ns, const uint8_t* ip) { return K5{{ns, le32(ip), 0, 0, 0}}; }
K5 key_ip6(uint32_t ns, const uint8_t* ip) {
    return K5{{ns, le32(ip), le32(ip + 4), le32(ip + 8), le32(ip + 12)}};
}

struct NsInfo {
    bool alive = false;
    uint8_t key[12] = {0};
    uint32_t plugins = 0;
    std::vector<uint32_t> order;  // clientHead dlist (insertion order)
};
struct ClientInfo {
    bool alive = false;
    uint32_t ns = 0;
    uint8_t mac[6] = {0}, ipv4[4] = {0}, ipv6[16] = {0}, dhcpv6[16] = {0};
    uint32_t plugins = 0;
    bool has_ra = false;
    uint8_t ra_prefix[16] = {0};
    uint8_t ra_plen = 0;
};

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    int alloc(size_t count) {
        if (count <= n && p) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (hipMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T)) != hipSuccess) return -1;
        n = count;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};
template <class T>
struct PinBuf {
    T* p = nullptr;
    size_t n = 0;
    int alloc(size_t count) {
        if (count <= n && p) return 0;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        if (hipHostMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T), hipHostMallocDefault) != hipSuccess)
            return -1;
        n = count;
        return 0;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
};

}  // namespace

struct emurx_ctx {
    emurx_cfg cfg{};
    hipStream_t stream = nullptr;
    uint32_t cb_mask = 0;  // Parser.Init: every callback parserNotSupported (eapol nil)

    // authoritative tables (Go map semantics)
    Map ns_map, mac_map, ip4_map, ip6_map;
    std::vector<NsInfo> ns;
    std::vector<ClientInfo> cl;
    bool dirty = true;

    // device tables
    uint32_t ns_buckets = 0, mac_buckets = 0, ip4_buckets = 0, ip6_buckets = 0;
    DevBuf<uint32_t> d_ns, d_nsinfo, d_mac, d_ip4, d_ip6, d_client;
    std::vector<uint32_t> h_ns, h_nsinfo, h_mac, h_ip4, h_ip6, h_client;

    // host batch staging (emurx_rx_stream): message, descriptors, and the batch outputs
    PinBuf<uint8_t> h_msg;
    PinBuf<emurx_desc> h_desc;
    PinBuf<uint32_t> h_qlist, h_tile_cnt;
    PinBuf<uint64_t> h_hist;
    DevBuf<uint8_t> d_msg;
    DevBuf<emurx_desc> d_desc;
    DevBuf<emurx_rec> d_rec;
    DevBuf<uint32_t> d_qlist, d_tile_cnt;
    DevBuf<uint64_t> d_hist;

    // Namespace-partition packing scratch (emurx_route_dev)
    DevBuf<uint32_t> d_route_cnt, d_route_grp, d_route_goff;  // grp: zero between batches

    // timing ring: 2 events per batch (around the k_rx launch)
    std::vector<hipEvent_t> ev;
    uint32_t slots = 0, ev_head = 0, ev_count = 0, stride = 1, batch_seq = 0;

    emurx_dev_tables tables() const {
        emurx_dev_tables T{};
        T.ns_tab = d_ns.p;
        T.ns_info = d_nsinfo.p;
        T.mac_tab = d_mac.p;
        T.ip4_tab = d_ip4.p;
        T.ip6_tab = d_ip6.p;
        T.client = d_client.p;
        T.ns_mask = ns_buckets - 1;
        T.mac_mask = mac_buckets - 1;
        T.ip4_mask = ip4_buckets - 1;
        T.ip6_mask = ip6_buckets - 1;
        T.max_ns = cfg.max_ns;
        T.max_clients = cfg.max_clients;
        T.cb_mask = cb_mask;
        return T;
    }
};

namespace {

int bind(emurx_t* h) { return hipSetDevice(h->cfg.device) == hipSuccess ? EMURX_OK : EMURX_EDEVICE; }

// open-addressing insert into a bucketed table (emurx_tables.h): first free slot of the
// first bucket, in linear bucket order from the home bucket, that has one
void bucket_put(std::vector<uint32_t>& t, uint32_t bmask, uint32_t words, uint32_t h, const uint32_t* e) {
    const uint32_t per = EMURX_BUCKET_WORDS / words;
    for (uint32_t b = h & bmask;; b = (b + 1) & bmask)
        for (uint32_t k = 0; k < per; ++k) {
            uint32_t* slot = &t[(size_t)b * EMURX_BUCKET_WORDS + k * words];
            if (slot[words - 1] == EMURX_EMPTY) {
                memcpy(slot, e, words * sizeof(uint32_t));
                return;
            }
        }
}
void empty_table(std::vector<uint32_t>& t, uint32_t buckets, uint32_t words) {
    t.assign((size_t)buckets * EMURX_BUCKET_WORDS, 0);
    for (size_t i = words - 1; i < t.size(); i += words) t[i] = EMURX_EMPTY;
}

int rebuild_and_upload(emurx_t* h, hipStream_t st) {
    if (!h->dirty) return EMURX_OK;
    (void)hipStreamSynchronize(st);  // previous upload may still read the staging vectors
    empty_table(h->h_ns, h->ns_buckets, 4);
    for (auto& kv : h->ns_map) {
        // a key with non-zero bytes [2:4] can never equal a parsed CTunnelKey (Set writes 0
        // there, thread_ctx.go:93): it has no device slot.  The free upper half of the vport
        // word carries the Namespace's plugin mask, so one probe answers GetNs + PluginCtx.Get.
        if (kv.first.w[0] >> 16) continue;
        uint32_t e[4] = {kv.first.w[0] | (h->ns[kv.second].plugins << 16), kv.first.w[1], kv.first.w[2],
                         kv.second};
        bucket_put(h->h_ns, h->ns_buckets - 1, 4, emurx_tk_hash(kv.first.w[0], e[1], e[2]), e);
    }
    h->h_nsinfo.assign((size_t)h->cfg.max_ns * 4, 0);
    for (uint32_t i = 0; i < h->ns.size(); ++i) {
        const NsInfo& n = h->ns[i];
        h->h_nsinfo[i * 4 + 0] = n.alive ? n.plugins : 0;
        h->h_nsinfo[i * 4 + 1] = (n.alive && !n.order.empty()) ? n.order.front() : EMURX_ID_NONE;
    }
    // client entries hash from their Namespace's tunnel key (emurx_tables.h)
    auto tk_of = [&](uint32_t ns) {
        const uint8_t* k = h->ns[ns].key;
        return emurx_tk_hash(le32(k), le32(k + 4), le32(k + 8));
    };
    auto fill4 = [&](std::vector<uint32_t>& t, uint32_t buckets, const Map& m, int kind) {
        empty_table(t, buckets, 4);
        for (auto& kv : m) {
            uint32_t e[4] = {kv.first.w[0], kv.first.w[1], kv.first.w[2], kv.second};
            const uint32_t tk = tk_of(e[0]);
            uint32_t hh = kind == 0 ? emurx_mac_hash(tk, e[1], e[2]) : emurx_ip4_hash(tk, e[1]);
            if (kind == 1) e[2] = 0;
            // MAC slots carry the client's plugin mask in the free upper half of mac[4..5]
            if (kind == 0) e[2] |= (h->cl[kv.second].plugins & 0xffffu) << 16;
            bucket_put(t, buckets - 1, 4, hh, e);
        }
    };
    fill4(h->h_mac, h->mac_buckets, h->mac_map, 0);
    fill4(h->h_ip4, h->ip4_buckets, h->ip4_map, 1);
    empty_table(h->h_ip6, h->ip6_buckets, 8);
    for (auto& kv : h->ip6_map) {
        const uint32_t* w = kv.first.w;
        uint32_t e[8] = {w[0], w[1], w[2], w[3], w[4], 0, 0, kv.second};
        bucket_put(h->h_ip6, h->ip6_buckets - 1, 8, emurx_ip6_hash(tk_of(w[0]), w[1], w[2], w[3], w[4]), e);
    }
    h->h_client.assign((size_t)h->cfg.max_clients * 8, 0);
    for (uint32_t i = 0; i < h->cl.size(); ++i) {
        const ClientInfo& c = h->cl[i];
        if (!c.alive) continue;
        uint32_t* o = &h->h_client[(size_t)i * 8];
        o[0] = le32(c.mac);
        o[1] = (uint32_t)(c.mac[4] | (c.mac[5] << 8));
        o[2] = c.plugins;
        o[3] = (c.has_ra ? 1u : 0u) | ((uint32_t)c.ra_plen << 8);
        o[4] = le32(c.ra_prefix);
        o[5] = le32(c.ra_prefix + 4);
    }
    struct {
        uint32_t* d;
        std::vector<uint32_t>* h;
    } up[] = {{h->d_ns.p, &h->h_ns},   {h->d_nsinfo.p, &h->h_nsinfo}, {h->d_mac.p, &h->h_mac},
              {h->d_ip4.p, &h->h_ip4}, {h->d_ip6.p, &h->h_ip6},       {h->d_client.p, &h->h_client}};
    for (auto& u : up)
        if (hipMemcpyAsync(u.d, u.h->data(), u.h->size() * 4, hipMemcpyHostToDevice, st) != hipSuccess)
            return EMURX_EDEVICE;
    if (hipStreamSynchronize(st) != hipSuccess) return EMURX_EDEVICE;
    h->dirty = false;
    return EMURX_OK;
}

uint32_t ntiles(uint32_t n) { return (n + EMURX_QUEUE_TILE - 1) / EMURX_QUEUE_TILE; }
size_t queue_cap(uint32_t n) { return (size_t)ntiles(n) * EMURX_QUEUE_TILE; }

int run_dev(emurx_t* h, const uint8_t* frames, const emurx_desc* desc, uint32_t n,
            const emurx_dev_out* out, void* stream, bool classify) {
    if (!h || !out || !out->hist || (n && (!frames || !desc))) return EMURX_EINVAL;
    if (((uintptr_t)frames & 15) || ((uintptr_t)desc & 7)) return EMURX_EINVAL;  // 16-B staging loads
    if (n > h->cfg.max_frames) return EMURX_ENOMEM;
    if (out->qlist && out->qcap < queue_cap(n)) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    if (classify && (rc = rebuild_and_upload(h, st))) return rc;
    emurx_dev_tables T = h->tables();
    const hipEvent_t* ev = nullptr;
    if (h->slots && (h->batch_seq++ % h->stride) == 0) {
        const uint32_t s = h->ev_head;
        ev = &h->ev[2 * s];
        h->ev_head = (s + 1) % h->slots;
        h->ev_count = std::min(h->ev_count + 1, h->slots);
    }
    int r = emurx_launch_batch(frames, desc, n, T, classify, *out, st, ev);
    return r ? EMURX_EDEVICE : EMURX_OK;
}

}  // namespace

extern "C" {

int emurx_abi_version(void) { return EMURX_ABI_VERSION; }

const char* emurx_strerror(int code) {
    switch (code) {
    case EMURX_OK: return "ok";
    case EMURX_EINVAL: return "invalid argument";
    case EMURX_ENOMEM: return "out of memory / capacity exceeded";
    case EMURX_EEXIST: return "already exists";
    case EMURX_ENOENT: return "not found";
    case EMURX_EDEVICE: return "HIP runtime error";
    case EMURX_ENOSPC: return "output buffer too small";
    default: return "unknown error";
    }
}

int emurx_open(const emurx_cfg* cfg, emurx_t** out) {
    if (!cfg || !out || cfg->max_ns == 0 || cfg->max_clients == 0 || cfg->max_frames == 0) return EMURX_EINVAL;
    emurx_t* h = new (std::nothrow) emurx_ctx();
    if (!h) return EMURX_ENOMEM;
    h->cfg = *cfg;
    if (h->cfg.max_bytes == 0) h->cfg.max_bytes = 1u << 20;
    int rc = bind(h);
    if (rc) { delete h; return rc; }
    if (hipStreamCreate(&h->stream) != hipSuccess) { delete h; return EMURX_EDEVICE; }
    // load factor <= 1/2 in slots: 4 slots (IPv6: 2) per 64-byte bucket
    h->ns_buckets = pow2_at_least(2ull * cfg->max_ns) / 4;
    h->mac_buckets = pow2_at_least(2ull * cfg->max_clients) / 4;
    h->ip4_buckets = pow2_at_least(2ull * cfg->max_clients) / 4;
    h->ip6_buckets = pow2_at_least(4ull * cfg->max_clients) / 2;
    h->ns.resize(cfg->max_ns);
    h->cl.resize(cfg->max_clients);
    const size_t BW = EMURX_BUCKET_WORDS;
    if (h->d_ns.alloc(h->ns_buckets * BW) || h->d_nsinfo.alloc((size_t)cfg->max_ns * 4) ||
        h->d_mac.alloc(h->mac_buckets * BW) || h->d_ip4.alloc(h->ip4_buckets * BW) ||
        h->d_ip6.alloc(h->ip6_buckets * BW) || h->d_client.alloc((size_t)cfg->max_clients * 8)) {
        emurx_close(h);
        return EMURX_ENOMEM;
    }
    h->dirty = true;
    if ((rc = rebuild_and_upload(h, h->stream))) { emurx_close(h); return rc; }
    *out = h;
    return EMURX_OK;
}

void emurx_close(emurx_t* h) {
    if (!h) return;
    bind(h);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    h->d_ns.release(); h->d_nsinfo.release(); h->d_mac.release(); h->d_ip4.release();
    h->d_ip6.release(); h->d_client.release();
    h->h_msg.release(); h->h_desc.release(); h->h_qlist.release(); h->h_tile_cnt.release();
    h->h_hist.release();
    h->d_msg.release(); h->d_desc.release(); h->d_rec.release(); h->d_qlist.release();
    h->d_tile_cnt.release(); h->d_hist.release();
    h->d_route_cnt.release(); h->d_route_grp.release(); h->d_route_goff.release();
    for (auto& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    h->ev.clear();
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

// Parser.Register parser.go:528-565 (unknown names are ignored, as in Go)
int emurx_register(emurx_t* h, const char* p) {
    if (!h || !p) return EMURX_EINVAL;
    static const struct { const char* name; uint32_t bits; } tab[] = {
        {"arp", 1u << EMURX_CB_ARP},         {"icmp", 1u << EMURX_CB_ICMP},
        {"igmp", 1u << EMURX_CB_IGMP},       {"dhcp", 1u << EMURX_CB_DHCP},
        {"dhcpsrv", 1u << EMURX_CB_DHCPSRV}, {"icmpv6", 1u << EMURX_CB_ICMPV6},
        {"dhcpv6", 1u << EMURX_CB_DHCPV6},   {"dot1x", 1u << EMURX_CB_EAPOL},
        {"mdns", 1u << EMURX_CB_MDNS},       {"ppp", 1u << EMURX_CB_PPP},
        {"transport", (1u << EMURX_CB_TCP) | (1u << EMURX_CB_UDP)}};
    for (auto& t : tab)
        if (!strcmp(p, t.name)) h->cb_mask |= t.bits;
    return EMURX_OK;
}
int emurx_set_callbacks_mask(emurx_t* h, uint32_t mask) {
    if (!h) return EMURX_EINVAL;
    h->cb_mask = mask & ((1u << EMURX_NUM_CB) - 1u);
    return EMURX_OK;
}
uint32_t emurx_get_callbacks_mask(const emurx_t* h) { return h ? h->cb_mask : 0; }

// ---- tables ------------------------------------------------------------------------------
// CThreadCtx.AddNs thread_ctx.go:786-795
int emurx_ns_add(emurx_t* h, const uint8_t key[12], uint32_t ns_id, uint32_t plugin_mask) {
    if (!h || !key) return EMURX_EINVAL;
    if (ns_id >= h->cfg.max_ns) return EMURX_ENOMEM;
    K5 k = key_ns(key);
    if (h->ns_map.count(k) || h->ns[ns_id].alive) return EMURX_EEXIST;
    NsInfo& n = h->ns[ns_id];
    n.alive = true;
    memcpy(n.key, key, 12);
    n.plugins = plugin_mask;
    n.order.clear();
    h->ns_map[k] = ns_id;
    h->dirty = true;
    return EMURX_OK;
}
// CThreadCtx.RemoveNs thread_ctx.go:797-812 (refused while clients are active)
int emurx_ns_remove(emurx_t* h, const uint8_t key[12]) {
    if (!h || !key) return EMURX_EINVAL;
    auto it = h->ns_map.find(key_ns(key));
    if (it == h->ns_map.end()) return EMURX_ENOENT;
    NsInfo& n = h->ns[it->second];
    if (!n.order.empty()) return EMURX_EEXIST;
    n.alive = false;
    h->ns_map.erase(it);
    h->dirty = true;
    return EMURX_OK;
}
int emurx_ns_set_plugins(emurx_t* h, uint32_t ns_id, uint32_t plugin_mask) {
    if (!h) return EMURX_EINVAL;
    if (ns_id >= h->cfg.max_ns || !h->ns[ns_id].alive) return EMURX_ENOENT;
    h->ns[ns_id].plugins = plugin_mask;
    h->dirty = true;
    return EMURX_OK;
}

// CNSCtx.AddClient ns_ctx.go:332-389
int emurx_client_add(emurx_t* h, uint32_t ns_id, uint32_t cid, const uint8_t mac[6],
                     const uint8_t ipv4[4], const uint8_t ipv6[16], const uint8_t dhcpv6[16],
                     uint32_t plugin_mask) {
    static const uint8_t z[16] = {0};
    if (!h || !mac) return EMURX_EINVAL;
    if (ns_id >= h->cfg.max_ns || !h->ns[ns_id].alive) return EMURX_ENOENT;
    if (cid >= h->cfg.max_clients) return EMURX_ENOMEM;
    if (!ipv4) ipv4 = z;
    if (!ipv6) ipv6 = z;
    if (!dhcpv6) dhcpv6 = z;
    if (zero(mac, 6)) return EMURX_EINVAL;
    if (h->mac_map.count(key_mac(ns_id, mac))) return EMURX_EEXIST;
    bool has4 = !zero(ipv4, 4), has6 = !zero(ipv6, 16), has6d = !zero(dhcpv6, 16);
    if (has4 && h->ip4_map.count(key_ip4(ns_id, ipv4))) return EMURX_EEXIST;
    if (has6 && h->ip6_map.count(key_ip6(ns_id, ipv6))) return EMURX_EEXIST;
    if (has6d && h->ip6_map.count(key_ip6(ns_id, dhcpv6))) return EMURX_EEXIST;
    if (h->cl[cid].alive) return EMURX_EEXIST;
    ClientInfo& c = h->cl[cid];
    c = ClientInfo();
    c.alive = true;
    c.ns = ns_id;
    c.plugins = plugin_mask;
    memcpy(c.mac, mac, 6);
    memcpy(c.ipv4, ipv4, 4);
    memcpy(c.ipv6, ipv6, 16);
    memcpy(c.dhcpv6, dhcpv6, 16);
    h->mac_map[key_mac(ns_id, mac)] = cid;
    if (has4) h->ip4_map[key_ip4(ns_id, ipv4)] = cid;
    if (has6) h->ip6_map[key_ip6(ns_id, ipv6)] = cid;
    if (has6d) h->ip6_map[key_ip6(ns_id, dhcpv6)] = cid;
    h->ns[ns_id].order.push_back(cid);
    h->dirty = true;
    return EMURX_OK;
}

// CNSCtx.RemoveClient ns_ctx.go:392-440 (map entries are deleted by key)
int emurx_client_remove(emurx_t* h, uint32_t ns_id, const uint8_t mac[6]) {
    if (!h || !mac) return EMURX_EINVAL;
    if (ns_id >= h->cfg.max_ns || !h->ns[ns_id].alive) return EMURX_ENOENT;
    if (zero(mac, 6)) return EMURX_EINVAL;
    auto it = h->mac_map.find(key_mac(ns_id, mac));
    if (it == h->mac_map.end()) return EMURX_ENOENT;
    uint32_t cid = it->second;
    ClientInfo& c = h->cl[cid];
    h->mac_map.erase(it);
    auto& ord = h->ns[ns_id].order;
    ord.erase(std::remove(ord.begin(), ord.end(), cid), ord.end());
    if (!zero(c.ipv4, 4)) h->ip4_map.erase(key_ip4(ns_id, c.ipv4));
    if (!zero(c.ipv6, 16)) h->ip6_map.erase(key_ip6(ns_id, c.ipv6));
    if (!zero(c.dhcpv6, 16)) h->ip6_map.erase(key_ip6(ns_id, c.dhcpv6));
    c.alive = false;
    h->dirty = true;
    return EMURX_OK;
}

int emurx_client_set_plugins(emurx_t* h, uint32_t cid, uint32_t plugin_mask) {
    if (!h) return EMURX_EINVAL;
    if (cid >= h->cfg.max_clients || !h->cl[cid].alive) return EMURX_ENOENT;
    h->cl[cid].plugins = plugin_mask;
    h->dirty = true;
    return EMURX_OK;
}

// CNSCtx.UpdateClientIpv4 / Ipv6 / DIpv6 ns_ctx.go:442-533
static int update_addr(emurx_t* h, uint32_t cid, int which, const uint8_t* nw) {
    if (!h || !nw) return EMURX_EINVAL;
    if (cid >= h->cfg.max_clients || !h->cl[cid].alive) return EMURX_ENOENT;
    ClientInfo& c = h->cl[cid];
    const int n = which == 4 ? 4 : 16;
    uint8_t* cur = which == 4 ? c.ipv4 : (which == 6 ? c.ipv6 : c.dhcpv6);
    Map& m = which == 4 ? h->ip4_map : h->ip6_map;
    auto key = [&](const uint8_t* a) { return which == 4 ? key_ip4(c.ns, a) : key_ip6(c.ns, a); };
    if (!memcmp(cur, nw, n)) return EMURX_OK;
    h->dirty = true;
    if (!zero(cur, n)) {
        auto it = m.find(key(cur));
        if (it == m.end()) { memset(cur, 0, n); return EMURX_ENOENT; }
        m.erase(it);
    }
    if (!zero(nw, n)) {
        if (m.count(key(nw))) { memset(cur, 0, n); return EMURX_EEXIST; }
        m[key(nw)] = cid;
    }
    memcpy(cur, nw, n);
    return EMURX_OK;
}
int emurx_client_update_ipv4(emurx_t* h, uint32_t cid, const uint8_t ipv4[4]) { return update_addr(h, cid, 4, ipv4); }
int emurx_client_update_ipv6(emurx_t* h, uint32_t cid, const uint8_t ipv6[16]) { return update_addr(h, cid, 6, ipv6); }
int emurx_client_update_dipv6(emurx_t* h, uint32_t cid, const uint8_t d[16]) { return update_addr(h, cid, 7, d); }

int emurx_client_set_ra(emurx_t* h, uint32_t cid, const uint8_t prefix[16], uint8_t plen) {
    if (!h || !prefix) return EMURX_EINVAL;
    if (cid >= h->cfg.max_clients || !h->cl[cid].alive) return EMURX_ENOENT;
    ClientInfo& c = h->cl[cid];
    c.has_ra = true;
    memcpy(c.ra_prefix, prefix, 16);
    c.ra_plen = plen;
    h->dirty = true;
    return EMURX_OK;
}

int emurx_sync(emurx_t* h, void* stream) {
    if (!h) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    return rebuild_and_upload(h, stream ? (hipStream_t)stream : h->stream);
}

// ---- data path ---------------------------------------------------------------------------
// the offset walk of VethIFZmq.OnRxStream veth_zmq.go:277-320 (uint16 running offset)
int emurx_zmq_descriptors(const uint8_t* msg, size_t len, emurx_desc* out, uint32_t cap,
                          uint32_t* n_out, int* parse_err) {
    if (!n_out || !parse_err || (len && !msg)) return EMURX_EINVAL;
    *n_out = 0;
    *parse_err = 0;
    const uint32_t blen = (uint32_t)len;
    if (blen < 4) { *parse_err = 1; return EMURX_OK; }
    uint32_t header = be32(msg);
    if ((header >> 16) != EMURX_ZMQ_MAGIC) { *parse_err = 1; return EMURX_OK; }
    const int pkts = (int)(header & 0xffff);
    uint16_t of = 4;
    for (int i = 0; i < pkts; ++i) {
        if (blen < (uint32_t)(uint16_t)(of + 4)) { *parse_err = 1; return EMURX_OK; }
        if ((uint16_t)(of + 4) < of) { *parse_err = 2; return EMURX_OK; }
        header = be32(msg + of);
        if ((header & 0xff000000u) != 0xAA000000u) { *parse_err = 1; return EMURX_OK; }
        const uint8_t vport = (uint8_t)(header >> 16);
        const uint16_t plen = (uint16_t)header;
        if (blen < (uint32_t)(uint16_t)(of + 4 + plen)) { *parse_err = 1; return EMURX_OK; }
        if (plen > EMURX_MAX_FRAME) { *parse_err = 2; return EMURX_OK; }
        if ((uint16_t)(of + 4 + plen) < (uint16_t)(of + 4)) { *parse_err = 2; return EMURX_OK; }
        if (*n_out >= cap) return EMURX_ENOSPC;
        out[*n_out] = emurx_desc{(uint32_t)(uint16_t)(of + 4), plen, vport, 0};
        ++*n_out;
        of = (uint16_t)(of + 4 + plen);
    }
    return EMURX_OK;
}

void emurx_hist_to_counters(const uint64_t hist[2 * EMURX_HIST_BINS], emurx_counters* c) {
    if (!hist || !c) return;
    uint64_t* s = c->parser;
    for (uint32_t st = 0; st < EMURX_NUM_STATUS; ++st) {
        for (uint32_t cb = 0; cb < (st <= EMURX_ST_NOT_SUPPORTED ? (uint32_t)EMURX_NUM_CB : 1u); ++cb) {
            const uint32_t b = st <= EMURX_ST_NOT_SUPPORTED ? EMURX_HIST_BIN(st, cb) : EMURX_HIST_BIN(st, 0);
            const uint64_t pk = hist[2 * b], by = hist[2 * b + 1];
            if (!pk) continue;
            if (st >= EMURX_ST_PANIC_L4LEN) { c->ref_panic += pk; continue; }
            if (st <= EMURX_ST_NOT_SUPPORTED) {
                switch (cb) {  // parser.go:602-713 / :787-799
                case EMURX_CB_ARP: s[EMURX_PC_arpPkts] += pk; s[EMURX_PC_arpBytes] += by; break;
                case EMURX_CB_ICMP: s[EMURX_PC_icmpPkts] += pk; s[EMURX_PC_icmpBytes] += by; break;
                case EMURX_CB_IGMP: s[EMURX_PC_igmpPkts] += pk; s[EMURX_PC_igmpBytes] += by; break;
                case EMURX_CB_TCP: s[EMURX_PC_tcpPkts] += pk; s[EMURX_PC_tcpBytes] += by; break;
                case EMURX_CB_ICMPV6: s[EMURX_PC_Icmpv6Pkt] += pk; s[EMURX_PC_Icmpv6Bytes] += by; break;
                case EMURX_CB_EAPOL: s[EMURX_PC_eapolPkts] += pk; s[EMURX_PC_eapolBytes] += by; break;
                case EMURX_CB_PPP: break;
                default:
                    s[EMURX_PC_udpPkts] += pk; s[EMURX_PC_udpBytes] += by;
                    if (cb == EMURX_CB_MDNS) { s[EMURX_PC_mDnsPkts] += pk; s[EMURX_PC_mDnsBytes] += by; }
                    if (cb == EMURX_CB_DHCP || cb == EMURX_CB_DHCPV6) { s[EMURX_PC_dhcpPkts] += pk; s[EMURX_PC_dhcpBytes] += by; }
                    if (cb == EMURX_CB_DHCPSRV) { s[EMURX_PC_dhcpSrvPkts] += pk; s[EMURX_PC_dhcpSrvBytes] += by; }
                }
                if (st == EMURX_ST_NOT_SUPPORTED) s[EMURX_PC_errParser] += pk;
                continue;
            }
            static const int err_counter[EMURX_NUM_STATUS] = {
                -1, -1, EMURX_PC_errPacketIsTooShort, EMURX_PC_errEAPolTooShort, EMURX_PC_errArpTooShort,
                EMURX_PC_errDot1qTooShort, EMURX_PC_errToManyDot1q, EMURX_PC_errIPv4TooShort,
                EMURX_PC_errIPv4HeaderTooShort, EMURX_PC_errIPv4Fragment, EMURX_PC_errIPv4cs,
                EMURX_PC_errIPv6TooShort, EMURX_PC_errIPv6HopLimitDrop, EMURX_PC_errIPv6Empty,
                EMURX_PC_errIPv6OptJumbo, EMURX_PC_errIPv6Fragment, EMURX_PC_errIcmpv4TooShort,
                EMURX_PC_errIcmpv4Cse, EMURX_PC_errTcpTooShort, EMURX_PC_tcpCsErr, EMURX_PC_errUdpTooShort,
                EMURX_PC_udpCsErr, EMURX_PC_errIcmpv6TooShort, EMURX_PC_errIcmpv6Cse,
                EMURX_PC_errIcmpv6Unsupported, EMURX_PC_errL4ProtoUnsupported,
                EMURX_PC_errL3ProtoUnsupported, -1, -1, -1, -1};
            s[err_counter[st]] += pk;
            s[EMURX_PC_errParser] += pk;  // HandleRxPacket thread_ctx.go:368-369
        }
    }
}

int emurx_classify_dev(emurx_t* h, const uint8_t* d_frames, const emurx_desc* d_desc, uint32_t n,
                       const emurx_dev_out* out, void* stream) {
    return run_dev(h, d_frames, d_desc, n, out, stream, true);
}
int emurx_parse_dev(emurx_t* h, const uint8_t* d_frames, const emurx_desc* d_desc, uint32_t n,
                    const emurx_dev_out* out, void* stream) {
    return run_dev(h, d_frames, d_desc, n, out, stream, false);
}

int emurx_rx_stream(emurx_t* h, const uint8_t* msg, size_t len, emurx_rec* out_rec,
                    uint32_t* out_qlist, uint32_t out_cap, uint32_t* n_out,
                    uint32_t out_qoff[EMURX_NUM_QUEUES + 1], emurx_counters* delta) {
    if (!h || !n_out || !out_qoff || !delta || (len && !msg)) return EMURX_EINVAL;
    memset(delta, 0, sizeof(*delta));
    *n_out = 0;
    int rc = bind(h);
    if (rc) return rc;
    const uint32_t cap = std::max<uint32_t>(std::min(out_cap, h->cfg.max_frames), 1);
    const size_t qcap_max = queue_cap(cap), hist_words = (size_t)EMURX_HIST_SHARDS * 2 * EMURX_HIST_BINS;
    if (h->h_desc.alloc(cap) || h->h_msg.alloc(len + 64) || h->h_qlist.alloc(EMURX_NUM_QUEUES * qcap_max) ||
        h->h_tile_cnt.alloc(ntiles(cap) * 16) || h->h_hist.alloc(hist_words) || h->d_msg.alloc(len + 64) ||
        h->d_desc.alloc(cap) || h->d_rec.alloc(cap) || h->d_qlist.alloc(EMURX_NUM_QUEUES * qcap_max) ||
        h->d_tile_cnt.alloc(ntiles(cap) * 16) || h->d_hist.alloc(hist_words))
        return EMURX_ENOMEM;
    int perr = 0;
    uint32_t n = 0;
    rc = emurx_zmq_descriptors(msg, len, h->h_desc.p, cap, &n, &perr);
    if (rc) return rc;
    delta->rx_batch = 1;  // VethStats.RxBatch veth_zmq.go:278
    if (perr == 1) delta->rx_parse_err = 1;
    if (perr == 2) delta->ref_panic += 1;
    for (uint32_t i = 0; i < n; ++i) {  // VethIFZmq.OnRx veth_zmq.go:233-234
        delta->rx_pkts++;
        delta->rx_bytes += h->h_desc.p[i].len;
    }
    *n_out = n;
    hipStream_t st = h->stream;
    if ((rc = rebuild_and_upload(h, st))) return rc;
    if (n == 0) {
        memset(out_qoff, 0, sizeof(uint32_t) * (EMURX_NUM_QUEUES + 1));
        return EMURX_OK;
    }
    if (!out_rec || !out_qlist) return EMURX_EINVAL;
    memcpy(h->h_msg.p, msg, len);
    memset(h->h_msg.p + len, 0, 64);
    // queue regions sized for this batch, so the whole qlist comes back in one copy
    const uint32_t nt = ntiles(n);
    const size_t qcap = queue_cap(n);
    emurx_dev_out o{h->d_rec.p, h->d_qlist.p, (uint32_t)qcap, h->d_tile_cnt.p, h->d_hist.p};
    bool ok = hipMemcpyAsync(h->d_msg.p, h->h_msg.p, len + 64, hipMemcpyHostToDevice, st) == hipSuccess &&
              hipMemcpyAsync(h->d_desc.p, h->h_desc.p, (size_t)n * sizeof(emurx_desc), hipMemcpyHostToDevice, st) == hipSuccess &&
              hipMemsetAsync(h->d_hist.p, 0, hist_words * sizeof(uint64_t), st) == hipSuccess;
    if (!ok) return EMURX_EDEVICE;
    if ((rc = run_dev(h, h->d_msg.p, h->d_desc.p, n, &o, st, true))) return rc;
    ok = hipMemcpyAsync(out_rec, h->d_rec.p, (size_t)n * sizeof(emurx_rec), hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipMemcpyAsync(h->h_qlist.p, h->d_qlist.p, EMURX_NUM_QUEUES * qcap * 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipMemcpyAsync(h->h_tile_cnt.p, h->d_tile_cnt.p, (size_t)nt * 16 * 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipMemcpyAsync(h->h_hist.p, h->d_hist.p, hist_words * sizeof(uint64_t), hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipStreamSynchronize(st) == hipSuccess;
    if (!ok) return EMURX_EDEVICE;
    // concatenate each queue's per-tile segments (out_qoff[q] .. out_qoff[q+1])
    uint32_t at = 0;
    for (int q = 0; q < EMURX_NUM_QUEUES; ++q) {
        out_qoff[q] = at;
        for (uint32_t t = 0; t < nt; ++t) {
            const uint32_t c = h->h_tile_cnt.p[t * 16 + q];
            if (c > EMURX_QUEUE_TILE || at + c > n) return EMURX_EDEVICE;
            memcpy(out_qlist + at, h->h_qlist.p + q * qcap + (size_t)t * EMURX_QUEUE_TILE, (size_t)c * 4);
            at += c;
        }
    }
    out_qoff[EMURX_NUM_QUEUES] = at;
    if (at != n) return EMURX_EDEVICE;
    uint64_t hist[2 * EMURX_HIST_BINS];
    emurx_hist_fold(h->h_hist.p, hist);
    emurx_hist_to_counters(hist, delta);
    return EMURX_OK;
}

void emurx_hist_fold(const uint64_t* shards, uint64_t out[2 * EMURX_HIST_BINS]) {
    for (int b = 0; b < 2 * EMURX_HIST_BINS; ++b) out[b] = 0;
    if (!shards) return;
    for (int s = 0; s < EMURX_HIST_SHARDS; ++s)
        for (int b = 0; b < 2 * EMURX_HIST_BINS; ++b) out[b] += shards[(size_t)s * 2 * EMURX_HIST_BINS + b];
}

int emurx_set_timing(emurx_t* h, uint32_t slots, uint32_t stride) {
    if (!h) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    (void)hipStreamSynchronize(h->stream);
    (void)hipDeviceSynchronize();
    for (auto& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    h->ev.assign((size_t)slots * 2, nullptr);
    for (auto& e : h->ev)
        if (hipEventCreate(&e) != hipSuccess) { h->slots = 0; return EMURX_EDEVICE; }
    h->slots = slots;
    h->stride = stride ? stride : 1;
    h->ev_head = h->ev_count = h->batch_seq = 0;
    return EMURX_OK;
}

int emurx_kernel_times(emurx_t* h, float* batch_ms, uint32_t cap, uint32_t* n_out) {
    if (!h || !n_out || (cap && !batch_ms)) return EMURX_EINVAL;
    *n_out = 0;
    if (!h->slots || !h->ev_count) return EMURX_OK;
    int rc = bind(h);
    if (rc) return rc;
    const uint32_t last = (h->ev_head + h->slots - 1) % h->slots;
    if (hipEventSynchronize(h->ev[2 * last + 1]) != hipSuccess) return EMURX_EDEVICE;
    const uint32_t n = std::min(h->ev_count, cap);
    const uint32_t first = (h->ev_head + h->slots - h->ev_count) % h->slots;
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t s = (first + (h->ev_count - n) + k) % h->slots;
        if (hipEventElapsedTime(&batch_ms[k], h->ev[2 * s], h->ev[2 * s + 1]) != hipSuccess)
            return EMURX_EDEVICE;
    }
    *n_out = n;
    h->ev_count = 0;
    return EMURX_OK;
}

uint32_t emurx_ns_owner(const uint8_t key[12], uint32_t n_parts) {
    if (!key || n_parts == 0) return 0;
    return emurx_owner(emurx_tk_hash(le32(key), le32(key + 4), le32(key + 8)), n_parts);
}

int emurx_route_dev(emurx_t* h, const emurx_rec* d_rec, uint32_t n, uint32_t n_parts, uint32_t my_rank,
                    uint32_t cap, emurx_route_rec* d_send, uint32_t* d_send_count, void* stream) {
    if (!h || !d_send_count || n_parts == 0 || n_parts > EMURX_MAX_PARTS || my_rank >= n_parts ||
        (n && (!d_rec || !d_send || cap == 0)))
        return EMURX_EINVAL;
    if (((uintptr_t)d_rec & 15) || ((uintptr_t)d_send & 7)) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    const size_t tiles = ((size_t)n + EMURX_QUEUE_TILE - 1) / EMURX_QUEUE_TILE;
    if (tiles > 1024u * 64u) return EMURX_EINVAL;  // 16M frames per batch
    const size_t gw = 1024 * 16;
    if (!h->d_route_grp.p) {
        if (h->d_route_grp.alloc(gw) || hipMemset(h->d_route_grp.p, 0, gw * sizeof(uint32_t)) != hipSuccess)
            return EMURX_ENOMEM;
    }
    if (h->d_route_cnt.alloc(std::max<size_t>(tiles, 1) * 16) || h->d_route_goff.alloc(gw)) return EMURX_ENOMEM;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    return emurx_launch_route(d_rec, n, n_parts, my_rank, cap, d_send, d_send_count, h->d_route_cnt.p,
                              h->d_route_grp.p, h->d_route_goff.p, st)
               ? EMURX_EDEVICE
               : EMURX_OK;
}

}  // extern "C"
