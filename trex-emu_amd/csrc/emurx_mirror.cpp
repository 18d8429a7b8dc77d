// emurx_mirror.cpp — host mirror of the Namespace / Client tables (see emurx_mirror.h).
//
// Go semantics follow src/emu/core/thread_ctx.go:786-812 (AddNs / RemoveNs) and
// src/emu/core/ns_ctx.go:332-533 (AddClient / RemoveClient / UpdateClientIpv4 / Ipv6 / DIpv6);
// the transport maps follow src/emu/plugins/transport/client_ctx.go:597-651 and :1142-1155.
// Every map insert / delete is mirrored onto its device slot in the same call.
#include "emurx_mirror.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace emurx_host {
namespace {

uint32_t pow2_at_least(uint64_t v) {
    uint64_t p = 16;
    while (p < v) p <<= 1;
    return (uint32_t)p;
}
uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
bool zero(const uint8_t* p, int n) {
    for (int i = 0; i < n; ++i)
        if (p[i]) return false;
    return true;
}
K5 key_ns(const uint8_t* k12) { return K5{{le32(k12), le32(k12 + 4), le32(k12 + 8), 0, 0}}; }
K5 key_mac(uint32_t ns, const uint8_t* m) { return K5{{ns, le32(m), (uint32_t)(m[4] | (m[5] << 8)), 0, 0}}; }
K5 key_ip4(uint32_t ns, const uint8_t* ip) { return K5{{ns, le32(ip), 0, 0, 0}}; }
K5 key_ip6(uint32_t ns, const uint8_t* ip) { return K5{{ns, le32(ip), le32(ip + 4), le32(ip + 8), le32(ip + 12)}}; }

}  // namespace

// ---- bucketed image ----------------------------------------------------------------------
void Hash::init(uint32_t nbuckets, uint32_t w) {
    words = w;
    buckets = std::max<uint32_t>(nbuckets, 1);
    resize_blocks(buckets);
    for (size_t i = words - 1; i < img.size(); i += words) img[i] = EMURX_EMPTY;
    live = tomb = 0;
}
uint32_t Hash::put(uint32_t hash, const uint32_t* e) {
    const uint32_t P = per();
    for (uint32_t b = hash & mask(), n = 0; n < buckets; b = (b + 1) & mask(), ++n)
        for (uint32_t k = 0; k < P; ++k) {
            uint32_t* s = &img[(size_t)b * EMURX_BUCKET_WORDS + k * words];
            const uint32_t v = s[words - 1];
            if (v != EMURX_EMPTY && v != EMURX_TOMB) continue;
            if (v == EMURX_TOMB) --tomb;
            memcpy(s, e, words * sizeof(uint32_t));
            ++live;
            touch(b);
            return b * P + k;
        }
    return kNoSlot;  // unreachable: reserve() keeps a quarter of the slots free
}
void Hash::del(uint32_t s) {
    uint32_t* p = at(s);
    for (uint32_t k = 0; k + 1 < words; ++k) p[k] = 0xFFFFFFFFu;
    p[words - 1] = EMURX_TOMB;
    --live;
    ++tomb;
    touch(s / per());
}

// ---- sizing ------------------------------------------------------------------------------
void Mirror::open(uint32_t mns, uint32_t mcl) {
    max_ns = mns;
    max_clients = mcl;
    ns.assign(max_ns, NsInfo());
    cl.assign(max_clients, ClientInfo());
    nsinfo.resize_blocks((uint32_t)(((size_t)max_ns * 4 + EMURX_BUCKET_WORDS - 1) / EMURX_BUCKET_WORDS));
    set_partition(1, 0);
}

Hash* Mirror::hashes(int k) {
    Hash* t[kNumTabs] = {&ns_t, &mac_t, &ip4_t, &ip6_t, &ci_t, &ft4_t, &ft6_t, &srv_t};
    return t[k];
}
bool Mirror::pending() const {
    return nsinfo.pending() || ns_t.pending() || mac_t.pending() || ip4_t.pending() || ip6_t.pending() ||
           ci_t.pending() || ft4_t.pending() || ft6_t.pending() || srv_t.pending();
}
void Mirror::clean_all() {
    nsinfo.clean();
    for (int k = 0; k < kNumTabs; ++k) hashes(k)->clean();
}

// Slots per entry by table (ns, mac, ip4, ip6, ci, ft4, ft6, srv).  A wave's lookups take as
// many dependent memory trips as the longest probe chain among its 64 lanes; at load 1/2,
// 93 % of 64-lane waves hold a key outside its 4-slot home bucket (2-slot buckets: all of
// them), at 1/8 (1/16 for 2 slots) about 2 % (4 %).  EMURX_TABLE_SPREAD="ns,mac,ip,ci"
// overrides the first five (the ip value for both IP tables), for measurements.
namespace {
struct Spread {
    uint32_t v[kNumTabs] = {8, 8, 16, 16, 16, 16, 32, 8};
    Spread() {
        const char* s = getenv("EMURX_TABLE_SPREAD");
        unsigned a = 0, b = 0, c = 0, d = 0;
        if (!s || sscanf(s, "%u,%u,%u,%u", &a, &b, &c, &d) != 4) return;
        const unsigned w[5] = {a, b, c, c, d};
        for (int k = 0; k < 5; ++k)
            if (w[k] >= 2 && w[k] <= 64 && !(w[k] & (w[k] - 1))) v[k] = w[k];
    }
};
const uint32_t* table_spread() {
    static const Spread s;
    return s.v;
}
constexpr uint64_t kSpreadCap = 2ull << 30;  // bytes per table
}  // namespace

// Every table starts at its target load (1 / spread) for its share of max_ns / max_clients
// (the whole of them with one partition, 1/n of them plus slack with n) and grows on demand.
void Mirror::set_partition(uint32_t n, uint32_t p) {
    n_parts = std::max<uint32_t>(n, 1);
    part = p;
    for (auto& kv : ns_map) {
        NsInfo& s = ns[kv.second.id];
        s.owned = n_parts == 1 || emurx_owner(emurx_tk_hash(kv.first.w[0], kv.first.w[1], kv.first.w[2]), n_parts) == part;
    }
    // a partition's fair share (load <= 1/2 then; the owner hash's imbalance, a few percent,
    // is absorbed below the 3/4 rebuild threshold, and a partition that receives far more grows)
    const uint64_t ens = std::max<uint64_t>(((uint64_t)max_ns + n_parts - 1) / n_parts, 16);
    const uint64_t ecl = std::max<uint64_t>(((uint64_t)max_clients + n_parts - 1) / n_parts, 64);
    // entries each table holds now (all of them: a rebuild re-filters by the new partition)
    const uint64_t live[kNumTabs] = {ns_map.size(), mac_map.size(), ip4_map.size(), ip6_map.size(),
                                     mac_map.size(), 0, 0, srv_map.size()};
    uint64_t f4 = 0;
    for (auto& kv : ft_map) f4 += kv.first.size() == 4 + 13;
    const uint64_t need[kNumTabs] = {live[0], live[1], live[2], live[3], live[4], f4, ft_map.size() - f4, live[7]};
    // IPv6: one address per client to start (a client may hold two, Ipv6 and Dhcpv6: the
    // table grows when they come)
    const uint64_t want[kNumTabs] = {ens, ecl, ecl, ecl, ecl, 8, 8, 16};
    const uint32_t per[kNumTabs] = {4, 4, 2, 2, 2, 2, 1, 4};
    const uint32_t* sp = table_spread();
    for (int k = 0; k < kNumTabs; ++k) {
        const uint64_t e = std::max(want[k], (need[k] + n_parts - 1) / n_parts);
        // sparser tables cost bytes, not lookups; above kSpreadCap a table falls back towards
        // the load of 1/2
        uint32_t s = sp[k];
        while (s > 2 && (uint64_t)pow2_at_least((uint64_t)s * e) * (EMURX_BUCKET_WORDS / per[k]) * 4 > kSpreadCap)
            s >>= 1;
        hashes(k)->spread = s;
        rebuild(k, std::max<uint32_t>(pow2_at_least((uint64_t)s * e) / per[k], 1));
    }
    nsinfo.resize_blocks(nsinfo.nblocks());
    for (uint32_t i = 0; i < max_ns; ++i)
        if (ns[i].alive) put_nsinfo(i);
    n_ctx = n_ctx_all = 0;
    for (uint32_t c = 0; c < max_clients; ++c)
        if (cl[c].alive && cl[c].has_ctx) {
            ++n_ctx_all;
            if (owned_ns(cl[c].ns)) ++n_ctx;
        }
}

// The table sized from its LIVE entries at half the spread (not the old bucket count halved: a
// table grown to ~2 / spread, e.g. IPv6 sized for one address per client that then got both
// Ipv6 and Dhcpv6, would land at load 1), never past the 3/4 bound Hash::put relies on with one
// more insert; false when that is no smaller than the table whose allocation failed (ENOMEM)
bool Mirror::shrink(int k) {
    Hash& t = *hashes(k);
    const uint32_t per = t.per();
    for (uint32_t sp = t.spread >> 1; sp >= 2; sp >>= 1) {  // the first denser spread that is smaller
        uint64_t slots = pow2_at_least(std::max<uint64_t>((uint64_t)sp * t.live, per));
        while ((uint64_t)(t.live + 1) * 4 > slots * 3) slots *= 2;
        const uint64_t nb = std::max<uint64_t>(slots / per, 1);
        if (nb >= t.buckets) continue;
        t.spread = sp;
        rebuild(k, (uint32_t)nb);
        return true;
    }
    return false;
}

uint32_t Mirror::tk_of(uint32_t ns_id) const {
    const uint8_t* k = ns[ns_id].key;
    return emurx_tk_hash(le32(k), le32(k + 4), le32(k + 8));
}

void Mirror::put_nsinfo(uint32_t id) {
    const NsInfo& n = ns[id];
    uint32_t* o = &nsinfo.img[(size_t)id * 4];
    const bool on = n.alive && n.owned;
    o[0] = on ? n.plugins : 0;
    o[1] = (on && !n.order.empty()) ? n.order.front() : EMURX_ID_NONE;
    nsinfo.touch_word((size_t)id * 4);
}

// ---- slot contents (emurx_tables.h) --------------------------------------------------------
void Mirror::ns_slot_put(const K5& k, Entry& e) {
    e.slot = kNoSlot;
    // a key with non-zero bytes [2:4] never equals a parsed CTunnelKey (Set writes 0 there,
    // thread_ctx.go:93): no device slot.  The vport word's free upper half carries the
    // Namespace's plugin mask, so one probe answers GetNs + ns.PluginCtx.Get.
    if (!owned_ns(e.id) || (k.w[0] >> 16)) return;
    const uint32_t s[4] = {k.w[0] | (ns[e.id].plugins << 16), k.w[1], k.w[2], e.id};
    e.slot = ns_t.put(emurx_tk_hash(k.w[0], k.w[1], k.w[2]), s);
    ns[e.id].slot = e.slot;
}
// the client's MAC and plugin mask ride in the MAC slot's free upper half and in the IP
// slots' spare words: PluginCtx.Get and IsUnicastToMe need no second read
// the upper half of a client slot's MAC word: the plugin mask and, in its top bit
// (EMURX_CPL_CTX), whether the client has a TransportCtx (the transport flow rule reads it
// from the MAC slot it has already loaded instead of the client-info table)
static uint32_t slot_half(const ClientInfo& c) { return (c.plugins & 0x7fffu) | (c.has_ctx ? EMURX_CPL_CTX : 0u); }
static void mac_words(const ClientInfo& c, uint32_t& lo, uint32_t& hip) {
    lo = le32(c.mac);
    hip = (uint32_t)(c.mac[4] | (c.mac[5] << 8)) | (slot_half(c) << 16);
}
void Mirror::mac_slot_put(const K5& k, Entry& e) {
    e.slot = kNoSlot;
    if (!owned_ns(k.w[0])) return;
    const uint32_t s[4] = {k.w[0], k.w[1], k.w[2] | (slot_half(cl[e.id]) << 16), e.id};
    e.slot = mac_t.put(emurx_mac_hash(tk_of(k.w[0]), k.w[1], k.w[2]), s);
}
void Mirror::ip4_slot_put(const K5& k, Entry& e) {
    e.slot = kNoSlot;
    if (!owned_ns(k.w[0])) return;
    uint32_t s[8] = {k.w[0], k.w[1], 0, 0, 0, 0, 0, e.id};
    mac_words(cl[e.id], s[2], s[3]);
    e.slot = ip4_t.put(emurx_ip4_hash(tk_of(k.w[0]), k.w[1]), s);
}
void Mirror::ip6_slot_put(const K5& k, Entry& e) {
    e.slot = kNoSlot;
    if (!owned_ns(k.w[0])) return;
    uint32_t s[8] = {k.w[0], k.w[1], k.w[2], k.w[3], k.w[4], 0, 0, e.id};
    mac_words(cl[e.id], s[5], s[6]);
    e.slot = ip6_t.put(emurx_ip6_hash(tk_of(k.w[0]), k.w[1], k.w[2], k.w[3], k.w[4]), s);
}
void Mirror::ci_put(uint32_t cid) {
    ClientInfo& c = cl[cid];
    c.ci_slot = kNoSlot;
    if (!c.alive || !owned_ns(c.ns)) return;
    const uint32_t s[8] = {cid, c.plugins, (c.has_ra ? 1u : 0u) | ((uint32_t)c.ra_plen << 8), le32(c.ra_prefix),
                           le32(c.ra_prefix + 4), c.has_ctx ? 1u : 0u, 0, 0};
    c.ci_slot = ci_t.put(emurx_ci_hash(cid), s);
}
void Mirror::ft_slot_put(const std::string& key, Entry& e) {
    e.slot = kNoSlot;
    const uint8_t* k = reinterpret_cast<const uint8_t*>(key.data());
    const uint32_t cid = le32(k);
    if (!owned_ns(cl[cid].ns)) return;
    const uint8_t* t = k + 4;
    if (key.size() == 4 + 13) {
        const uint32_t s[8] = {cid, le32(t), le32(t + 4), le32(t + 8), t[12], 0, 0, e.id};
        e.slot = ft4_t.put(emurx_ft4_hash(cid, s[1], s[2], s[3], s[4]), s);
    } else {
        uint32_t s[16] = {cid};
        for (int j = 0; j < 4; ++j) {
            s[1 + j] = le32(t + 4 * j);
            s[5 + j] = le32(t + 16 + 4 * j);
        }
        s[9] = le32(t + 32);
        s[10] = t[36];
        s[15] = e.id;
        e.slot = ft6_t.put(emurx_ft6_hash(cid, s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9], s[10]), s);
    }
}
void Mirror::srv_slot_put(uint64_t k, Entry& e) {
    e.slot = kNoSlot;
    const uint32_t cid = (uint32_t)(k >> 32);
    if (!owned_ns(cl[cid].ns)) return;
    const uint32_t s[4] = {cid, (uint32_t)k, 0, 1};
    e.slot = srv_t.put(emurx_srv_hash(s[0], s[1]), s);
}
void Mirror::drop(Hash& t, Entry& e) {
    if (e.slot != kNoSlot) t.del(e.slot);
    e.slot = kNoSlot;
}

void Mirror::rebuild(int which, uint32_t nb) {
    switch (which) {
    case kTabNs:
        ns_t.init(nb, 4);
        for (auto& n : ns) n.slot = kNoSlot;
        for (auto& kv : ns_map) ns_slot_put(kv.first, kv.second);
        break;
    case kTabMac:
        mac_t.init(nb, 4);
        for (auto& kv : mac_map) mac_slot_put(kv.first, kv.second);
        break;
    case kTabIp4:
        ip4_t.init(nb, 8);
        for (auto& kv : ip4_map) ip4_slot_put(kv.first, kv.second);
        break;
    case kTabIp6:
        ip6_t.init(nb, 8);
        for (auto& kv : ip6_map) ip6_slot_put(kv.first, kv.second);
        break;
    case kTabCi:
        ci_t.init(nb, 8);
        for (uint32_t c = 0; c < max_clients; ++c) ci_put(c);
        break;
    case kTabFt4:
    case kTabFt6: {
        Hash& t = which == kTabFt4 ? ft4_t : ft6_t;
        t.init(nb, which == kTabFt4 ? 8 : 16);
        for (auto& kv : ft_map)
            if ((kv.first.size() == 4 + 13) == (which == kTabFt4)) ft_slot_put(kv.first, kv.second);
        break;
    }
    case kTabSrv:
        srv_t.init(nb, 4);
        for (auto& kv : srv_map) srv_slot_put(kv.first, kv.second);
        break;
    }
}
void Mirror::reserve(Hash& t, int which, uint32_t k) {
    if (!t.full(k)) return;
    rebuild(which, t.next_buckets(k));
}

// ---- Go map operations ---------------------------------------------------------------------
// CThreadCtx.AddNs thread_ctx.go:786-795
int Mirror::ns_add(const uint8_t key[12], uint32_t id, uint32_t plugins) {
    if (id >= max_ns) return EMURX_ENOMEM;
    const K5 k = key_ns(key);
    if (ns_map.count(k) || ns[id].alive) return EMURX_EEXIST;
    reserve(ns_t, kTabNs);
    NsInfo& n = ns[id];
    n.alive = true;
    memcpy(n.key, key, 12);
    n.plugins = plugins;
    n.order.clear();
    n.owned = n_parts == 1 || emurx_owner(emurx_tk_hash(k.w[0], k.w[1], k.w[2]), n_parts) == part;
    Entry& e = ns_map[k];
    e.id = id;
    ns_slot_put(k, e);
    put_nsinfo(id);
    touch_ns(id);
    return EMURX_OK;
}
// CThreadCtx.RemoveNs thread_ctx.go:797-812 (refused while clients are active)
int Mirror::ns_remove(const uint8_t key[12]) {
    const K5 k = key_ns(key);
    auto it = ns_map.find(k);
    if (it == ns_map.end()) return EMURX_ENOENT;
    const uint32_t id = it->second.id;
    NsInfo& n = ns[id];
    if (!n.order.empty()) return EMURX_EEXIST;
    drop(ns_t, it->second);
    ns_map.erase(it);
    n.alive = false;
    n.slot = kNoSlot;
    put_nsinfo(id);
    touch_ns(id);
    if (removed.size() >= (1u << 16)) {  // forget old removals: older snapshots count as stale
        removed.clear();
        removed_floor = gen;
    }
    removed[k] = gen;
    return EMURX_OK;
}
int Mirror::ns_set_plugins(uint32_t id, uint32_t plugins) {
    if (id >= max_ns || !ns[id].alive) return EMURX_ENOENT;
    NsInfo& n = ns[id];
    n.plugins = plugins;
    if (n.slot != kNoSlot) ns_t.rewrite(n.slot, 0, (ns_t.at(n.slot)[0] & 0xffffu) | (plugins << 16));
    put_nsinfo(id);
    touch_ns(id);
    return EMURX_OK;
}

// CNSCtx.AddClient ns_ctx.go:332-389
int Mirror::client_add(uint32_t ns_id, uint32_t cid, const uint8_t mac[6], const uint8_t ipv4[4],
                       const uint8_t ipv6[16], const uint8_t dhcpv6[16], uint32_t plugins) {
    static const uint8_t z[16] = {0};
    if (ns_id >= max_ns || !ns[ns_id].alive) return EMURX_ENOENT;
    if (cid >= max_clients) return EMURX_ENOMEM;
    if (!ipv4) ipv4 = z;
    if (!ipv6) ipv6 = z;
    if (!dhcpv6) dhcpv6 = z;
    if (zero(mac, 6)) return EMURX_EINVAL;
    if (mac_map.count(key_mac(ns_id, mac))) return EMURX_EEXIST;
    const bool has4 = !zero(ipv4, 4), has6 = !zero(ipv6, 16), has6d = !zero(dhcpv6, 16);
    if (has4 && ip4_map.count(key_ip4(ns_id, ipv4))) return EMURX_EEXIST;
    if (has6 && ip6_map.count(key_ip6(ns_id, ipv6))) return EMURX_EEXIST;
    if (has6d && ip6_map.count(key_ip6(ns_id, dhcpv6))) return EMURX_EEXIST;
    if (cl[cid].alive) return EMURX_EEXIST;
    reserve(mac_t, kTabMac);
    reserve(ip4_t, kTabIp4);
    reserve(ip6_t, kTabIp6, 2);
    reserve(ci_t, kTabCi);
    ClientInfo& c = cl[cid];
    c = ClientInfo();
    c.alive = true;
    c.ns = ns_id;
    c.plugins = plugins;
    memcpy(c.mac, mac, 6);
    memcpy(c.ipv4, ipv4, 4);
    memcpy(c.ipv6, ipv6, 16);
    memcpy(c.dhcpv6, dhcpv6, 16);
    auto put = [&](Map& m, const K5& k, void (Mirror::*fn)(const K5&, Entry&)) {
        auto it = m.find(k);
        if (it != m.end()) {  // the same address twice (Ipv6 == Dhcpv6): one map entry
            it->second.id = cid;
            return;
        }
        Entry& e = m[k];
        e.id = cid;
        (this->*fn)(k, e);
    };
    put(mac_map, key_mac(ns_id, mac), &Mirror::mac_slot_put);
    if (has4) put(ip4_map, key_ip4(ns_id, ipv4), &Mirror::ip4_slot_put);
    if (has6) put(ip6_map, key_ip6(ns_id, ipv6), &Mirror::ip6_slot_put);
    if (has6d) put(ip6_map, key_ip6(ns_id, dhcpv6), &Mirror::ip6_slot_put);
    ci_put(cid);
    ns[ns_id].order.push_back(cid);  // clientHead.AddLast
    if (ns[ns_id].order.size() == 1) put_nsinfo(ns_id);
    touch_ns(ns_id);
    return EMURX_OK;
}

void Mirror::drop_transport(uint32_t cid) {
    for (auto it = ft_map.begin(); it != ft_map.end();) {
        if (le32(reinterpret_cast<const uint8_t*>(it->first.data())) == cid) {
            drop(it->first.size() == 4 + 13 ? ft4_t : ft6_t, it->second);
            it = ft_map.erase(it);
        } else {
            ++it;
        }
    }
    for (auto it = srv_map.begin(); it != srv_map.end();) {
        if ((uint32_t)(it->first >> 32) == cid) {
            drop(srv_t, it->second);
            it = srv_map.erase(it);
        } else {
            ++it;
        }
    }
    ClientInfo& c = cl[cid];
    if (c.has_ctx && owned_ns(c.ns)) --n_ctx;
    if (c.has_ctx) --n_ctx_all;
    c.has_ctx = false;
}

// CNSCtx.RemoveClient ns_ctx.go:392-440 (map entries are deleted by key)
int Mirror::client_remove(uint32_t ns_id, const uint8_t mac[6]) {
    if (ns_id >= max_ns || !ns[ns_id].alive) return EMURX_ENOENT;
    if (zero(mac, 6)) return EMURX_EINVAL;
    auto it = mac_map.find(key_mac(ns_id, mac));
    if (it == mac_map.end()) return EMURX_ENOENT;
    const uint32_t cid = it->second.id;
    ClientInfo& c = cl[cid];
    drop(mac_t, it->second);
    mac_map.erase(it);
    auto& ord = ns[ns_id].order;
    const bool front = !ord.empty() && ord.front() == cid;
    ord.erase(std::remove(ord.begin(), ord.end(), cid), ord.end());
    auto erase = [&](Map& m, Hash& t, const K5& k) {
        auto f = m.find(k);
        if (f == m.end()) return;
        drop(t, f->second);
        m.erase(f);
    };
    if (!zero(c.ipv4, 4)) erase(ip4_map, ip4_t, key_ip4(ns_id, c.ipv4));
    if (!zero(c.ipv6, 16)) erase(ip6_map, ip6_t, key_ip6(ns_id, c.ipv6));
    if (!zero(c.dhcpv6, 16)) erase(ip6_map, ip6_t, key_ip6(ns_id, c.dhcpv6));
    drop_transport(cid);  // TransportCtx.onRemove: its sockets go with the client
    if (c.ci_slot != kNoSlot) ci_t.del(c.ci_slot);
    c.ci_slot = kNoSlot;
    c.alive = false;
    if (front) put_nsinfo(ns_id);
    touch_ns(ns_id);
    return EMURX_OK;
}

// the plugin mask rides in every slot of the client
void Mirror::rewrite_client_slots(uint32_t cid) {
    ClientInfo& c = cl[cid];
    uint32_t lo, hip;
    mac_words(c, lo, hip);
    auto mine = [&](Map& m, const K5& k) -> Entry* {
        auto f = m.find(k);
        return f != m.end() && f->second.id == cid && f->second.slot != kNoSlot ? &f->second : nullptr;
    };
    if (Entry* e = mine(mac_map, key_mac(c.ns, c.mac))) mac_t.rewrite(e->slot, 2, hip);
    if (!zero(c.ipv4, 4))
        if (Entry* e = mine(ip4_map, key_ip4(c.ns, c.ipv4))) ip4_t.rewrite(e->slot, 3, hip);
    if (!zero(c.ipv6, 16))
        if (Entry* e = mine(ip6_map, key_ip6(c.ns, c.ipv6))) ip6_t.rewrite(e->slot, 6, hip);
    if (!zero(c.dhcpv6, 16))
        if (Entry* e = mine(ip6_map, key_ip6(c.ns, c.dhcpv6))) ip6_t.rewrite(e->slot, 6, hip);
    if (c.ci_slot != kNoSlot) {
        ci_t.rewrite(c.ci_slot, 1, c.plugins);
        ci_t.rewrite(c.ci_slot, 2, (c.has_ra ? 1u : 0u) | ((uint32_t)c.ra_plen << 8));
        ci_t.rewrite(c.ci_slot, 3, le32(c.ra_prefix));
        ci_t.rewrite(c.ci_slot, 4, le32(c.ra_prefix + 4));
        ci_t.rewrite(c.ci_slot, 5, c.has_ctx ? 1u : 0u);
    }
}
int Mirror::client_set_plugins(uint32_t cid, uint32_t plugins) {
    if (cid >= max_clients || !cl[cid].alive) return EMURX_ENOENT;
    cl[cid].plugins = plugins;
    rewrite_client_slots(cid);
    touch_ns(cl[cid].ns);
    return EMURX_OK;
}

// CNSCtx.UpdateClientIpv4 / Ipv6 / DIpv6 ns_ctx.go:442-533
int Mirror::update_addr(uint32_t cid, int which, const uint8_t* nw) {
    if (cid >= max_clients || !cl[cid].alive) return EMURX_ENOENT;
    ClientInfo& c = cl[cid];
    const int n = which == 4 ? 4 : 16;
    uint8_t* cur = which == 4 ? c.ipv4 : (which == 6 ? c.ipv6 : c.dhcpv6);
    Map& m = which == 4 ? ip4_map : ip6_map;
    Hash& t = which == 4 ? ip4_t : ip6_t;
    auto key = [&](const uint8_t* a) { return which == 4 ? key_ip4(c.ns, a) : key_ip6(c.ns, a); };
    if (!memcmp(cur, nw, n)) return EMURX_OK;
    touch_ns(c.ns);
    if (!zero(nw, n)) reserve(t, which == 4 ? kTabIp4 : kTabIp6);
    if (!zero(cur, n)) {
        auto it = m.find(key(cur));
        if (it == m.end()) {
            memset(cur, 0, n);
            return EMURX_ENOENT;
        }
        drop(t, it->second);
        m.erase(it);
    }
    if (!zero(nw, n)) {
        if (m.count(key(nw))) {
            memset(cur, 0, n);
            return EMURX_EEXIST;
        }
        Entry& e = m[key(nw)];
        e.id = cid;
        if (which == 4) ip4_slot_put(key(nw), e);
        else ip6_slot_put(key(nw), e);
    }
    memcpy(cur, nw, n);
    return EMURX_OK;
}

int Mirror::client_set_ra(uint32_t cid, const uint8_t prefix[16], uint8_t plen) {
    if (cid >= max_clients || !cl[cid].alive) return EMURX_ENOENT;
    ClientInfo& c = cl[cid];
    c.has_ra = true;
    memcpy(c.ra_prefix, prefix, 16);
    c.ra_plen = plen;
    rewrite_client_slots(cid);
    touch_ns(c.ns);
    return EMURX_OK;
}

// ---- transport (TransportCtx.addFlowv4/6 / removeFlowv4/6 client_ctx.go:597-651, serverCb
// lookupServerPort :1142-1155, GetTransportCtx socketApi.go:174-193) ------------------------
int Mirror::client_set_transport(uint32_t cid, bool has) {
    if (cid >= max_clients || !cl[cid].alive) return EMURX_ENOENT;
    ClientInfo& c = cl[cid];
    if (c.has_ctx != has && owned_ns(c.ns)) n_ctx += has ? 1 : -1;
    if (c.has_ctx != has) n_ctx_all += has ? 1 : -1;
    c.has_ctx = has;
    rewrite_client_slots(cid);
    touch_ns(c.ns);
    return EMURX_OK;
}
int Mirror::flow_add(uint32_t cid, const uint8_t* tuple, uint32_t tlen, uint32_t flow) {
    if (!tuple || (tlen != 13 && tlen != 37)) return EMURX_EINVAL;
    if (cid >= max_clients || !cl[cid].alive) return EMURX_ENOENT;
    if (flow > EMURX_FLOW_ID_MAX) return EMURX_EINVAL;
    std::string k(4 + tlen, '\0');
    memcpy(&k[0], &cid, 4);
    memcpy(&k[4], tuple, tlen);
    if (ft_map.count(k)) return EMURX_EEXIST;  // ft_add_err_already_exits
    if (tlen == 13) reserve(ft4_t, kTabFt4);
    else reserve(ft6_t, kTabFt6);
    Entry& e = ft_map[k];
    e.id = flow;
    ft_slot_put(k, e);
    client_set_transport(cid, true);
    return EMURX_OK;
}
int Mirror::flow_remove(uint32_t cid, const uint8_t* tuple, uint32_t tlen) {
    if (!tuple || (tlen != 13 && tlen != 37)) return EMURX_EINVAL;
    if (cid >= max_clients || !cl[cid].alive) return EMURX_ENOENT;
    std::string k(4 + tlen, '\0');
    memcpy(&k[0], &cid, 4);
    memcpy(&k[4], tuple, tlen);
    auto it = ft_map.find(k);
    if (it == ft_map.end()) return EMURX_ENOENT;  // ft_remove_err_not_exits
    drop(tlen == 13 ? ft4_t : ft6_t, it->second);
    ft_map.erase(it);
    touch_ns(cl[cid].ns);
    return EMURX_OK;
}
int Mirror::server_add(uint32_t cid, uint16_t port, uint8_t proto) {
    if (proto != 6 && proto != 17) return EMURX_EINVAL;
    if (cid >= max_clients || !cl[cid].alive) return EMURX_ENOENT;
    const uint64_t k = ((uint64_t)cid << 32) | port | ((uint32_t)proto << 16);
    if (srv_map.count(k)) return EMURX_EEXIST;
    reserve(srv_t, kTabSrv);
    Entry& e = srv_map[k];
    e.id = 1;
    srv_slot_put(k, e);
    client_set_transport(cid, true);
    return EMURX_OK;
}
int Mirror::server_remove(uint32_t cid, uint16_t port, uint8_t proto) {
    if (proto != 6 && proto != 17) return EMURX_EINVAL;
    if (cid >= max_clients || !cl[cid].alive) return EMURX_ENOENT;
    auto it = srv_map.find(((uint64_t)cid << 32) | port | ((uint32_t)proto << 16));
    if (it == srv_map.end()) return EMURX_ENOENT;
    drop(srv_t, it->second);
    srv_map.erase(it);
    touch_ns(cl[cid].ns);
    return EMURX_OK;
}

// ---- mid-batch rule -------------------------------------------------------------------------
bool Mirror::stale(const emurx_rec& r, uint64_t since) const {
    if (since >= gen || r.status != EMURX_ST_OK) return false;  // nothing changed / no lookup ran
    const K5 k{{r.vport, r.vlan[0], r.vlan[1], 0, 0}};        // CTunnelKey words (thread_ctx.go:92-97)
    auto it = ns_map.find(k);
    if (it != ns_map.end() && ns[it->second.id].gen > since) return true;
    if (since < removed_floor) return true;
    auto rm = removed.find(k);
    return rm != removed.end() && rm->second > since;
}

// ---- the device walk over the host image (tests of the table maintenance) -------------------
int Mirror::image_lookup(uint32_t table, const uint32_t* key, uint32_t* value) {
    if (table >= kNumTabs || !key || !value) return EMURX_EINVAL;
    Hash& t = *hashes((int)table);
    uint32_t h = 0, nk = 0;
    uint32_t kw[11] = {0};
    switch (table) {
    case kTabNs: h = emurx_tk_hash(key[0], key[1], key[2]); nk = 3; break;
    case kTabMac:
        if (key[0] >= max_ns || !ns[key[0]].alive) return EMURX_ENOENT;
        h = emurx_mac_hash(tk_of(key[0]), key[1], key[2]); nk = 3; break;
    case kTabIp4:
        if (key[0] >= max_ns || !ns[key[0]].alive) return EMURX_ENOENT;
        h = emurx_ip4_hash(tk_of(key[0]), key[1]); nk = 2; break;
    case kTabIp6:
        if (key[0] >= max_ns || !ns[key[0]].alive) return EMURX_ENOENT;
        h = emurx_ip6_hash(tk_of(key[0]), key[1], key[2], key[3], key[4]); nk = 5; break;
    case kTabCi: h = emurx_ci_hash(key[0]); nk = 1; break;
    case kTabFt4: h = emurx_ft4_hash(key[0], key[1], key[2], key[3], key[4]); nk = 5; break;
    case kTabFt6:
        h = emurx_ft6_hash(key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7], key[8], key[9], key[10]);
        nk = 11; break;
    case kTabSrv: h = emurx_srv_hash(key[0], key[1]); nk = 2; break;
    }
    memcpy(kw, key, nk * 4);
    for (uint32_t b = h & t.mask(), n = 0; n < t.buckets; b = (b + 1) & t.mask(), ++n) {
        bool hole = false;
        for (uint32_t k = 0; k < t.per(); ++k) {
            const uint32_t* s = &t.img[(size_t)b * EMURX_BUCKET_WORDS + k * t.words];
            const uint32_t v = s[t.words - 1];
            if (v == EMURX_EMPTY) { hole = true; continue; }
            if (v == EMURX_TOMB) continue;
            bool eq = true;
            for (uint32_t j = 0; j < nk && eq; ++j) {
                uint32_t x = s[j];
                if ((table == kTabNs && j == 0) || (table == kTabMac && j == 2)) x &= 0xffffu;  // plugin halves
                eq = x == kw[j];
            }
            if (eq) {
                *value = table == kTabCi ? s[1] : v;  // client info: its plugin mask
                return EMURX_OK;
            }
        }
        if (hole) break;
    }
    return EMURX_ENOENT;
}

}  // namespace emurx_host
