// emurx_mirror.h — host side of the Namespace / Client tables.
//
// The mirror keeps the reference's Go maps with their exact semantics (return codes of
// AddNs / AddClient / UpdateClient* ...) AND the image of every device table in the layout of
// emurx_tables.h.  Each mutation edits the image slot by slot and marks the 64-byte blocks it
// touched; emurx_api.cpp ships only those blocks to the device (emurx_delta) before the next
// batch.  Deleted slots become tombstones (key words 0xFFFFFFFF, value EMURX_TOMB): a probe
// walks past them and never matches them, so a chain stays intact without moving entries.
// A table whose live + tombstone slots pass 3/4 is rebuilt (doubled when live passes 1/2)
// and shipped whole.
//
// Partitioned mode (set_partition): the maps stay complete (Go semantics do not change), but
// the device images hold only the Namespaces this partition owns (emurx_owner of their
// CTunnelKey) and those Namespaces' clients, flows and listeners.
//
// Generations: every mutation advances `gen` and stamps the Namespace it touched.  A record
// classified against the tables as they stood at generation g is stale iff its Namespace
// (found by its tunnel key now, or removed since) was stamped after g.
//
// No HIP here: host-only handles (cfg.device < 0) use the mirror alone.
#pragma once
#include <stdint.h>

#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/emu_rx.h"
#include "emurx_tables.h"

namespace emurx_host {

constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

// table keys: (ns_id or tunnel-key words, address words) — the per-Namespace Go maps flattened
struct K5 {
    uint32_t w[5];
    bool operator==(const K5& o) const { return !memcmp(w, o.w, sizeof(w)); }
};
struct K5Hash {
    size_t operator()(const K5& k) const { return emurx_hash(k.w[0], k.w[1], k.w[2], k.w[3], k.w[4]); }
};
struct Entry {
    uint32_t id;    // ns id / client id / flow id
    uint32_t slot;  // device slot index, kNoSlot when not on this partition's device
};
using Map = std::unordered_map<K5, Entry, K5Hash>;

// image of a device array of 64-byte blocks + the blocks edited since the last upload
struct Blocks {
    std::vector<uint32_t> img;
    std::vector<uint32_t> dirty;
    std::vector<uint8_t> mark;
    bool all = true;  // ship the whole image (first upload, rebuild, growth)
    uint32_t nblocks() const { return (uint32_t)(img.size() / EMURX_BUCKET_WORDS); }
    void resize_blocks(uint32_t blocks) {
        img.assign((size_t)blocks * EMURX_BUCKET_WORDS, 0);
        mark.assign(blocks, 0);
        dirty.clear();
        all = true;
    }
    void touch(uint32_t block) {
        if (all || mark[block]) return;
        mark[block] = 1;
        dirty.push_back(block);
    }
    void touch_word(size_t w) { touch((uint32_t)(w / EMURX_BUCKET_WORDS)); }
    bool pending() const { return all || !dirty.empty(); }
    void clean() {
        for (uint32_t b : dirty) mark[b] = 0;
        dirty.clear();
        all = false;
    }
};

// open addressing over 64-byte buckets (emurx_tables.h), slots of `words` words.
// `spread` is the table's target of slots per live entry (a power of two >= 2): a lookup's
// wave waits for the longest probe chain among its 64 lanes, so the tables are kept sparse
// enough that almost every key sits in its home bucket (emurx_table_spread).
struct Hash : Blocks {
    uint32_t words = 4, buckets = 0, live = 0, tomb = 0, spread = 2;
    uint32_t per() const { return EMURX_BUCKET_WORDS / words; }
    uint32_t nslots() const { return buckets * per(); }
    uint32_t mask() const { return buckets - 1; }
    uint32_t* at(uint32_t s) { return &img[(size_t)(s / per()) * EMURX_BUCKET_WORDS + (s % per()) * words]; }
    void init(uint32_t nbuckets, uint32_t w);
    // first empty or tombstone slot in bucket order from the home bucket
    uint32_t put(uint32_t hash, const uint32_t* e);
    void del(uint32_t s);
    void rewrite(uint32_t s, uint32_t word, uint32_t v) {
        at(s)[word] = v;
        touch(s / per());
    }
    // k more inserts would take live + tombstones past 2 / spread of the slots (3/4 at
    // spread 2): twice the target load, then a rebuild drops the tombstones
    bool full(uint32_t k = 1) const {
        const uint64_t used = (uint64_t)live + tomb + k;
        return spread <= 2 ? used * 4 > (uint64_t)nslots() * 3 : used * spread > (uint64_t)nslots() * 2;
    }
    // bucket count for a rebuild: doubled once live would pass the target load 1 / spread
    uint32_t next_buckets(uint32_t k = 1) const {
        return (uint64_t)(live + k) * spread > nslots() ? buckets * 2 : buckets;
    }
};

struct NsInfo {
    bool alive = false;
    bool owned = false;
    uint8_t key[12] = {0};
    uint32_t plugins = 0;
    std::vector<uint32_t> order;  // clientHead dlist (insertion order)
    uint32_t slot = kNoSlot;
    uint64_t gen = 0;             // generation of the last mutation of this Namespace
};
struct ClientInfo {
    bool alive = false;
    uint32_t ns = 0;
    uint8_t mac[6] = {0}, ipv4[4] = {0}, ipv6[16] = {0}, dhcpv6[16] = {0};
    uint32_t plugins = 0;
    bool has_ra = false;
    uint8_t ra_prefix[16] = {0};
    uint8_t ra_plen = 0;
    bool has_ctx = false;  // CClient.GetTransportCtx() != nil
    uint32_t ci_slot = kNoSlot;
};

struct Mirror {
    uint32_t max_ns = 0, max_clients = 0, n_parts = 1, part = 0;
    Map ns_map, mac_map, ip4_map, ip6_map;
    std::vector<NsInfo> ns;
    std::vector<ClientInfo> cl;
    std::unordered_map<std::string, Entry> ft_map;  // (client id, tuple bytes) -> flow id
    std::unordered_map<uint64_t, Entry> srv_map;    // client id << 32 | port | proto << 16
    uint32_t n_ctx = 0;                             // owned live clients with a TransportCtx
    uint32_t n_ctx_all = 0;                         // live clients with a TransportCtx, all partitions
    Hash ns_t, mac_t, ip4_t, ip6_t, ci_t, ft4_t, ft6_t, srv_t;
    Blocks nsinfo;                                  // 4 words per ns id, dense
    uint64_t gen = 1;
    std::unordered_map<K5, uint64_t, K5Hash> removed;  // tunnel key -> generation of its RemoveNs
    uint64_t removed_floor = 0;                        // removals older than this were forgotten

    void open(uint32_t max_ns, uint32_t max_clients);
    // device images hold only the Namespaces with emurx_owner(key, n) == part; rebuilds all
    void set_partition(uint32_t n, uint32_t part);
    // table k at half its spread (its device allocation failed): rebuilt; false at spread 2
    bool shrink(int k);
    bool pending() const;  // some image has edits not shipped yet
    Hash* hashes(int k);   // the 8 hash images (k < 8), for the uploader
    const Hash* hashes(int k) const { return const_cast<Mirror*>(this)->hashes(k); }
    void clean_all();

    // Go-map operations (emu_rx.h return codes)
    int ns_add(const uint8_t key[12], uint32_t id, uint32_t plugins);
    int ns_remove(const uint8_t key[12]);
    int ns_set_plugins(uint32_t id, uint32_t plugins);
    int client_add(uint32_t ns_id, uint32_t cid, const uint8_t mac[6], const uint8_t ipv4[4],
                   const uint8_t ipv6[16], const uint8_t dhcpv6[16], uint32_t plugins);
    int client_remove(uint32_t ns_id, const uint8_t mac[6]);
    int client_set_plugins(uint32_t cid, uint32_t plugins);
    int update_addr(uint32_t cid, int which, const uint8_t* nw);
    int client_set_ra(uint32_t cid, const uint8_t prefix[16], uint8_t plen);
    int flow_add(uint32_t cid, const uint8_t* tuple, uint32_t tlen, uint32_t flow);
    int flow_remove(uint32_t cid, const uint8_t* tuple, uint32_t tlen);
    int server_add(uint32_t cid, uint16_t port, uint8_t proto);
    int server_remove(uint32_t cid, uint16_t port, uint8_t proto);
    int client_set_transport(uint32_t cid, bool has);

    // mid-batch rule: may `r` differ from a classification against the live tables?
    bool stale(const emurx_rec& r, uint64_t since) const;
    // the device image's answer for a key (the kernels' bucket walk over the host image)
    int image_lookup(uint32_t table, const uint32_t* key, uint32_t* value);

   private:
    uint32_t tk_of(uint32_t ns_id) const;
    bool owned_ns(uint32_t ns_id) const { return ns_id < ns.size() && ns[ns_id].owned; }
    void touch_ns(uint32_t ns_id) { ns[ns_id].gen = ++gen; }
    void put_nsinfo(uint32_t ns_id);
    // image entries (the slot contents of emurx_tables.h) and their inserts
    void ns_slot_put(const K5& k, Entry& e);
    void mac_slot_put(const K5& k, Entry& e);
    void ip4_slot_put(const K5& k, Entry& e);
    void ip6_slot_put(const K5& k, Entry& e);
    void ci_put(uint32_t cid);
    void ft_slot_put(const std::string& k, Entry& e);
    void srv_slot_put(uint64_t k, Entry& e);
    void drop(Hash& t, Entry& e);
    void reserve(Hash& t, int which, uint32_t k = 1);  // rebuild `t` first when k more inserts would not fit
    void rebuild(int which, uint32_t buckets);
    void rewrite_client_slots(uint32_t cid);
    void drop_transport(uint32_t cid);
};

// table ids of Mirror::image_lookup (and Mirror::hashes order)
enum { kTabNs = 0, kTabMac, kTabIp4, kTabIp6, kTabCi, kTabFt4, kTabFt6, kTabSrv, kNumTabs };

}  // namespace emurx_host
