// emurx_mirror.h — host side of the Namespace / Client tables.
//
// The mirror keeps the reference's Go maps with their exact semantics (return codes of
// AddNs / AddClient / UpdateClient* ...) AND the image of every device table in the layout of
// emurx_tables.h.  Each mutation edits the image slot by slot and marks the 64-byte blocks it
// touched; emurx_api.cpp ships only those blocks to the device (emurx_delta) before the next
// batch.  The tables are two-choice bucketized cuckoo tables: an insert takes a free slot of
// either candidate bucket or evicts an entry to ITS other bucket (a random walk, every moved
// entry's slot index updated through a back pointer); a delete clears its slot.  An insert
// that finds no place within kMaxKicks rebuilds the table with a new hash seed (then larger);
// a table past its growth load is rebuilt larger.  Rebuilt tables are shipped whole.
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

// A two-choice bucketized cuckoo table image (emurx_tables.h): nb buckets of bw words (8,
// or 16 for the IPv6 flow table) holding bw / words slots; the slot's marker word mw is
// EMURX_EMPTY when free.  Every entry sits in emurx_b1 or emurx_b2 of its table hash.
struct Hash : Blocks {
    uint32_t words = 4, bw = EMURX_CBUCKET_WORDS, mw = 3, nb = 0, live = 0, seed = 0;
    double target = 0.5, grow_at = 0.8;  // load of a freshly sized table, load that triggers growth
    std::vector<uint32_t> hs;     // per slot: the entry's table hash (its two buckets), for evictions
    std::vector<uint32_t*> back;  // per slot: where the entry's owner keeps its slot index
    bool failed = false;          // an insert found no place: rebuild (new seed) before shipping
    uint64_t rng = 0x9E3779B97F4A7C15ull;
    static constexpr int kMaxKicks = 512;
    uint32_t per() const { return bw / words; }
    uint32_t nslots() const { return nb * per(); }
    uint32_t* at(uint32_t s) { return &img[(size_t)(s / per()) * bw + (s % per()) * words]; }
    const uint32_t* at(uint32_t s) const { return &img[(size_t)(s / per()) * bw + (s % per()) * words]; }
    bool is_free(uint32_t s) const { return at(s)[mw] == EMURX_EMPTY; }
    void touch_slot(uint32_t s) { touch((uint32_t)((size_t)(s / per()) * bw / EMURX_BUCKET_WORDS)); }
    // nbuckets buckets of bucket_words words, slots of w words with marker word m, all free
    void init(uint32_t nbuckets, uint32_t w, uint32_t bucket_words, uint32_t m);
    // insert entry e (its table hash h) into a free slot of its buckets, evicting along a
    // random walk when both are full; *bp (and every moved entry's back pointer) receives the
    // slot.  false: some entry was left without a slot (*its* back pointer = kNoSlot, failed set)
    bool put(uint32_t h, const uint32_t* e, uint32_t* bp);
    void del(uint32_t s);
    void rewrite(uint32_t s, uint32_t word, uint32_t v) {
        at(s)[word] = v;
        touch_slot(s);
    }
    // k more inserts would take the table past its growth load
    bool full(uint32_t k = 1) const { return (double)(live + k) > grow_at * nslots(); }
    // buckets for `entries` at the target load
    uint32_t sized(uint64_t entries) const;

   private:
    void place(uint32_t s, const uint32_t* e, uint32_t h, uint32_t* bp);
    uint32_t rand32() {
        rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
        return (uint32_t)(rng >> 16);
    }
};

struct NsInfo {
    bool alive = false;
    bool owned = false;
    uint8_t key[12] = {0};
    uint32_t plugins = 0;
    std::vector<uint32_t> order;  // clientHead dlist (insertion order)
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
    Hash ns_t, mac_t, ip4_t, ip6_t, ci_t, ft4_t, ft6_t, srv_t;
    Blocks nsinfo;                                  // 4 words per ns id, dense
    uint64_t gen = 1;
    std::unordered_map<K5, uint64_t, K5Hash> removed;  // tunnel key -> generation of its RemoveNs
    uint64_t removed_floor = 0;                        // removals older than this were forgotten

    void open(uint32_t max_ns, uint32_t max_clients);
    // device images hold only the Namespaces with emurx_owner(key, n) == part; rebuilds all
    void set_partition(uint32_t n, uint32_t part);
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
    void reserve(Hash& t, int which, uint32_t k = 1);  // rebuild `t` larger first when k more inserts would not fit
    // refill table `which` from the maps in `buckets` buckets (a new seed, then more buckets, when
    // an insert fails); reseed: start with a new seed
    void rebuild(int which, uint32_t buckets, bool reseed = false);
    void settle();  // rebuild every table an insert failed on (after each mutation)
    void rewrite_client_slots(uint32_t cid);
    void drop_transport(uint32_t cid);
};

// table ids of Mirror::image_lookup (and Mirror::hashes order)
enum { kTabNs = 0, kTabMac, kTabIp4, kTabIp6, kTabCi, kTabFt4, kTabFt6, kTabSrv, kNumTabs };

}  // namespace emurx_host
