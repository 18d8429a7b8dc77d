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
#include <string>
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
    bool has_ctx = false;  // CClient.GetTransportCtx() != nil
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

// One in-flight batch of the batched ZMQ ingest: pinned staging + device scratch + results.
struct IngestSlot {
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr;
    bool pending = false;
    uint32_t nmsg = 0, slots = 0;  // messages and descriptor slots of the batch in flight
    PinBuf<uint8_t> h_buf;         // messages, written by the caller (+64 B pad)
    PinBuf<uint32_t> h_ctl;        // emurx_msg[nmsg], slot_base[nmsg + 1]
    PinBuf<uint32_t> h_stat, h_qlist, h_qoff, h_mframes;
    PinBuf<uint8_t> h_mstatus;
    PinBuf<emurx_rec> h_rec;
    PinBuf<emurx_desc> h_desc;
    PinBuf<uint64_t> h_hist;
    DevBuf<uint8_t> d_buf;
    DevBuf<uint32_t> d_ctl, d_stat, d_qlist, d_tile_cnt, d_seg_off, d_packed, d_qoff;
    DevBuf<emurx_desc> d_desc;
    DevBuf<emurx_rec> d_rec;
    DevBuf<uint64_t> d_hist, d_hist_out;  // d_hist: zero between batches (k_qscan clears it)
    std::vector<uint32_t> remap;          // slot -> frame index, only when a message fell short
    void release() {
        if (st) (void)hipStreamSynchronize(st);
        h_buf.release(); h_ctl.release(); h_stat.release(); h_qlist.release(); h_qoff.release();
        h_mframes.release(); h_mstatus.release(); h_rec.release(); h_desc.release(); h_hist.release();
        d_buf.release(); d_ctl.release(); d_stat.release(); d_qlist.release(); d_tile_cnt.release();
        d_seg_off.release(); d_packed.release(); d_qoff.release(); d_desc.release(); d_rec.release();
        d_hist.release(); d_hist_out.release();
        if (done) (void)hipEventDestroy(done);
        if (st) (void)hipStreamDestroy(st);
        done = nullptr;
        st = nullptr;
        pending = false;
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

    // transport tables: (client id, tuple bytes) -> flow id; listeners (client id, port | proto << 16)
    std::unordered_map<std::string, uint32_t> ft_map;
    std::unordered_map<uint64_t, uint32_t> srv_map;
    uint32_t ft4_buckets = 1, ft6_buckets = 1, srv_buckets = 1;
    DevBuf<uint32_t> d_ft4, d_ft6, d_srv;
    std::vector<uint32_t> h_ft4, h_ft6, h_srv;
    bool ft_on = false;

    // device tables
    uint32_t ns_buckets = 0, mac_buckets = 0, ip4_buckets = 0, ip6_buckets = 0;
    DevBuf<uint32_t> d_ns, d_nsinfo, d_mac, d_ip4, d_ip6, d_client;
    std::vector<uint32_t> h_ns, h_nsinfo, h_mac, h_ip4, h_ip6, h_client;

    // batched host ingest: EMURX_INGEST_SLOTS public slots + one private to emurx_rx_stream
    IngestSlot ing[EMURX_INGEST_SLOTS + 1];

    // tx ZMQ framing scratch (emurx_tx_zmq_dev): per-level chain transfer tables
    DevBuf<uint8_t> d_txz;

    // route count pass fused into classify launches (emurx_set_route_parts): the counts of
    // the last such launch wait in d_route_cnt / d_route_grp for emurx_route_dev
    uint32_t route_parts = 0, route_n = 0;
    const emurx_rec* route_rec = nullptr;
    bool route_pending = false;

    // Namespace-partition packing scratch (emurx_route_dev)
    DevBuf<uint32_t> d_route_cnt, d_route_grp, d_route_goff;  // grp: zero between batches

    // k_rx staging slab per launch (emurx_launch_batch): the narrow 6 KiB slab runs 6
    // workgroups per CU instead of 5, but a wave whose frames span 6-7 KiB then takes the
    // slower window path.  Sampled tiles report how many of their waves fall in that band
    // into device words; the first launch and then at most every 8th copies them to pinned
    // memory behind itself (stream order, an event, no synchronisation), and the first
    // launch after the copy has landed decides.  The kernel
    // writing host memory directly was tried: host reads of lines the GPU keeps writing made
    // some launches 5x slower.  EMURX_STAGE=wide|narrow forces one size (tests, A/B).
    DevBuf<uint32_t> d_stage_fb;  // 64 sampled tiles x 4 waves: gen << 2 | has_frames << 1 | mid
    PinBuf<uint32_t> stage_fb;    // its copy
    uint32_t stage_gen = 0, stage_mode = 0;  // 0 auto, 1 wide, 2 narrow
    bool stage_copy = false, stage_pending = false;
    uint32_t stage_copy_gen = 0;
    hipEvent_t stage_ev = nullptr;
    bool stage_narrow = false;
    uint32_t last_stage = 0;

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
        T.ft_on = ft_on ? 1u : 0u;
        T.ft4_tab = d_ft4.p;
        T.ft6_tab = d_ft6.p;
        T.srv_tab = d_srv.p;
        T.ft4_mask = ft4_buckets - 1;
        T.ft6_mask = ft6_buckets - 1;
        T.srv_mask = srv_buckets - 1;
        return T;
    }
};

namespace {

// every entry point re-binds the handle's device (goroutines migrate between OS threads);
// hipGetDevice is a thread-local read, hipSetDevice only when the thread is elsewhere
int bind(emurx_t* h) {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur == h->cfg.device) return EMURX_OK;
    return hipSetDevice(h->cfg.device) == hipSuccess ? EMURX_OK : EMURX_EDEVICE;
}

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

// transport tables, sized to their entries (load <= 1/2 in slots), device buffers grown on demand
int build_transport(emurx_t* h) {
    size_t n4 = 0, n6 = 0;
    for (auto& kv : h->ft_map) (kv.first.size() == 4 + 13 ? n4 : n6)++;
    h->ft4_buckets = pow2_at_least(2 * n4 + 2) / 2;
    h->ft6_buckets = pow2_at_least(2 * n6 + 1);
    h->srv_buckets = pow2_at_least(2 * h->srv_map.size() + 4) / 4;
    empty_table(h->h_ft4, h->ft4_buckets, 8);
    empty_table(h->h_ft6, h->ft6_buckets, 16);
    empty_table(h->h_srv, h->srv_buckets, 4);
    for (auto& kv : h->ft_map) {
        const uint8_t* k = reinterpret_cast<const uint8_t*>(kv.first.data());
        const uint32_t cid = le32(k);
        const uint8_t* t = k + 4;
        if (kv.first.size() == 4 + 13) {
            uint32_t e[8] = {cid, le32(t), le32(t + 4), le32(t + 8), t[12], 0, 0, kv.second};
            bucket_put(h->h_ft4, h->ft4_buckets - 1, 8, emurx_ft4_hash(cid, e[1], e[2], e[3], e[4]), e);
        } else {
            uint32_t e[16] = {cid};
            for (int j = 0; j < 4; ++j) {
                e[1 + j] = le32(t + 4 * j);
                e[5 + j] = le32(t + 16 + 4 * j);
            }
            e[9] = le32(t + 32);
            e[10] = t[36];
            e[15] = kv.second;
            bucket_put(h->h_ft6, h->ft6_buckets - 1, 16, emurx_ft6_hash(cid, e[1], e[2], e[3], e[4], e[5], e[6], e[7], e[8], e[9], e[10]), e);
        }
    }
    for (auto& kv : h->srv_map) {
        uint32_t e[4] = {(uint32_t)(kv.first >> 32), (uint32_t)kv.first, 0, 1};
        bucket_put(h->h_srv, h->srv_buckets - 1, 4, emurx_srv_hash(e[0], e[1]), e);
    }
    h->ft_on = false;
    for (auto& c : h->cl) h->ft_on = h->ft_on || (c.alive && c.has_ctx);
    if (h->d_ft4.alloc(h->h_ft4.size()) || h->d_ft6.alloc(h->h_ft6.size()) || h->d_srv.alloc(h->h_srv.size()))
        return -1;
    return 0;
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
    // the client's MAC and plugin mask ride in the MAC slot's free upper half and in the IPv4 /
    // IPv6 slots' spare words: the rules that check them (PluginCtx.Get, IsUnicastToMe) need
    // no second read of the client record
    auto mac_words = [&](uint32_t cid, uint32_t& lo, uint32_t& hip) {
        const ClientInfo& c = h->cl[cid];
        lo = le32(c.mac);
        hip = (uint32_t)(c.mac[4] | (c.mac[5] << 8)) | ((c.plugins & 0xffffu) << 16);
    };
    empty_table(h->h_mac, h->mac_buckets, 4);
    for (auto& kv : h->mac_map) {
        uint32_t e[4] = {kv.first.w[0], kv.first.w[1], kv.first.w[2], kv.second};
        const uint32_t hh = emurx_mac_hash(tk_of(e[0]), e[1], e[2]);
        e[2] |= (h->cl[kv.second].plugins & 0xffffu) << 16;
        bucket_put(h->h_mac, h->mac_buckets - 1, 4, hh, e);
    }
    empty_table(h->h_ip4, h->ip4_buckets, 8);
    for (auto& kv : h->ip4_map) {
        uint32_t e[8] = {kv.first.w[0], kv.first.w[1], 0, 0, 0, 0, 0, kv.second};
        mac_words(kv.second, e[2], e[3]);
        bucket_put(h->h_ip4, h->ip4_buckets - 1, 8, emurx_ip4_hash(tk_of(e[0]), e[1]), e);
    }
    empty_table(h->h_ip6, h->ip6_buckets, 8);
    for (auto& kv : h->ip6_map) {
        const uint32_t* w = kv.first.w;
        uint32_t e[8] = {w[0], w[1], w[2], w[3], w[4], 0, 0, kv.second};
        mac_words(kv.second, e[5], e[6]);
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
        o[6] = c.has_ctx ? 1u : 0u;
    }
    if (build_transport(h)) return EMURX_ENOMEM;
    struct {
        uint32_t* d;
        std::vector<uint32_t>* h;
    } up[] = {{h->d_ns.p, &h->h_ns},   {h->d_nsinfo.p, &h->h_nsinfo}, {h->d_mac.p, &h->h_mac},
              {h->d_ip4.p, &h->h_ip4}, {h->d_ip6.p, &h->h_ip6},       {h->d_client.p, &h->h_client},
              {h->d_ft4.p, &h->h_ft4}, {h->d_ft6.p, &h->h_ft6},       {h->d_srv.p, &h->h_srv}};
    for (auto& u : up)
        if (hipMemcpyAsync(u.d, u.h->data(), u.h->size() * 4, hipMemcpyHostToDevice, st) != hipSuccess)
            return EMURX_EDEVICE;
    if (hipStreamSynchronize(st) != hipSuccess) return EMURX_EDEVICE;
    h->dirty = false;
    return EMURX_OK;
}

uint32_t ntiles(uint32_t n) { return (n + EMURX_QUEUE_TILE - 1) / EMURX_QUEUE_TILE; }
size_t queue_cap(uint32_t n) { return (size_t)ntiles(n) * EMURX_QUEUE_TILE; }

// the staging slab of the next k_rx launch (see emurx_ctx::stage_fb); advances stage_gen
bool choose_stage_(emurx_t* h) {
    ++h->stage_gen;
    h->stage_gen &= 0x3fffffffu;
    if (h->stage_mode) return h->stage_mode == 2;
    // decide as soon as the last copy-back has landed (an event query, no waiting)
    if (h->stage_pending && hipEventQuery(h->stage_ev) == hipSuccess) {
        h->stage_pending = false;
        // the sampled waves of the 16 launches up to the copied one (a 1M-frame launch
        // rewrites all 256 words, a small one only the first few)
        uint32_t waves = 0, mid = 0;
        for (int i = 0; i < 256; ++i) {
            const uint32_t w = h->stage_fb.p[i];
            const uint32_t age = (h->stage_copy_gen - (w >> 2)) & 0x3fffffffu;
            if ((w >> 2) && age < 16) {
                waves += (w >> 1) & 1;
                mid += w & 1;
            }
        }
        // a wave in the 6-7 KiB band costs several staged waves on the window path; below
        // 1% of the sampled waves the extra workgroup per CU wins (configs B, E), above it
        // loses (C)
        if (waves) h->stage_narrow = mid * 100 <= waves;
    }
    // the first launch and then at most every 8th copies its samples back
    if (!h->stage_pending && (!h->stage_copy_gen || ((h->stage_gen - h->stage_copy_gen) & 0x3fffffffu) >= 8))
        h->stage_copy = true;
    return h->stage_narrow;
}
int stage_copy_back(emurx_t* h, hipStream_t st) {
    if (!h->stage_copy) return 0;
    h->stage_copy = false;
    if (hipMemcpyAsync(h->stage_fb.p, h->d_stage_fb.p, 256 * sizeof(uint32_t), hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipEventRecord(h->stage_ev, st) != hipSuccess)
        return -1;
    h->stage_pending = true;
    h->stage_copy_gen = h->stage_gen;
    return 0;
}
bool choose_stage(emurx_t* h) {
    const bool narrow = choose_stage_(h);
    h->last_stage = narrow ? 6144u : 7168u;
    return narrow;
}

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
    const bool narrow = choose_stage(h);
    emurx_route_counts rt{h->route_parts, h->d_route_cnt.p, h->d_route_grp.p};
    const bool fuse = classify && h->route_parts && out->rec && n;
    if (fuse && h->route_pending &&  // counts nobody routed: clear them
        hipMemsetAsync(h->d_route_grp.p, 0, 1024 * 16 * sizeof(uint32_t), st) != hipSuccess)
        return EMURX_EDEVICE;
    int r = emurx_launch_batch(frames, desc, n, T, classify, *out, st, ev, narrow, h->d_stage_fb.p, h->stage_gen,
                               fuse ? &rt : nullptr);
    if (fuse) {
        h->route_pending = true;
        h->route_rec = out->rec;
        h->route_n = n;
    }
    if (!r) r = stage_copy_back(h, st);
    return r ? EMURX_EDEVICE : EMURX_OK;
}

// ---- batched ZMQ ingest (emurx_ingest_*; emurx_rx_stream uses the private last slot) ----
int ingest_buffer(emurx_t* h, uint32_t slot, size_t bytes, uint8_t** buf) {
    IngestSlot& s = h->ing[slot];
    if (s.pending || bytes > 0xFFFFFFFFull - 64) return EMURX_EINVAL;
    if (s.h_buf.alloc(bytes + 64) || s.d_buf.alloc(bytes + 64)) return EMURX_ENOMEM;
    *buf = s.h_buf.p;
    return EMURX_OK;
}

int ingest_submit(emurx_t* h, uint32_t slot, const emurx_msg* msgs, uint32_t nmsg) {
    IngestSlot& s = h->ing[slot];
    if (s.pending || (nmsg && (!msgs || !s.h_buf.p))) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    if (!s.st && hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking) != hipSuccess) return EMURX_EDEVICE;
    if (!s.done && hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) return EMURX_EDEVICE;
    const size_t cap = s.h_buf.p ? s.h_buf.n - 64 : 0;
    if (s.h_ctl.alloc((size_t)3 * nmsg + 1)) return EMURX_ENOMEM;
    uint32_t* ctl = s.h_ctl.p;
    uint32_t* base = ctl + 2 * (size_t)nmsg;
    uint64_t S = 0;
    size_t end = 0;
    for (uint32_t m = 0; m < nmsg; ++m) {
        const uint64_t e = (uint64_t)msgs[m].off + msgs[m].len;
        if (e > cap) return EMURX_EINVAL;
        end = std::max<size_t>(end, (size_t)e);
        ctl[2 * m] = msgs[m].off;
        ctl[2 * m + 1] = msgs[m].len;
        base[m] = (uint32_t)S;
        // descriptor slots: the frames the header announces, at most one per 4 bytes of the
        // first 64 KiB (the uint16 running offset never passes 65535 on an accepted frame)
        const uint8_t* p = s.h_buf.p + msgs[m].off;
        const uint32_t len = msgs[m].len;
        if (len >= 4 && (be32(p) >> 16) == EMURX_ZMQ_MAGIC)
            S += std::min<uint32_t>(be32(p) & 0xffff, (std::min<uint32_t>(len, 65536) - 4) / 4);
        if (S > h->cfg.max_frames) return EMURX_ENOSPC;
    }
    base[nmsg] = (uint32_t)S;
    const uint32_t n = (uint32_t)S, nt = ntiles(n);
    const size_t qcap = std::max<size_t>(queue_cap(n), EMURX_QUEUE_TILE);
    const size_t hw = (size_t)EMURX_HIST_SHARDS * 2 * EMURX_HIST_BINS;
    const bool fresh_hist = !s.d_hist.p;
    if (s.d_ctl.alloc((size_t)3 * nmsg + 1) || s.d_stat.alloc(nmsg) || s.d_desc.alloc(n) || s.d_rec.alloc(n) ||
        s.d_qlist.alloc(EMURX_NUM_QUEUES * qcap) || s.d_tile_cnt.alloc((size_t)std::max<uint32_t>(nt, 1) * 16) ||
        s.d_seg_off.alloc((size_t)std::max<uint32_t>(nt, 1) * 16) || s.d_packed.alloc(n) || s.d_qoff.alloc(16) ||
        s.d_hist.alloc(hw) || s.d_hist_out.alloc(2 * EMURX_HIST_BINS) || s.h_stat.alloc(nmsg) ||
        s.h_rec.alloc(n) || s.h_desc.alloc(n) || s.h_qlist.alloc(n) || s.h_qoff.alloc(16) ||
        s.h_hist.alloc(2 * EMURX_HIST_BINS) || s.h_mframes.alloc(nmsg) || s.h_mstatus.alloc(nmsg))
        return EMURX_ENOMEM;
    if (h->dirty) {  // batches in flight read the device tables: let them finish first
        for (auto& o : h->ing)
            if (o.st) (void)hipStreamSynchronize(o.st);
        if ((rc = rebuild_and_upload(h, h->stream))) return rc;
    }
    hipStream_t st = s.st;
    const auto H2D = hipMemcpyHostToDevice, D2H = hipMemcpyDeviceToHost;
    bool ok = true;
    if (fresh_hist) ok = ok && hipMemsetAsync(s.d_hist.p, 0, hw * sizeof(uint64_t), st) == hipSuccess;
    ok = ok && hipMemcpyAsync(s.d_ctl.p, ctl, ((size_t)3 * nmsg + 1) * 4, H2D, st) == hipSuccess;
    if (end) ok = ok && hipMemcpyAsync(s.d_buf.p, s.h_buf.p, end, H2D, st) == hipSuccess;
    if (!ok) return EMURX_EDEVICE;
    if (emurx_launch_zmq_walk(s.d_buf.p, s.d_ctl.p, nmsg, s.d_desc.p, s.d_stat.p, st)) return EMURX_EDEVICE;
    if (n) {
        const emurx_dev_out o{s.d_rec.p, s.d_qlist.p, (uint32_t)qcap, s.d_tile_cnt.p, s.d_hist.p};
        const bool narrow = choose_stage(h);
        if (emurx_launch_batch(s.d_buf.p, s.d_desc.p, n, h->tables(), true, o, st, nullptr, narrow,
                               h->d_stage_fb.p, h->stage_gen) ||
            stage_copy_back(h, st))
            return EMURX_EDEVICE;
    }
    if (emurx_launch_queue_pack(s.d_qlist.p, (uint32_t)qcap, s.d_tile_cnt.p, n, s.d_seg_off.p, s.d_packed.p,
                                s.d_qoff.p, s.d_hist.p, s.d_hist_out.p, st))
        return EMURX_EDEVICE;
    if (n)
        ok = hipMemcpyAsync(s.h_rec.p, s.d_rec.p, (size_t)n * sizeof(emurx_rec), D2H, st) == hipSuccess &&
             hipMemcpyAsync(s.h_desc.p, s.d_desc.p, (size_t)n * sizeof(emurx_desc), D2H, st) == hipSuccess &&
             hipMemcpyAsync(s.h_qlist.p, s.d_packed.p, (size_t)n * 4, D2H, st) == hipSuccess;
    if (nmsg) ok = ok && hipMemcpyAsync(s.h_stat.p, s.d_stat.p, (size_t)nmsg * 4, D2H, st) == hipSuccess;
    ok = ok && hipMemcpyAsync(s.h_qoff.p, s.d_qoff.p, (EMURX_NUM_QUEUES + 1) * 4, D2H, st) == hipSuccess &&
         hipMemcpyAsync(s.h_hist.p, s.d_hist_out.p, 2 * EMURX_HIST_BINS * 8, D2H, st) == hipSuccess &&
         hipEventRecord(s.done, st) == hipSuccess;
    if (!ok) return EMURX_EDEVICE;
    s.pending = true;
    s.nmsg = nmsg;
    s.slots = n;
    return EMURX_OK;
}

int ingest_wait(emurx_t* h, uint32_t slot, emurx_ingest_result* res) {
    IngestSlot& s = h->ing[slot];
    if (!s.pending) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    s.pending = false;
    if (hipEventSynchronize(s.done) != hipSuccess) return EMURX_EDEVICE;
    memset(res, 0, sizeof(*res));
    emurx_counters& d = res->delta;
    d.rx_batch = s.nmsg;  // one OnRxStream per message, veth_zmq.go:278
    uint64_t nf = 0;
    for (uint32_t m = 0; m < s.nmsg; ++m) {
        const uint32_t w = s.h_stat.p[m], f = w & 0xffffff, e = w >> 24;
        s.h_mframes.p[m] = f;
        s.h_mstatus.p[m] = (uint8_t)e;
        nf += f;
        if (e == EMURX_MSG_PARSE_ERR) d.rx_parse_err++;
        if (e == EMURX_MSG_PANIC) d.ref_panic++;
    }
    if (nf > s.slots) return EMURX_EDEVICE;
    if (nf < s.slots) {  // messages that announced more frames than they carried: close the holes
        const uint32_t* base = s.h_ctl.p + 2 * (size_t)s.nmsg;
        s.remap.assign(s.slots, EMURX_ID_NONE);
        uint32_t c = 0;
        for (uint32_t m = 0; m < s.nmsg; ++m) {
            const uint32_t f = s.h_mframes.p[m];
            if (c != base[m] && f) {
                memmove(s.h_rec.p + c, s.h_rec.p + base[m], (size_t)f * sizeof(emurx_rec));
                memmove(s.h_desc.p + c, s.h_desc.p + base[m], (size_t)f * sizeof(emurx_desc));
            }
            for (uint32_t k = 0; k < f; ++k) s.remap[base[m] + k] = c + k;
            c += f;
        }
        for (uint64_t i = 0; i < nf; ++i) {
            const uint32_t j = s.h_qlist.p[i];
            if (j >= s.slots || s.remap[j] == EMURX_ID_NONE) return EMURX_EDEVICE;
            s.h_qlist.p[i] = s.remap[j];
        }
    }
    memcpy(res->qoff, s.h_qoff.p, sizeof(res->qoff));
    if (res->qoff[EMURX_NUM_QUEUES] != nf) return EMURX_EDEVICE;
    emurx_hist_to_counters(s.h_hist.p, &d);
    d.rx_pkts = nf;  // VethIFZmq.OnRx veth_zmq.go:233-234
    for (int b = 0; b < EMURX_HIST_BINS; ++b) d.rx_bytes += s.h_hist.p[2 * b + 1];
    res->rec = s.h_rec.p;
    res->desc = s.h_desc.p;
    res->qlist = s.h_qlist.p;
    res->msg_frames = s.h_mframes.p;
    res->msg_status = s.h_mstatus.p;
    res->n_frames = (uint32_t)nf;
    res->n_msgs = s.nmsg;
    return EMURX_OK;
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
    h->ip4_buckets = pow2_at_least(2ull * cfg->max_clients) / 2;  // one address per client, 2 slots per bucket
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
    if (const char* e = getenv("EMURX_STAGE")) h->stage_mode = !strcmp(e, "wide") ? 1 : !strcmp(e, "narrow") ? 2 : 0;
    if (h->stage_fb.alloc(256) || h->d_stage_fb.alloc(256) ||
        hipEventCreateWithFlags(&h->stage_ev, hipEventDisableTiming) != hipSuccess ||
        hipMemset(h->d_stage_fb.p, 0, 256 * sizeof(uint32_t)) != hipSuccess) {
        emurx_close(h);
        return EMURX_ENOMEM;
    }
    memset(h->stage_fb.p, 0, 256 * sizeof(uint32_t));
    h->dirty = true;
    if ((rc = rebuild_and_upload(h, h->stream))) { emurx_close(h); return rc; }
    *out = h;
    return EMURX_OK;
}

void emurx_close(emurx_t* h) {
    if (!h) return;
    bind(h);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (auto& s : h->ing) s.release();
    h->stage_fb.release();
    h->d_stage_fb.release();
    if (h->stage_ev) (void)hipEventDestroy(h->stage_ev);
    h->d_ns.release(); h->d_nsinfo.release(); h->d_mac.release(); h->d_ip4.release();
    h->d_ip6.release(); h->d_client.release();
    h->d_ft4.release(); h->d_ft6.release(); h->d_srv.release();
    h->d_route_cnt.release(); h->d_route_grp.release(); h->d_route_goff.release();
    h->d_txz.release();
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

int emurx_clients_add(emurx_t* h, const emurx_client_spec* c, uint32_t n, uint32_t* n_added) {
    if (!h || (n && !c)) return EMURX_EINVAL;
    uint32_t k = 0;
    int rc = EMURX_OK;
    for (; k < n; ++k)
        if ((rc = emurx_client_add(h, c[k].ns_id, c[k].client_id, c[k].mac, c[k].ipv4, c[k].ipv6, c[k].dhcpv6,
                                   c[k].plugin_mask)))
            break;
    if (n_added) *n_added = k;
    return rc;
}

static void drop_transport(emurx_t* h, uint32_t cid) {
    for (auto it = h->ft_map.begin(); it != h->ft_map.end();)
        it = le32(reinterpret_cast<const uint8_t*>(it->first.data())) == cid ? h->ft_map.erase(it) : std::next(it);
    for (auto it = h->srv_map.begin(); it != h->srv_map.end();)
        it = (uint32_t)(it->first >> 32) == cid ? h->srv_map.erase(it) : std::next(it);
    h->cl[cid].has_ctx = false;
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
    drop_transport(h, cid);  // TransportCtx.onRemove: its sockets go with the client
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

// ---- transport flow tables (TransportCtx.addFlowv4/6 / removeFlowv4/6 client_ctx.go:597-651,
// serverCb / lookupServerPort :1142-1155, GetTransportCtx socketApi.go:174-193) -----------
static int flow_key(emurx_t* h, uint32_t cid, const uint8_t* tuple, uint32_t tlen, std::string& k) {
    if (!h || !tuple || (tlen != 13 && tlen != 37)) return EMURX_EINVAL;
    if (cid >= h->cfg.max_clients || !h->cl[cid].alive) return EMURX_ENOENT;
    k.assign(4 + tlen, '\0');
    memcpy(&k[0], &cid, 4);
    memcpy(&k[4], tuple, tlen);
    return EMURX_OK;
}
int emurx_flow_add(emurx_t* h, uint32_t cid, const uint8_t* tuple, uint32_t tlen, uint32_t flow_id) {
    std::string k;
    int rc = flow_key(h, cid, tuple, tlen, k);
    if (rc) return rc;
    if (flow_id > EMURX_FLOW_ID_MAX) return EMURX_EINVAL;
    if (h->ft_map.count(k)) return EMURX_EEXIST;  // ft_add_err_already_exits
    h->ft_map[k] = flow_id;
    h->cl[cid].has_ctx = true;
    h->dirty = true;
    return EMURX_OK;
}
int emurx_flow_remove(emurx_t* h, uint32_t cid, const uint8_t* tuple, uint32_t tlen) {
    std::string k;
    int rc = flow_key(h, cid, tuple, tlen, k);
    if (rc) return rc;
    if (!h->ft_map.erase(k)) return EMURX_ENOENT;  // ft_remove_err_not_exits
    h->dirty = true;
    return EMURX_OK;
}
static int srv_key(emurx_t* h, uint32_t cid, uint16_t port, uint8_t proto, uint64_t& k) {
    if (!h || (proto != 6 && proto != 17)) return EMURX_EINVAL;
    if (cid >= h->cfg.max_clients || !h->cl[cid].alive) return EMURX_ENOENT;
    k = ((uint64_t)cid << 32) | port | ((uint32_t)proto << 16);
    return EMURX_OK;
}
int emurx_server_add(emurx_t* h, uint32_t cid, uint16_t port, uint8_t proto) {
    uint64_t k;
    int rc = srv_key(h, cid, port, proto, k);
    if (rc) return rc;
    if (h->srv_map.count(k)) return EMURX_EEXIST;
    h->srv_map[k] = 1;
    h->cl[cid].has_ctx = true;
    h->dirty = true;
    return EMURX_OK;
}
int emurx_server_remove(emurx_t* h, uint32_t cid, uint16_t port, uint8_t proto) {
    uint64_t k;
    int rc = srv_key(h, cid, port, proto, k);
    if (rc) return rc;
    if (!h->srv_map.erase(k)) return EMURX_ENOENT;
    h->dirty = true;
    return EMURX_OK;
}
int emurx_client_set_transport(emurx_t* h, uint32_t cid, int has_ctx) {
    if (!h) return EMURX_EINVAL;
    if (cid >= h->cfg.max_clients || !h->cl[cid].alive) return EMURX_ENOENT;
    h->cl[cid].has_ctx = has_ctx != 0;
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
    // one message through the batched ingest (device framing walk), on the private slot
    const uint32_t slot = EMURX_INGEST_SLOTS;
    uint8_t* buf = nullptr;
    if ((rc = ingest_buffer(h, slot, std::max<size_t>(len, 1), &buf))) return rc;
    if (len) memcpy(buf, msg, len);
    memset(buf + len, 0, 64);
    const emurx_msg m{0, (uint32_t)len};
    if ((rc = ingest_submit(h, slot, &m, 1))) return rc;
    emurx_ingest_result r;
    if ((rc = ingest_wait(h, slot, &r))) return rc;
    if (r.n_frames > out_cap) return EMURX_ENOSPC;
    if (r.n_frames && (!out_rec || !out_qlist)) return EMURX_EINVAL;
    if (r.n_frames) {
        memcpy(out_rec, r.rec, (size_t)r.n_frames * sizeof(emurx_rec));
        memcpy(out_qlist, r.qlist, (size_t)r.n_frames * 4);
    }
    memcpy(out_qoff, r.qoff, sizeof(r.qoff));
    *delta = r.delta;
    *n_out = r.n_frames;
    return EMURX_OK;
}

int emurx_ingest_buffer(emurx_t* h, uint32_t slot, size_t bytes, uint8_t** buf) {
    if (!h || !buf || slot >= EMURX_INGEST_SLOTS) return EMURX_EINVAL;
    int rc = bind(h);
    return rc ? rc : ingest_buffer(h, slot, bytes, buf);
}
int emurx_ingest_submit(emurx_t* h, uint32_t slot, const emurx_msg* msgs, uint32_t nmsg) {
    if (!h || slot >= EMURX_INGEST_SLOTS) return EMURX_EINVAL;
    return ingest_submit(h, slot, msgs, nmsg);
}
int emurx_ingest_wait(emurx_t* h, uint32_t slot, emurx_ingest_result* res) {
    if (!h || !res || slot >= EMURX_INGEST_SLOTS) return EMURX_EINVAL;
    return ingest_wait(h, slot, res);
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

uint32_t emurx_last_stage(const emurx_t* h) { return h ? h->last_stage : 0; }

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

int emurx_tx_checksum_dev(emurx_t* h, uint8_t* d_frames, const emurx_tx_desc* d_desc, uint32_t n,
                          uint8_t* d_status, void* stream) {
    if (!h || (n && (!d_frames || !d_desc))) return EMURX_EINVAL;
    if ((uintptr_t)d_desc & 15) return EMURX_EINVAL;  // one 16-byte load per descriptor
    int rc = bind(h);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    return emurx_launch_tx_csum(d_frames, d_desc, n, d_status, st) ? EMURX_EDEVICE : EMURX_OK;
}

int emurx_tx_zmq_dev(emurx_t* h, const uint8_t* d_frames, const emurx_desc* d_desc, uint32_t n,
                     uint8_t* d_out, uint64_t out_cap, uint64_t* d_msg_off, uint64_t* d_info, void* stream) {
    if (!h || !d_msg_off || !d_info || (n && (!d_frames || !d_desc || (!d_out && out_cap))))
        return EMURX_EINVAL;
    if (n > (1u << 30) || ((uintptr_t)d_out & 15) || ((uintptr_t)d_desc & 7)) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    const size_t need = emurx_txz_scratch_bytes(n);
    if (need > h->d_txz.n) {  // grows on demand; a launch in flight may still read the old one
        (void)hipStreamSynchronize(st);
        if (h->d_txz.alloc(need)) return EMURX_ENOMEM;
    }
    return emurx_launch_tx_zmq(d_frames, d_desc, n, d_out, out_cap, d_msg_off, d_info, h->d_txz.p, st)
               ? EMURX_EDEVICE
               : EMURX_OK;
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
    // the owners of exactly this batch were counted by its classify launch: skip that pass
    const bool counted = h->route_pending && d_rec == h->route_rec && n == h->route_n && n_parts == h->route_parts;
    if (h->route_pending && !counted &&
        hipMemsetAsync(h->d_route_grp.p, 0, gw * sizeof(uint32_t), st) != hipSuccess)
        return EMURX_EDEVICE;
    h->route_pending = false;
    return emurx_launch_route(d_rec, n, n_parts, my_rank, cap, d_send, d_send_count, h->d_route_cnt.p,
                              h->d_route_grp.p, h->d_route_goff.p, st, counted)
               ? EMURX_EDEVICE
               : EMURX_OK;
}

int emurx_set_route_parts(emurx_t* h, uint32_t n_parts) {
    if (!h || n_parts > EMURX_MAX_PARTS) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    (void)hipStreamSynchronize(h->stream);
    const size_t gw = 1024 * 16, tiles = ((size_t)h->cfg.max_frames + EMURX_QUEUE_TILE - 1) / EMURX_QUEUE_TILE;
    if (n_parts) {
        if (tiles > 1024u * 64u) return EMURX_EINVAL;
        if (!h->d_route_grp.p) {
            if (h->d_route_grp.alloc(gw) || hipMemset(h->d_route_grp.p, 0, gw * sizeof(uint32_t)) != hipSuccess)
                return EMURX_ENOMEM;
        }
        if (h->d_route_cnt.alloc(std::max<size_t>(tiles, 1) * 16) || h->d_route_goff.alloc(gw)) return EMURX_ENOMEM;
    }
    if (h->route_pending && h->d_route_grp.p &&
        hipMemset(h->d_route_grp.p, 0, gw * sizeof(uint32_t)) != hipSuccess)
        return EMURX_EDEVICE;
    h->route_pending = false;
    h->route_parts = n_parts;
    return EMURX_OK;
}

}  // extern "C"
