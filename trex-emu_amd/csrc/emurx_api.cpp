// emurx_api.cpp — C-ABI of the MI355X receive path (include/emu_rx.h).
//
// Owns the Namespace / Client tables (emurx_mirror.*: the Go maps plus the image of every
// device table, edited slot by slot), ships the edited 64-byte blocks to the device before
// the next batch that reads them (one H2D copy + one k_apply launch, stream-ordered against
// every stream that read the tables, no host synchronisation), the device scratch of a batch,
// and the host batch entry points that replace VethIFZmq.OnRxStream's per-frame loop
// (src/emu/core/veth_zmq.go:277-320).  No exception or abort crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/emu_rx.h"
#include "emurx_kernels.h"
#include "emurx_mirror.h"
#include "emurx_tables.h"

using emurx_host::Blocks;
using emurx_host::Hash;
using emurx_host::Mirror;

namespace {

uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    int alloc(size_t count) {
        if (count <= n && p) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (!EMURX_HIP_OK(hipMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T)))) return -1;
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
        if (!EMURX_HIP_OK(hipHostMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T), hipHostMallocDefault)))
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

// a typed place inside a slot's result block (IngestSlot::h_res / d_res)
template <class T>
struct View {
    T* p = nullptr;
};
// One in-flight batch of the batched ZMQ ingest: pinned staging + device scratch + results.
// The results (records, descriptors, packed queues, message status, qoff, folded histogram)
// share one device block and one pinned block of the same layout (set_results): the pipeline
// copies them back with one D2H, and the one-launch path writes the pinned block directly.
struct IngestSlot {
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr;
    bool pending = false;
    uint32_t nmsg = 0, slots = 0;  // messages and descriptor slots of the batch in flight
    PinBuf<uint8_t> h_buf;         // messages, written by the caller (+64 B pad)
    PinBuf<uint32_t> h_ctl;        // emurx_msg[nmsg], slot_base[nmsg + 1]
    PinBuf<uint32_t> h_mframes;
    PinBuf<uint8_t> h_mstatus;
    PinBuf<uint8_t> h_res;                 // the result block, pinned
    View<uint32_t> h_stat, h_qlist, h_qoff;
    View<emurx_rec> h_rec;
    View<emurx_desc> h_desc;
    View<uint64_t> h_hist;
    DevBuf<uint8_t> d_buf;
    DevBuf<uint32_t> d_ctl, d_qlist, d_tile_cnt, d_seg_off;
    DevBuf<uint64_t> d_hist;               // zero between batches (k_qscan clears it)
    DevBuf<uint8_t> d_res;                 // the result block, device
    View<uint32_t> d_stat, d_packed, d_qoff;
    View<emurx_desc> d_desc;
    View<emurx_rec> d_rec;
    View<uint64_t> d_hist_out;
    size_t res_bytes = 0;                  // the current batch's result block
    // the fused small-batch path's scratch (k_ingest_small), zero between batches
    DevBuf<uint32_t> d_qseg, d_tcnt, d_ticket;
    DevBuf<uint64_t> d_hsmall;
    PinBuf<uint32_t> h_done;  // the small path's completion word: the batch's seq, written last
    uint32_t seq = 0;
    bool small = false;       // the batch in flight took the small path
    std::vector<uint32_t> remap;          // slot -> frame index, only when a message fell short
    void release() {
        if (st) (void)hipStreamSynchronize(st);
        d_qseg.release(); d_tcnt.release(); d_ticket.release(); d_hsmall.release(); h_done.release();
        h_buf.release(); h_ctl.release(); h_mframes.release(); h_mstatus.release(); h_res.release();
        d_buf.release(); d_ctl.release(); d_qlist.release(); d_tile_cnt.release(); d_seg_off.release();
        d_hist.release(); d_res.release();
        if (done) (void)hipEventDestroy(done);
        if (st) (void)hipStreamDestroy(st);
        done = nullptr;
        st = nullptr;
        pending = false;
    }
};

// one staging slot of the table-delta ring: pinned entries, read by k_apply over the bus
// (no copy launch: a delta is a few KiB)
struct DeltaSlot {
    PinBuf<emurx_delta> h;
    hipEvent_t ev = nullptr;  // recorded after the k_apply that read h
    bool used = false;
};
constexpr int kDeltaRing = 4;
constexpr size_t kMaxReaders = 16;

}  // namespace

struct emurx_ctx {
    emurx_cfg cfg{};
    bool host_only = false;  // cfg.device < 0: the table mirror alone, no HIP calls
    hipStream_t stream = nullptr;
    uint32_t cb_mask = 0;  // Parser.Init: every callback parserNotSupported (eapol nil)

    Mirror m;  // Go maps + device table images (emurx_mirror.h)

    // device tables: the 8 hash images (emurx_host::kTab*) and the dense ns info
    DevBuf<uint32_t> d_tab[emurx_host::kNumTabs];
    DevBuf<uint32_t> d_nsinfo;
    // table shipment: delta ring, the streams that read the tables since the last shipment,
    // and which shipment every stream has waited for
    DeltaSlot ring[kDeltaRing];
    uint32_t ring_i = 0;
    hipEvent_t ship_ev = nullptr;
    uint64_t ship_gen = 0;
    std::vector<hipStream_t> readers;
    std::vector<hipEvent_t> reader_ev;
    std::vector<std::pair<hipStream_t, uint64_t>> waited;
    uint64_t shipped_blocks = 0, shipped_whole = 0;  // counters (emurx_table_stats)

    // batched host ingest: EMURX_INGEST_SLOTS public slots + one private to emurx_rx_stream
    IngestSlot ing[EMURX_INGEST_SLOTS + 1];
    bool ingest_small = true;  // small batches in one launch (k_ingest_small); EMURX_INGEST_SMALL=0: never
    bool ingest_spin = true;   // wait for them on their completion word; EMURX_INGEST_SPIN=0: on the event
    // the one-launch path's bounds: its tiles must all be resident (the device's capacity for
    // k_ingest_small, measured at emurx_open), and a workgroup waits for the others at most
    // EMURX_INGEST_SPIN_US (default 200 us) plus 0.1 ns per byte of the batch's messages (the
    // tiles read them over PCIe at 20-50 GB/s, so a bigger batch's tiles arrive further apart:
    // at most 1.2 ms for the largest one-launch batch); 0 forces the degraded pack (tests)
    uint32_t small_tiles = EMURX_SMALL_TILES;
    double spin_base_us = 200.0;
    uint32_t wall_khz = 100000;  // the GPU's wall clock (hipDeviceAttributeWallClockRate)

    // tx ZMQ framing scratch (emurx_tx_zmq_dev): per-level chain transfer tables
    DevBuf<uint8_t> d_txz;
    // the tx write kernel's image per call (EMURX_TXZ_*), from the bounds of the tiles' output
    // rows an earlier call's chain kernel folded into two scratch words: copied back behind that
    // call (an event, no synchronisation) as the staging slab's feedback is, the first call and
    // then at most every txz_every-th (8, doubled when a decision repeats, up to 256).  Every
    // image writes every tile correctly; the choice is speed only.  EMURX_TXZ=wide|narrow|long
    // forces one.
    PinBuf<uint32_t> txz_fb;
    hipEvent_t txz_ev = nullptr;
    bool txz_pending = false;
    int txz_variant = EMURX_TXZ_WIDE, txz_mode = -1;
    uint32_t txz_calls = 0, txz_last_copy = 0, txz_every = 8, txz_same = 0;
    int last_txz = -1;

    // Namespace-partition packing scratch (emurx_route_dev / emurx_classify_route_dev /
    // emurx_parse_route_dev): one set per stream, so routes of batches pipelined over several
    // streams run side by side; past kRouteSets streams a set changes hands behind an event
    struct RouteScratch {
        hipStream_t st = nullptr;
        bool used = false;
        hipEvent_t done = nullptr;                      // recorded after each route on st
        DevBuf<uint32_t> cnt, grp, goff;                // grp: zero between batches
        DevBuf<uint32_t> tcur;                          // tail cursors of the partitioned source
        void release() {
            cnt.release(); grp.release(); goff.release(); tcur.release();
            if (done) (void)hipEventDestroy(done);
            done = nullptr;
        }
    };
    static constexpr size_t kRouteSets = 4;
    RouteScratch route[kRouteSets];
    uint32_t route_next = 0;  // the set a new stream takes over when all are in use

    // k_rx staging slab per launch (emurx_launch_batch): the narrow 6 KiB slab runs 6
    // workgroups per CU instead of 5, but a wave whose frames span 6-7 KiB then takes the
    // slower window path.  Sampled tiles report how many of their waves fall in that band
    // into device words; the first launch and then at most every `stage_every`-th copies them to pinned
    // memory behind itself (stream order, an event, no synchronisation), and the first
    // launch after the copy has landed decides.  The kernel
    // writing host memory directly was tried: host reads of lines the GPU keeps writing made
    // some launches 5x slower.  EMURX_STAGE=wide|narrow forces one size (tests, A/B).
    DevBuf<uint32_t> d_stage_fb;  // 64 sampled tiles x 4 waves: gen << 2 | has_frames << 1 | mid
    PinBuf<uint32_t> stage_fb;    // its copy
    uint32_t stage_gen = 0, stage_mode = 0;  // 0 auto, 1 wide, 2 narrow
    bool stage_copy = false, stage_pending = false;
    uint32_t stage_copy_gen = 0;
    // launches between copy-backs: 8, doubled after each decision that repeats the one before
    // it (from the second in a row), up to 256; back to 8 when a decision changes the slab.  A
    // copy-back is a blit between two k_rx launches on the caller's stream (it breaks the
    // overlap with the next launch): config B's 20-step command ran 2-3 % slower with one per 8
    uint32_t stage_every = 8, stage_same = 0;
    hipEvent_t stage_ev = nullptr;
    bool stage_narrow = false;
    uint32_t last_stage = 0;

    // the Namespace-owner exchange's communicator (emurx_comm.cpp), or none
    emurx_comm_state* comm = nullptr;

    // timing ring: 2 events per batch (around the k_rx launch)
    std::vector<hipEvent_t> ev;
    uint32_t slots = 0, ev_head = 0, ev_count = 0, stride = 1, batch_seq = 0;

    emurx_dev_tables tables() const {
        using namespace emurx_host;
        emurx_dev_tables T{};
        T.ns_tab = d_tab[kTabNs].p;
        T.ns_info = d_nsinfo.p;
        T.mac_tab = d_tab[kTabMac].p;
        T.ip4_tab = d_tab[kTabIp4].p;
        T.ip6_tab = d_tab[kTabIp6].p;
        T.ci_tab = d_tab[kTabCi].p;
        T.ns_mask = m.ns_t.mask();
        T.mac_mask = m.mac_t.mask();
        T.ip4_mask = m.ip4_t.mask();
        T.ip6_mask = m.ip6_t.mask();
        T.ci_mask = m.ci_t.mask();
        T.max_ns = cfg.max_ns;
        T.cb_mask = cb_mask;
        T.ft_on = m.n_ctx ? 1u : 0u;
        T.ft4_tab = d_tab[kTabFt4].p;
        T.ft6_tab = d_tab[kTabFt6].p;
        T.srv_tab = d_tab[kTabSrv].p;
        T.ft4_mask = m.ft4_t.mask();
        T.ft6_mask = m.ft6_t.mask();
        T.srv_mask = m.srv_t.mask();
        return T;
    }
};

namespace {

// every entry point re-binds the handle's device (goroutines migrate between OS threads);
// hipGetDevice is a thread-local read, hipSetDevice only when the thread is elsewhere
int bind(emurx_t* h) {
    if (h->host_only) return EMURX_EDEVICE;
    int cur = -1;
    if (EMURX_HIP_OK(hipGetDevice(&cur)) && cur == h->cfg.device) return EMURX_OK;
    return EMURX_HIP_OK(hipSetDevice(h->cfg.device)) ? EMURX_OK : EMURX_EDEVICE;
}

uint64_t& waited_gen(emurx_t* h, hipStream_t s) {
    for (auto& w : h->waited)
        if (w.first == s) return w.second;
    h->waited.emplace_back(s, 0);
    return h->waited.back().second;
}

// Ship the edited table blocks on `st`: after every stream that read the tables since the
// last shipment (an event recorded on it now, waited on by st), before every later reader
// (ship_ev, waited on by each reader stream once).  Edited blocks travel as emurx_delta
// entries in a ring of pinned buffers that one k_apply launch reads directly.
// Whole images (first upload, a rebuilt or grown table, or a quarter of a table edited)
// are copied synchronously; growing a device table waits for the device first, since
// batches in flight may still read the old buffer.
int ship_tables(emurx_t* h, hipStream_t st) {
    using namespace emurx_host;
    Mirror& m = h->m;
    for (size_t k = 0; k < h->readers.size(); ++k) {
        const hipStream_t r = h->readers[k];
        if (r == st) continue;
        while (h->reader_ev.size() <= k) {  // one event per reader slot (slots skipped above included)
            hipEvent_t e;
            if (!EMURX_HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming))) return EMURX_EDEVICE;
            h->reader_ev.push_back(e);
        }
        if (!EMURX_HIP_OK(hipEventRecord(h->reader_ev[k], r)) || !EMURX_HIP_OK(hipStreamWaitEvent(st, h->reader_ev[k], 0)))
            return EMURX_EDEVICE;
    }
    Blocks* img[kNumTabs + 1];
    DevBuf<uint32_t>* dev[kNumTabs + 1];
    for (int k = 0; k < kNumTabs; ++k) {
        img[k] = m.hashes(k);
        dev[k] = &h->d_tab[k];
    }
    img[kNumTabs] = &m.nsinfo;
    dev[kNumTabs] = &h->d_nsinfo;
    bool whole = false, grow = false;
    size_t nd = 0;
    for (int k = 0; k <= kNumTabs; ++k) {
        if (!img[k]->all && img[k]->dirty.size() * 4 > img[k]->nblocks()) img[k]->all = true;
        whole = whole || img[k]->all;
        grow = grow || (img[k]->all && img[k]->img.size() > dev[k]->n);
        if (!img[k]->all) nd += img[k]->dirty.size();
    }
    if (grow && !EMURX_HIP_OK(hipDeviceSynchronize())) return EMURX_EDEVICE;
    if (whole) {
        if (!EMURX_HIP_OK(hipStreamSynchronize(st))) return EMURX_EDEVICE;
        // a table whose device allocation fails is rebuilt at half its spread and tried again
        // (emurx_cfg: memory traded for lookup latency, down to 2 slots per entry);
        // EMURX_DEBUG_TABLE_LIMIT (bytes) fails every larger allocation, for tests
        static const size_t lim = getenv("EMURX_DEBUG_TABLE_LIMIT") ? strtoull(getenv("EMURX_DEBUG_TABLE_LIMIT"), nullptr, 0)
                                                                     : ~(size_t)0;
        for (int k = 0; k <= kNumTabs; ++k) {
            if (!img[k]->all) continue;
            while (img[k]->img.size() * 4 > lim || dev[k]->alloc(img[k]->img.size())) {
                if (k == kNumTabs || !m.shrink(k)) return EMURX_ENOMEM;
                // the out-of-memory status our own hipMalloc left pending: recovered from here
                if (hipPeekAtLastError() == hipErrorOutOfMemory) (void)hipGetLastError();
            }
            if (!EMURX_HIP_OK(hipMemcpy(dev[k]->p, img[k]->img.data(), img[k]->img.size() * 4, hipMemcpyHostToDevice)))
                return EMURX_EDEVICE;
            h->shipped_whole++;
        }
    }
    if (nd) {
        DeltaSlot& s = h->ring[h->ring_i++ % kDeltaRing];
        if (s.used && !EMURX_HIP_OK(hipEventSynchronize(s.ev))) return EMURX_EDEVICE;
        if (s.h.alloc(nd)) return EMURX_ENOMEM;
        size_t j = 0;
        for (int k = 0; k <= kNumTabs; ++k) {
            if (img[k]->all) continue;
            for (uint32_t b : img[k]->dirty) {
                emurx_delta& e = s.h.p[j++];
                e.dst = (uint64_t)(uintptr_t)(dev[k]->p + (size_t)b * EMURX_BUCKET_WORDS);
                e.pad = 0;
                memcpy(e.w, &img[k]->img[(size_t)b * EMURX_BUCKET_WORDS], sizeof(e.w));
            }
        }
        if (emurx_launch_apply(s.h.p, (uint32_t)nd, st) || !EMURX_HIP_OK(hipEventRecord(s.ev, st)))
            return EMURX_EDEVICE;
        s.used = true;
        h->shipped_blocks += nd;
    }
    m.clean_all();
    if (!EMURX_HIP_OK(hipEventRecord(h->ship_ev, st))) return EMURX_EDEVICE;
    waited_gen(h, st) = ++h->ship_gen;
    h->readers.clear();
    return EMURX_OK;
}

// Before a launch on `st` that reads the tables: ship pending edits, or wait for the last
// shipment if this stream has not yet; remember st as a reader for the next shipment.
int prepare_read(emurx_t* h, hipStream_t st) {
    int rc;
    if (h->m.pending()) {
        if ((rc = ship_tables(h, st))) return rc;
    } else {
        uint64_t& w = waited_gen(h, st);
        if (w < h->ship_gen) {
            if (!EMURX_HIP_OK(hipStreamWaitEvent(st, h->ship_ev, 0))) return EMURX_EDEVICE;
            w = h->ship_gen;
        }
    }
    if (std::find(h->readers.begin(), h->readers.end(), st) == h->readers.end()) {
        if (h->readers.size() >= kMaxReaders) {  // many distinct streams: drain them all once
            if (!EMURX_HIP_OK(hipDeviceSynchronize())) return EMURX_EDEVICE;
            h->readers.clear();
        }
        h->readers.push_back(st);
    }
    if (h->waited.size() > 4 * kMaxReaders) h->waited.clear();  // forgotten streams wait again: harmless
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
    if (h->stage_pending && hipEventQuery(h->stage_ev) == hipSuccess) {  // "not ready" is no error
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
        if (waves) {
            const bool narrow = mid * 100 <= waves;
            if (narrow != h->stage_narrow) {
                h->stage_same = 0;
                h->stage_every = 8;
            } else if (++h->stage_same >= 2 && h->stage_every < 256) {
                h->stage_every *= 2;
            }
            h->stage_narrow = narrow;
        }
    }
    // the first launch and then at most every stage_every-th copies its samples back
    if (!h->stage_pending &&
        (!h->stage_copy_gen || ((h->stage_gen - h->stage_copy_gen) & 0x3fffffffu) >= h->stage_every))
        h->stage_copy = true;
    return h->stage_narrow;
}
int stage_copy_back(emurx_t* h, hipStream_t st) {
    if (!h->stage_copy) return 0;
    h->stage_copy = false;
    if (!EMURX_HIP_OK(hipMemcpyAsync(h->stage_fb.p, h->d_stage_fb.p, 256 * sizeof(uint32_t), hipMemcpyDeviceToHost, st)) ||
        !EMURX_HIP_OK(hipEventRecord(h->stage_ev, st)))
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

// route scratch of stream st for batches of up to max_frames: per-tile counts, per-group sums
// (kept zero between routes) and group offsets.  A stream keeps its set; a new stream takes a
// free one, or the next in turn after waiting (on the device) for its last route.
int route_scratch(emurx_t* h, uint32_t n, hipStream_t st, emurx_t::RouteScratch** out) {
    const size_t gw = 1024 * 16, tiles = std::max<size_t>(ntiles(std::max(n, h->cfg.max_frames)), 1);
    if (tiles > 1024u * 64u) return EMURX_EINVAL;  // 16M frames per batch
    emurx_t::RouteScratch* r = nullptr;
    for (auto& x : h->route)
        if (x.used && x.st == st) r = &x;
    if (!r)
        for (auto& x : h->route)
            if (!r && !x.used) r = &x;
    if (!r) {
        r = &h->route[h->route_next++ % emurx_t::kRouteSets];
        if (!EMURX_HIP_OK(hipStreamWaitEvent(st, r->done, 0))) return EMURX_EDEVICE;
    }
    if (!r->done && !EMURX_HIP_OK(hipEventCreateWithFlags(&r->done, hipEventDisableTiming))) return EMURX_EDEVICE;
    r->st = st;
    r->used = true;
    if (!r->grp.p) {
        if (r->grp.alloc(gw) || !EMURX_HIP_OK(hipMemset(r->grp.p, 0, gw * sizeof(uint32_t)))) return EMURX_ENOMEM;
    }
    if (r->cnt.alloc(tiles * 16) || r->goff.alloc(gw) || r->tcur.alloc(EMURX_MAX_PARTS * EMURX_TAIL_SHARDS * EMURX_TAIL_CURSOR_STRIDE))
        return EMURX_ENOMEM;
    *out = r;
    return EMURX_OK;
}
// after a route's last launch on st: its scratch set may change hands behind this event
int route_done(emurx_t::RouteScratch* r, hipStream_t st) {
    return EMURX_HIP_OK(hipEventRecord(r->done, st)) ? EMURX_OK : EMURX_EDEVICE;
}

// A launch path may ship table edits (k_apply, cross-stream events, a synchronisation for a
// whole or grown table) and bakes the table addresses, which a later growth reallocates, into
// its kernel arguments: it must not be recorded into a hipGraph
int not_capturing(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (!EMURX_HIP_OK(hipStreamIsCapturing(st, &cs))) return EMURX_EDEVICE;
    return cs == hipStreamCaptureStatusNone ? EMURX_OK : EMURX_EINVAL;
}

// one k_rx launch; kind: 0 parse only, 1 classify, 2 parse + lookup keys (partitioned source);
// rt: kind 1 the route count pass fused in (emurx_classify_route_dev), kind 2 the packing
// of the lookup records (emurx_parse_route_dev)
int run_dev(emurx_t* h, const uint8_t* frames, const emurx_desc* desc, uint32_t n, const emurx_dev_out* out,
            hipStream_t st, int kind, const emurx_route_args* rt) {
    int rc;
    if ((rc = not_capturing(st))) return rc;
    if (kind == 1 && (rc = prepare_read(h, st))) return rc;
    emurx_dev_tables T = h->tables();
    const hipEvent_t* ev = nullptr;
    if (h->slots && (h->batch_seq++ % h->stride) == 0) {
        const uint32_t s = h->ev_head;
        ev = &h->ev[2 * s];
        h->ev_head = (s + 1) % h->slots;
        h->ev_count = std::min(h->ev_count + 1, h->slots);
    }
    const bool narrow = choose_stage(h);
    int r = emurx_launch_batch(frames, desc, n, T, kind, *out, st, ev, narrow, h->d_stage_fb.p, h->stage_gen, rt);
    if (!r) r = stage_copy_back(h, st);
    return r ? EMURX_EDEVICE : EMURX_OK;
}

int check_batch_args(emurx_t* h, const uint8_t* frames, const emurx_desc* desc, uint32_t n,
                     const emurx_dev_out* out) {
    if (!h || !out || !out->hist || (n && (!frames || !desc))) return EMURX_EINVAL;
    if (((uintptr_t)frames & 15) || ((uintptr_t)desc & 7)) return EMURX_EINVAL;  // 16-B staging loads
    if (n > h->cfg.max_frames) return EMURX_ENOMEM;
    if (out->qlist && out->qcap < queue_cap(n)) return EMURX_EINVAL;
    return bind(h);
}

// ---- batched ZMQ ingest (emurx_ingest_*; emurx_rx_stream uses the private last slot) ----
int ingest_buffer(emurx_t* h, uint32_t slot, size_t bytes, uint8_t** buf) {
    IngestSlot& s = h->ing[slot];
    if (s.pending || bytes > 0xFFFFFFFFull - 64) return EMURX_EINVAL;
    if (s.h_buf.alloc(bytes + 64) || s.d_buf.alloc(bytes + 64)) return EMURX_ENOMEM;
    *buf = s.h_buf.p;
    return EMURX_OK;
}

// Does a batch fit the one-launch path (k_ingest_small)?  At most EMURX_SMALL_MSGS messages and
// EMURX_SMALL_TILES tiles of descriptor slots, and every tile's messages (those with slots in
// it, and those whose status word it writes: tile min(base / 256, tiles - 1)) within the
// kernel's LDS budget, counted exactly as the kernel stages them: 16-byte vectors from the
// message's aligned start, plus two of slack.
bool small_fits(const uint32_t* ctl, uint32_t nmsg, uint32_t n, uint32_t max_tiles, uint32_t trange[EMURX_SMALL_TILES]) {
    if (nmsg > EMURX_SMALL_MSGS || n > std::min<uint32_t>(max_tiles, EMURX_SMALL_TILES) * EMURX_QUEUE_TILE) return false;
    const uint32_t nt = std::max<uint32_t>(ntiles(n), 1);
    const uint32_t* base = ctl + 2 * (size_t)nmsg;
    uint64_t vec[EMURX_SMALL_TILES] = {0};
    uint32_t lo[EMURX_SMALL_TILES], hi[EMURX_SMALL_TILES];
    for (uint32_t t = 0; t < nt; ++t) lo[t] = UINT32_MAX, hi[t] = 0;
    for (uint32_t m = 0; m < nmsg; ++m) {
        const uint32_t off = ctl[2 * m], len = ctl[2 * m + 1];
        const uint64_t v = len ? (((off & 15u) + (uint64_t)len + 15) >> 4) + 2 : 0;
        const uint32_t b0 = base[m], b1 = base[m + 1], ts = std::min(b0 / EMURX_QUEUE_TILE, nt - 1);
        uint32_t t0 = ts, t1 = ts;
        if (b1 > b0) {
            t0 = std::min(t0, b0 / EMURX_QUEUE_TILE);
            t1 = std::max(t1, std::min((b1 - 1) / EMURX_QUEUE_TILE, nt - 1));
        }
        for (uint32_t t = t0; t <= t1; ++t) {
            vec[t] += v;
            lo[t] = std::min(lo[t], m);
            hi[t] = std::max(hi[t], m);
        }
    }
    for (uint32_t t = 0; t < nt; ++t) {
        if (vec[t] * 16 > EMURX_SMALL_LDS) return false;
        trange[t] = lo[t] == UINT32_MAX ? 0u : lo[t] | ((hi[t] - lo[t] + 1) << 16);
    }
    return true;
}

// the result block of a batch of n descriptor slots and nmsg messages (256-byte aligned parts):
// allocates both copies and points the views into them
int set_results(IngestSlot& s, uint32_t n, uint32_t nmsg) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_desc = al((size_t)n * sizeof(emurx_rec)), o_q = o_desc + al((size_t)n * sizeof(emurx_desc));
    const size_t o_stat = o_q + al((size_t)n * 4), o_qoff = o_stat + al((size_t)nmsg * 4), o_hist = o_qoff + 256;
    const size_t total = o_hist + 2 * EMURX_HIST_BINS * sizeof(uint64_t);
    if (s.h_res.alloc(total) || s.d_res.alloc(total)) return EMURX_ENOMEM;
    uint8_t* hb = s.h_res.p;
    uint8_t* db = s.d_res.p;
    s.h_rec.p = reinterpret_cast<emurx_rec*>(hb);
    s.h_desc.p = reinterpret_cast<emurx_desc*>(hb + o_desc);
    s.h_qlist.p = reinterpret_cast<uint32_t*>(hb + o_q);
    s.h_stat.p = reinterpret_cast<uint32_t*>(hb + o_stat);
    s.h_qoff.p = reinterpret_cast<uint32_t*>(hb + o_qoff);
    s.h_hist.p = reinterpret_cast<uint64_t*>(hb + o_hist);
    s.d_rec.p = reinterpret_cast<emurx_rec*>(db);
    s.d_desc.p = reinterpret_cast<emurx_desc*>(db + o_desc);
    s.d_packed.p = reinterpret_cast<uint32_t*>(db + o_q);
    s.d_stat.p = reinterpret_cast<uint32_t*>(db + o_stat);
    s.d_qoff.p = reinterpret_cast<uint32_t*>(db + o_qoff);
    s.d_hist_out.p = reinterpret_cast<uint64_t*>(db + o_hist);
    s.res_bytes = total;
    return EMURX_OK;
}

int ingest_submit(emurx_t* h, uint32_t slot, const emurx_msg* msgs, uint32_t nmsg) {
    IngestSlot& s = h->ing[slot];
    if (s.pending || (nmsg && (!msgs || !s.h_buf.p))) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    if (!s.st && !EMURX_HIP_OK(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking))) return EMURX_EDEVICE;
    if (!s.done && !EMURX_HIP_OK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming))) return EMURX_EDEVICE;
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
    if (s.d_ctl.alloc((size_t)3 * nmsg + 1) || s.d_qlist.alloc(EMURX_NUM_QUEUES * qcap) ||
        s.d_tile_cnt.alloc((size_t)std::max<uint32_t>(nt, 1) * 16) ||
        s.d_seg_off.alloc((size_t)std::max<uint32_t>(nt, 1) * 16) || s.d_hist.alloc(hw) || set_results(s, n, nmsg) ||
        s.h_mframes.alloc(nmsg) || s.h_mstatus.alloc(nmsg))
        return EMURX_ENOMEM;
    hipStream_t st = s.st;
    if ((rc = prepare_read(h, st))) return rc;  // table deltas ordered against every reader
    // the pipeline's histogram shards start zeroed (k_qscan leaves them zero)
    if (fresh_hist && !EMURX_HIP_OK(hipMemsetAsync(s.d_hist.p, 0, hw * sizeof(uint64_t), st))) return EMURX_EDEVICE;
    uint32_t trange[EMURX_SMALL_TILES];
    if (h->ingest_small && small_fits(ctl, nmsg, n, h->small_tiles, trange)) {
        // one launch: control words and messages read from the pinned buffers, every result
        // written into the pinned result buffers (no copies)
        if (!s.d_ticket.p) {
            if (s.d_qseg.alloc((size_t)EMURX_SMALL_TILES * EMURX_NUM_QUEUES * EMURX_QUEUE_TILE) ||
                s.d_tcnt.alloc((size_t)EMURX_SMALL_TILES * 16) || s.d_hsmall.alloc(2 * EMURX_HIST_BINS) ||
                s.h_done.alloc(1) || s.d_ticket.alloc(3))
                return EMURX_ENOMEM;
            *(volatile uint32_t*)s.h_done.p = s.seq;
            if (!EMURX_HIP_OK(hipMemsetAsync(s.d_hsmall.p, 0, 2 * EMURX_HIST_BINS * sizeof(uint64_t), st)) ||
                !EMURX_HIP_OK(hipMemsetAsync(s.d_ticket.p, 0, 3 * sizeof(uint32_t), st)))
                return EMURX_EDEVICE;
        }
        if (emurx_launch_ingest_small(s.h_buf.p, ctl, nmsg, n, h->tables(), s.h_rec.p, s.h_desc.p, s.h_qlist.p,
                                      s.h_stat.p, s.h_qoff.p, s.h_hist.p, s.d_qseg.p, s.d_tcnt.p, s.d_hsmall.p,
                                      s.d_ticket.p, s.h_done.p, (s.seq + 1) & 0x7fffffffu,
                                      h->spin_base_us > 0 ? (uint32_t)((h->spin_base_us + 1e-4 * (double)end) * h->wall_khz / 1000.0) : 0u,
                                      trange, st) ||
            !EMURX_HIP_OK(hipEventRecord(s.done, st)))
            return EMURX_EDEVICE;
        s.seq = (s.seq + 1) & 0x7fffffffu;  // bit 31 of the completion word: the batch was degraded
        s.small = true;
        s.pending = true;
        s.nmsg = nmsg;
        s.slots = n;
        return EMURX_OK;
    }
    const auto H2D = hipMemcpyHostToDevice, D2H = hipMemcpyDeviceToHost;
    bool ok = EMURX_HIP_OK(hipMemcpyAsync(s.d_ctl.p, ctl, ((size_t)3 * nmsg + 1) * 4, H2D, st));
    if (end) ok = ok && EMURX_HIP_OK(hipMemcpyAsync(s.d_buf.p, s.h_buf.p, end, H2D, st));
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
    // every result in one copy: records, descriptors, packed queues, status, qoff, histogram
    ok = EMURX_HIP_OK(hipMemcpyAsync(s.h_res.p, s.d_res.p, s.res_bytes, D2H, st)) &&
         EMURX_HIP_OK(hipEventRecord(s.done, st));
    if (!ok) return EMURX_EDEVICE;
    s.small = false;
    s.pending = true;
    s.nmsg = nmsg;
    s.slots = n;
    return EMURX_OK;
}

// The small path's completion: spin on the pinned word k_ingest_small writes after every result
// (a few microseconds sooner than the end-of-kernel signal hipEventSynchronize waits for).
// Bounded: after 2 ms the caller waits on the event, which also reports a failed kernel.
bool spin_done(const uint32_t* word, uint32_t seq) {
    const volatile uint32_t* w = word;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 1;; ++k) {
        if ((*w & 0x7fffffffu) == seq) {
            std::atomic_thread_fence(std::memory_order_acquire);
            return true;
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
        if ((k & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) return false;
    }
}

int ingest_wait(emurx_t* h, uint32_t slot, emurx_ingest_result* res) {
    IngestSlot& s = h->ing[slot];
    if (!s.pending) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    s.pending = false;
    if (!(s.small && h->ingest_spin && spin_done(s.h_done.p, s.seq)) && !EMURX_HIP_OK(hipEventSynchronize(s.done)))
        return EMURX_EDEVICE;
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
    res->one_launch = s.small ? 1u : 0u;
    res->degraded = s.small ? (*(volatile uint32_t*)s.h_done.p >> 31) : 0u;
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

// handle internals for emurx_comm.cpp (emurx_kernels.h)
int emurx_handle_bind(emurx_t* h) { return bind(h); }
int emurx_handle_device(const emurx_t* h) { return h->host_only ? -1 : h->cfg.device; }
hipStream_t emurx_handle_stream(emurx_t* h) { return h->stream; }
emurx_comm_state*& emurx_handle_comm(emurx_t* h) { return h->comm; }

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
    case EMURX_ECOMM: return "RCCL communication error";
    default: return "unknown error";
    }
}

int emurx_open(const emurx_cfg* cfg, emurx_t** out) {
    if (!cfg || !out || cfg->max_ns == 0 || cfg->max_clients == 0 || cfg->max_frames == 0) return EMURX_EINVAL;
    emurx_t* h = new (std::nothrow) emurx_ctx();
    if (!h) return EMURX_ENOMEM;
    h->cfg = *cfg;
    if (h->cfg.max_bytes == 0) h->cfg.max_bytes = 1u << 20;
    h->host_only = cfg->device < 0;
    try {
        h->m.open(cfg->max_ns, cfg->max_clients);
    } catch (...) {
        delete h;
        return EMURX_ENOMEM;
    }
    if (h->host_only) {
        *out = h;
        return EMURX_OK;
    }
    int rc = bind(h);
    if (rc) { delete h; return rc; }
    if (!EMURX_HIP_OK(hipStreamCreate(&h->stream))) { delete h; return EMURX_EDEVICE; }
    if (const char* e = getenv("EMURX_STAGE")) h->stage_mode = !strcmp(e, "wide") ? 1 : !strcmp(e, "narrow") ? 2 : 0;
    if (const char* e = getenv("EMURX_INGEST_SMALL")) h->ingest_small = strcmp(e, "0") != 0;
    if (const char* e = getenv("EMURX_TXZ"))
        h->txz_mode = !strcmp(e, "wide") ? EMURX_TXZ_WIDE : !strcmp(e, "narrow") ? EMURX_TXZ_NARROW
                    : !strcmp(e, "long") ? EMURX_TXZ_LONG : -1;
    if (const char* e = getenv("EMURX_INGEST_SPIN")) h->ingest_spin = strcmp(e, "0") != 0;
    {
        // the one-launch ingest's wait bound in wall-clock ticks, and its grid cap
        int khz = 100000;
        if (EMURX_HIP_OK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, cfg->device)) && khz > 0)
            h->wall_khz = (uint32_t)khz;
        if (const char* e = getenv("EMURX_INGEST_SPIN_US")) h->spin_base_us = std::min(std::max(0.0, strtod(e, nullptr)), 1e6);
        const uint32_t cap = emurx_ingest_small_capacity(cfg->device);
        h->small_tiles = std::min<uint32_t>(EMURX_SMALL_TILES, cap);
    }
    if (h->stage_fb.alloc(256) || h->d_stage_fb.alloc(256) ||
        !EMURX_HIP_OK(hipEventCreateWithFlags(&h->stage_ev, hipEventDisableTiming)) ||
        !EMURX_HIP_OK(hipEventCreateWithFlags(&h->ship_ev, hipEventDisableTiming)) ||
        !EMURX_HIP_OK(hipMemset(h->d_stage_fb.p, 0, 256 * sizeof(uint32_t)))) {
        emurx_close(h);
        return EMURX_ENOMEM;
    }
    for (auto& s : h->ring)
        if (!EMURX_HIP_OK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming))) {
            emurx_close(h);
            return EMURX_EDEVICE;
        }
    memset(h->stage_fb.p, 0, 256 * sizeof(uint32_t));
    emurx_t::RouteScratch* rs = nullptr;
    if ((rc = ship_tables(h, h->stream)) || (rc = route_scratch(h, cfg->max_frames, h->stream, &rs)) == EMURX_ENOMEM) {
        emurx_close(h);
        return rc ? rc : EMURX_ENOMEM;
    }
    *out = h;
    return EMURX_OK;
}

void emurx_close(emurx_t* h) {
    if (!h) return;
    if (h->host_only) {
        delete h;
        return;
    }
    bind(h);
    (void)hipDeviceSynchronize();
    emurx_comm_free(h->comm);
    h->comm = nullptr;
    for (auto& s : h->ing) s.release();
    h->stage_fb.release();
    h->d_stage_fb.release();
    if (h->stage_ev) (void)hipEventDestroy(h->stage_ev);
    if (h->ship_ev) (void)hipEventDestroy(h->ship_ev);
    for (auto& s : h->ring) {
        s.h.release();
        if (s.ev) (void)hipEventDestroy(s.ev);
    }
    for (auto e : h->reader_ev) (void)hipEventDestroy(e);
    for (auto& t : h->d_tab) t.release();
    h->d_nsinfo.release();
    for (auto& r : h->route) r.release();
    h->d_txz.release();
    h->txz_fb.release();
    if (h->txz_ev) (void)hipEventDestroy(h->txz_ev);
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

// ---- tables (emurx_mirror.cpp: Go map semantics + device image edits) ----------------------
// CThreadCtx.AddNs / RemoveNs thread_ctx.go:786-812
int emurx_ns_add(emurx_t* h, const uint8_t key[12], uint32_t ns_id, uint32_t plugin_mask) {
    if (!h || !key) return EMURX_EINVAL;
    return h->m.ns_add(key, ns_id, plugin_mask);
}
int emurx_ns_remove(emurx_t* h, const uint8_t key[12]) {
    if (!h || !key) return EMURX_EINVAL;
    return h->m.ns_remove(key);
}
int emurx_ns_set_plugins(emurx_t* h, uint32_t ns_id, uint32_t plugin_mask) {
    if (!h) return EMURX_EINVAL;
    return h->m.ns_set_plugins(ns_id, plugin_mask);
}
// CNSCtx.AddClient ns_ctx.go:332-389
int emurx_client_add(emurx_t* h, uint32_t ns_id, uint32_t cid, const uint8_t mac[6], const uint8_t ipv4[4],
                     const uint8_t ipv6[16], const uint8_t dhcpv6[16], uint32_t plugin_mask) {
    if (!h || !mac) return EMURX_EINVAL;
    return h->m.client_add(ns_id, cid, mac, ipv4, ipv6, dhcpv6, plugin_mask);
}
// ctx_client_add rpc_base_cmds.go:350-406: the listed clients in order, stop at the first error
int emurx_clients_add(emurx_t* h, const emurx_client_spec* c, uint32_t n, uint32_t* n_added) {
    if (!h || (n && !c)) return EMURX_EINVAL;
    uint32_t k = 0;
    int rc = EMURX_OK;
    for (; k < n; ++k)
        if ((rc = h->m.client_add(c[k].ns_id, c[k].client_id, c[k].mac, c[k].ipv4, c[k].ipv6, c[k].dhcpv6,
                                  c[k].plugin_mask)))
            break;
    if (n_added) *n_added = k;
    return rc;
}
// CNSCtx.RemoveClient ns_ctx.go:392-440
int emurx_client_remove(emurx_t* h, uint32_t ns_id, const uint8_t mac[6]) {
    if (!h || !mac) return EMURX_EINVAL;
    return h->m.client_remove(ns_id, mac);
}
int emurx_client_set_plugins(emurx_t* h, uint32_t cid, uint32_t plugin_mask) {
    if (!h) return EMURX_EINVAL;
    return h->m.client_set_plugins(cid, plugin_mask);
}
// CNSCtx.UpdateClientIpv4 / Ipv6 / DIpv6 ns_ctx.go:442-533
int emurx_client_update_ipv4(emurx_t* h, uint32_t cid, const uint8_t ipv4[4]) {
    return h && ipv4 ? h->m.update_addr(cid, 4, ipv4) : EMURX_EINVAL;
}
int emurx_client_update_ipv6(emurx_t* h, uint32_t cid, const uint8_t ipv6[16]) {
    return h && ipv6 ? h->m.update_addr(cid, 6, ipv6) : EMURX_EINVAL;
}
int emurx_client_update_dipv6(emurx_t* h, uint32_t cid, const uint8_t d[16]) {
    return h && d ? h->m.update_addr(cid, 7, d) : EMURX_EINVAL;
}
int emurx_client_set_ra(emurx_t* h, uint32_t cid, const uint8_t prefix[16], uint8_t plen) {
    if (!h || !prefix) return EMURX_EINVAL;
    return h->m.client_set_ra(cid, prefix, plen);
}
// transport flow tables (TransportCtx.addFlowv4/6 / removeFlowv4/6 client_ctx.go:597-651,
// serverCb / lookupServerPort :1142-1155, GetTransportCtx socketApi.go:174-193)
int emurx_flow_add(emurx_t* h, uint32_t cid, const uint8_t* tuple, uint32_t tlen, uint32_t flow_id) {
    return h ? h->m.flow_add(cid, tuple, tlen, flow_id) : EMURX_EINVAL;
}
int emurx_flow_remove(emurx_t* h, uint32_t cid, const uint8_t* tuple, uint32_t tlen) {
    return h ? h->m.flow_remove(cid, tuple, tlen) : EMURX_EINVAL;
}
int emurx_server_add(emurx_t* h, uint32_t cid, uint16_t port, uint8_t proto) {
    return h ? h->m.server_add(cid, port, proto) : EMURX_EINVAL;
}
int emurx_server_remove(emurx_t* h, uint32_t cid, uint16_t port, uint8_t proto) {
    return h ? h->m.server_remove(cid, port, proto) : EMURX_EINVAL;
}
int emurx_client_set_transport(emurx_t* h, uint32_t cid, int has_ctx) {
    return h ? h->m.client_set_transport(cid, has_ctx != 0) : EMURX_EINVAL;
}

int emurx_sync(emurx_t* h, void* stream) {
    if (!h) return EMURX_EINVAL;
    if (h->host_only) return EMURX_OK;  // nothing to ship to
    int rc = bind(h);
    if (rc) return rc;
    return prepare_read(h, stream ? (hipStream_t)stream : h->stream);
}
int emurx_table_stats(const emurx_t* h, uint64_t* delta_blocks, uint64_t* whole_tables, uint64_t* image_bytes) {
    if (!h) return EMURX_EINVAL;
    if (delta_blocks) *delta_blocks = h->shipped_blocks;
    if (whole_tables) *whole_tables = h->shipped_whole;
    if (image_bytes) {
        uint64_t b = h->m.nsinfo.img.size() * 4;
        for (int k = 0; k < emurx_host::kNumTabs; ++k) b += h->m.hashes(k)->img.size() * 4;
        *image_bytes = b;
    }
    return EMURX_OK;
}
int emurx_set_partition(emurx_t* h, uint32_t n_parts, uint32_t part) {
    if (!h || n_parts == 0 || n_parts > EMURX_MAX_PARTS || part >= n_parts) return EMURX_EINVAL;
    h->m.set_partition(n_parts, part);
    return EMURX_OK;
}
uint64_t emurx_table_gen(const emurx_t* h) { return h ? h->m.gen : 0; }
int emurx_recs_stale(const emurx_t* h, const emurx_rec* rec, uint32_t n, uint64_t gen, uint8_t* stale) {
    if (!h || (n && (!rec || !stale))) return EMURX_EINVAL;
    for (uint32_t i = 0; i < n; ++i) stale[i] = h->m.stale(rec[i], gen) ? 1 : 0;
    return EMURX_OK;
}
int emurx_image_lookup(emurx_t* h, uint32_t table, const uint32_t* key, uint32_t* value) {
    if (!h) return EMURX_EINVAL;
    return h->m.image_lookup(table, key, value);
}
int emurx_image_check(emurx_t* h, uint64_t* mismatched) {
    using namespace emurx_host;
    if (!h || !mismatched) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    if ((rc = prepare_read(h, h->stream))) return rc;
    if (!EMURX_HIP_OK(hipStreamSynchronize(h->stream))) return EMURX_EDEVICE;
    uint64_t bad = 0;
    std::vector<uint32_t> buf;
    for (int k = 0; k <= kNumTabs; ++k) {
        const Blocks& b = k < kNumTabs ? *h->m.hashes(k) : h->m.nsinfo;
        const DevBuf<uint32_t>& d = k < kNumTabs ? h->d_tab[k] : h->d_nsinfo;
        buf.resize(b.img.size());
        if (b.img.size() > d.n) return EMURX_EDEVICE;
        if (!buf.empty() && !EMURX_HIP_OK(hipMemcpy(buf.data(), d.p, buf.size() * 4, hipMemcpyDeviceToHost)))
            return EMURX_EDEVICE;
        for (size_t i = 0; i < buf.size(); ++i) bad += buf[i] != b.img[i];
    }
    *mismatched = bad;
    return EMURX_OK;
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
    int rc = check_batch_args(h, d_frames, d_desc, n, out);
    if (rc) return rc;
    return run_dev(h, d_frames, d_desc, n, out, stream ? (hipStream_t)stream : h->stream, 1, nullptr);
}
int emurx_parse_dev(emurx_t* h, const uint8_t* d_frames, const emurx_desc* d_desc, uint32_t n,
                    const emurx_dev_out* out, void* stream) {
    int rc = check_batch_args(h, d_frames, d_desc, n, out);
    if (rc) return rc;
    return run_dev(h, d_frames, d_desc, n, out, stream ? (hipStream_t)stream : h->stream, 0, nullptr);
}

int emurx_classify_route_dev(emurx_t* h, const uint8_t* d_frames, const emurx_desc* d_desc, uint32_t n,
                             const emurx_dev_out* out, uint32_t n_parts, uint32_t my_rank, uint32_t cap,
                             emurx_route_rec* d_send, uint32_t* d_send_count, void* stream) {
    int rc = check_batch_args(h, d_frames, d_desc, n, out);
    if (rc) return rc;
    if (!out->rec || !d_send_count || n_parts == 0 || n_parts > EMURX_MAX_PARTS || my_rank >= n_parts ||
        (n && (!d_send || cap == 0)) || ((uintptr_t)d_send & 7))
        return EMURX_EINVAL;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    // before anything is enqueued: nothing of a refused call may end up in the caller's graph
    if ((rc = not_capturing(st))) return rc;
    emurx_t::RouteScratch* rs = nullptr;
    if ((rc = route_scratch(h, n, st, &rs))) return rc;
    const emurx_route_args rt{n_parts, my_rank, cap, rs->cnt.p, rs->grp.p, nullptr, nullptr};
    if (n && (rc = run_dev(h, d_frames, d_desc, n, out, st, 1, &rt))) {
        // k_rx may have added its owner counts into grp before the failure; only k_route_scan
        // clears them, so clear them here or the next route on this set starts from garbage
        (void)hipMemsetAsync(rs->grp.p, 0, rs->grp.n * sizeof(uint32_t), st);
        return rc;
    }
    if (emurx_launch_route(out->rec, n, n_parts, my_rank, cap, d_send, d_send_count, rs->cnt.p, rs->grp.p,
                           rs->goff.p, st, true)) {
        (void)hipMemsetAsync(rs->grp.p, 0, rs->grp.n * sizeof(uint32_t), st);
        return EMURX_EDEVICE;
    }
    return route_done(rs, st);
}

// the whole send / receive buffer of n_parts lookup regions in 32-byte units fits 32 bits (k_rx
// kind 2 addresses heads by such units)
static bool lookup_regions_fit(uint32_t n_parts, uint32_t cap, uint32_t tail_cap) {
    return EMURX_LOOKUP_REGION_BYTES(cap, tail_cap) / 32 * n_parts < (1ull << 32) &&
           (uint64_t)EMURX_TAIL_SHARDS * tail_cap < (1ull << 32) - 4;
}

int emurx_parse_route_dev(emurx_t* h, const uint8_t* d_frames, const emurx_desc* d_desc, uint32_t n,
                          const emurx_dev_out* out, uint32_t n_parts, uint32_t my_rank, uint32_t cap,
                          uint32_t tail_cap, emurx_lookup_rec* d_send, uint32_t* d_send_count, void* stream) {
    int rc = check_batch_args(h, d_frames, d_desc, n, out);
    if (rc) return rc;
    if (!d_send_count || n_parts == 0 || n_parts > EMURX_MAX_PARTS || my_rank >= n_parts ||
        (n && (!d_send || cap == 0)) || ((uintptr_t)d_send & 15) || !lookup_regions_fit(n_parts, cap, tail_cap))
        return EMURX_EINVAL;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    // before anything is enqueued: nothing of a refused call may end up in the caller's graph
    if ((rc = not_capturing(st))) return rc;
    emurx_t::RouteScratch* rs = nullptr;
    if ((rc = route_scratch(h, n, st, &rs))) return rc;
    // owner counts from the L2 headers + group scan, then k_rx packs at those offsets
    if (emurx_launch_owner_count(d_frames, d_desc, n, n_parts, d_send_count, rs->cnt.p, rs->grp.p, rs->goff.p,
                                 rs->tcur.p, st))
        return EMURX_EDEVICE;
    // tcp / udp heads carry their c5tuplekey while ANY client has a TransportCtx: the maps are
    // complete on every partition's handle, the flow tables only on the owner's
    const uint32_t tup_on = h->m.n_ctx_all ? 1u : 0u;
    const emurx_route_args rt{n_parts, my_rank, cap, rs->cnt.p, rs->grp.p, rs->goff.p, d_send,
                              tail_cap, rs->tcur.p, d_send_count, tup_on};
    if (n && (rc = run_dev(h, d_frames, d_desc, n, out, st, 2, &rt))) return rc;
    return route_done(rs, st);
}

int emurx_zmq_walk_dev(emurx_t* h, const uint8_t* d_buf, const uint32_t* d_ctl, uint32_t nmsg, emurx_desc* d_desc,
                       uint32_t* d_msg_stat, uint32_t flags, void* stream) {
    if (!h || (nmsg && (!d_buf || !d_ctl || !d_desc || !d_msg_stat)) || ((uintptr_t)d_desc & 7) ||
        ((uintptr_t)d_ctl & 7) || (flags & ~EMURX_WALK_NO_KEYS))
        return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    if ((rc = not_capturing(st))) return rc;
    return emurx_launch_zmq_walk(d_buf, d_ctl, nmsg, d_desc, d_msg_stat, st, !(flags & EMURX_WALK_NO_KEYS))
               ? EMURX_EDEVICE
               : EMURX_OK;
}

int emurx_lookup_dev(emurx_t* h, const emurx_lookup_rec* d_recv, const uint32_t* d_recv_count, uint32_t n_parts,
                     uint32_t cap, uint32_t tail_cap, emurx_route_rec* d_out, uint32_t* d_flow, void* stream) {
    if (!h || !d_recv_count || n_parts == 0 || n_parts > EMURX_MAX_PARTS || (cap && (!d_recv || !d_out)) ||
        ((uintptr_t)d_recv & 15) || ((uintptr_t)d_out & 7) || !lookup_regions_fit(n_parts, cap, tail_cap))
        return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    if ((rc = not_capturing(st)) || (rc = prepare_read(h, st))) return rc;
    return emurx_launch_lookup(d_recv, d_recv_count, n_parts, cap, tail_cap, h->tables(), d_out, d_flow, st) ? EMURX_EDEVICE
                                                                                                    : EMURX_OK;
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
int emurx_ingest_stream(emurx_t* h, uint32_t slot, void** stream) {
    if (!h || !stream || slot >= EMURX_INGEST_SLOTS) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    IngestSlot& s = h->ing[slot];
    if (!s.st && !EMURX_HIP_OK(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking))) return EMURX_EDEVICE;
    *stream = (void*)s.st;
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
    (void)hipDeviceSynchronize();
    for (auto& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    h->ev.assign((size_t)slots * 2, nullptr);
    // timing only: no system-scope fence at the record (on gfx950 that fence is a cache
    // write-back and invalidate, which both inflated the bracketed launch and slowed the next)
    for (auto& e : h->ev)
        if (!EMURX_HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence))) { h->slots = 0; return EMURX_EDEVICE; }
    h->slots = slots;
    h->stride = stride ? stride : 1;
    h->ev_head = h->ev_count = h->batch_seq = 0;
    return EMURX_OK;
}

uint32_t emurx_last_stage(const emurx_t* h) { return h ? h->last_stage : 0; }
int32_t emurx_last_txz(const emurx_t* h) {
    if (!h || h->last_txz < 0) return -1;
    return h->last_txz == EMURX_TXZ_NARROW ? 4608 : h->last_txz == EMURX_TXZ_LONG ? 0 : 6144;
}

int emurx_kernel_times(emurx_t* h, float* batch_ms, uint32_t cap, uint32_t* n_out) {
    if (!h || !n_out || (cap && !batch_ms)) return EMURX_EINVAL;
    *n_out = 0;
    if (!h->slots || !h->ev_count) return EMURX_OK;
    int rc = bind(h);
    if (rc) return rc;
    const uint32_t last = (h->ev_head + h->slots - 1) % h->slots;
    if (!EMURX_HIP_OK(hipEventSynchronize(h->ev[2 * last + 1]))) return EMURX_EDEVICE;
    const uint32_t n = std::min(h->ev_count, cap);
    const uint32_t first = (h->ev_head + h->slots - h->ev_count) % h->slots;
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t s = (first + (h->ev_count - n) + k) % h->slots;
        if (!EMURX_HIP_OK(hipEventElapsedTime(&batch_ms[k], h->ev[2 * s], h->ev[2 * s + 1])))
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
    if (n >= EMURX_TX_ZMQ_MAX_FRAMES || ((uintptr_t)d_out & 15) || ((uintptr_t)d_desc & 7)) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    const size_t need = emurx_txz_scratch_bytes(n);
    if (need > h->d_txz.n) {  // grows on demand; a launch in flight may still read the old one
        (void)hipStreamSynchronize(st);
        if (h->d_txz.alloc(need)) return EMURX_ENOMEM;
        // the chain's arrival counters (and the feedback words) start at zero (each call's last
        // arrival resets its own counter)
        if (!EMURX_HIP_OK(hipMemset(h->d_txz.p, 0, need))) return EMURX_EDEVICE;
        h->txz_pending = false;
    }
    if (!h->txz_ev && (h->txz_fb.alloc(2) || !EMURX_HIP_OK(hipEventCreateWithFlags(&h->txz_ev, hipEventDisableTiming))))
        return EMURX_ENOMEM;
    if (h->txz_pending && hipEventQuery(h->txz_ev) == hipSuccess) {  // "not ready" is no error
        h->txz_pending = false;
        // hi: the largest upper bound of a sampled tile's output rows; lo: the smallest lower
        // bound (0 words: nothing sampled, the choice stands)
        const uint32_t hi = h->txz_fb.p[0], lo = ~h->txz_fb.p[1];
        const int v = !hi                                ? h->txz_variant
                      : hi <= emurx_txz_img_narrow_rows ? EMURX_TXZ_NARROW
                      : lo > emurx_txz_img_wide_rows    ? EMURX_TXZ_LONG
                                                        : EMURX_TXZ_WIDE;
        if (v != h->txz_variant) {
            h->txz_same = 0;
            h->txz_every = 8;
        } else if (++h->txz_same >= 2 && h->txz_every < 256) {
            h->txz_every *= 2;
        }
        h->txz_variant = v;
    }
    const bool fb = h->txz_mode < 0 && n && !h->txz_pending && (!h->txz_calls || h->txz_calls - h->txz_last_copy >= h->txz_every);
    ++h->txz_calls;
    const int variant = h->txz_mode >= 0 ? h->txz_mode : h->txz_variant;
    if (emurx_launch_tx_zmq(d_frames, d_desc, n, d_out, out_cap, d_msg_off, d_info, h->d_txz.p, st, variant, fb))
        return EMURX_EDEVICE;
    h->last_txz = variant;
    if (fb) {  // the two words behind this call, then cleared for the next sample
        if (!EMURX_HIP_OK(hipMemcpyAsync(h->txz_fb.p, h->d_txz.p, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st)) ||
            !EMURX_HIP_OK(hipMemsetAsync(h->d_txz.p, 0, 2 * sizeof(uint32_t), st)) ||
            !EMURX_HIP_OK(hipEventRecord(h->txz_ev, st)))
            return EMURX_EDEVICE;
        h->txz_pending = true;
        h->txz_last_copy = h->txz_calls;
    }
    return EMURX_OK;
}

uint32_t emurx_ns_owner(const uint8_t key[12], uint32_t n_parts) {
    if (!key || n_parts == 0) return 0;
    return emurx_owner(emurx_tk_hash(le32(key), le32(key + 4), le32(key + 8)), n_parts);
}
uint8_t emurx_owner_key(const uint8_t key[12]) {
    if (!key) return 0;
    return (uint8_t)emurx_owner_key(emurx_tk_hash(le32(key), le32(key + 4), le32(key + 8)));
}
int emurx_desc_keys_dev(emurx_t* h, const uint8_t* d_frames, emurx_desc* d_desc, uint32_t n, void* stream) {
    if (!h || (n && (!d_frames || !d_desc)) || ((uintptr_t)d_desc & 7)) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    return emurx_launch_desc_keys(d_frames, d_desc, n, stream ? (hipStream_t)stream : h->stream) ? EMURX_EDEVICE
                                                                                                 : EMURX_OK;
}

int emurx_route_dev(emurx_t* h, const emurx_rec* d_rec, uint32_t n, uint32_t n_parts, uint32_t my_rank,
                    uint32_t cap, emurx_route_rec* d_send, uint32_t* d_send_count, void* stream) {
    if (!h || !d_send_count || n_parts == 0 || n_parts > EMURX_MAX_PARTS || my_rank >= n_parts ||
        (n && (!d_rec || !d_send || cap == 0)))
        return EMURX_EINVAL;
    if (((uintptr_t)d_rec & 15) || ((uintptr_t)d_send & 7)) return EMURX_EINVAL;
    int rc = bind(h);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    // before anything is enqueued: nothing of a refused call may end up in the caller's graph
    if ((rc = not_capturing(st))) return rc;
    emurx_t::RouteScratch* rs = nullptr;
    if ((rc = route_scratch(h, n, st, &rs))) return rc;
    if (emurx_launch_route(d_rec, n, n_parts, my_rank, cap, d_send, d_send_count, rs->cnt.p, rs->grp.p, rs->goff.p,
                           st, false))
        return EMURX_EDEVICE;
    return route_done(rs, st);
}

}  // extern "C"
