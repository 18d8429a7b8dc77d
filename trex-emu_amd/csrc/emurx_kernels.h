// emurx_kernels.h — launcher of the rx parse / classify / queue kernel (emurx_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <tuple>
#include <type_traits>
#include <utility>

#include "../../include/emu_rx.h"
#include "emurx_tables.h"

// HIP status check of the host code: false on failure.  EMURX_DEBUG=1 names the failing call
// (file:line and HIP's message) on stderr; the entry points still return EMURX_EDEVICE.
inline bool emurx_hip_ok(hipError_t e, const char* file, int line) {
    if (e == hipSuccess) return true;
    static const bool dbg = getenv("EMURX_DEBUG") != nullptr;
    if (dbg) fprintf(stderr, "emurx: HIP error at %s:%d: %s\n", file, line, hipGetErrorString(e));
    return false;
}
#define EMURX_HIP_OK(x) emurx_hip_ok((x), __FILE__, __LINE__)

// One kernel launch whose status is the return value of hipLaunchKernel: the launchers never
// read or clear the thread's last-error state, so an error a caller's own earlier HIP call
// left pending stays pending for the caller (and is not taken for this launch's).
template <typename... P, typename... A>
inline hipError_t emurx_launch(void (*k)(P...), dim3 grid, dim3 block, size_t lds, hipStream_t st, A&&... a) {
    static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
    std::tuple<std::decay_t<P>...> args{std::forward<A>(a)...};
    return std::apply(
        [&](auto&... e) {
            void* p[] = {(void*)&e...};
            return hipLaunchKernel((const void*)k, grid, block, p, lds, st);
        },
        args);
}

// Enqueue one batch on `st`: a single k_rx launch, no host synchronisation (capturable in a
// hipGraph).  ev[0..1] (optional) are recorded before and after it.  narrow: the 6 KiB
// staging slab (6 workgroups per CU) instead of 7 KiB (5).  fb (optional, host-visible,
// 64 * 4 words): the sampled tiles' stage feedback, tagged with gen.  Returns 0 or -1.
// rt (optional, classify only): the route count pass fused into k_rx: per-(tile, owner) counts
// into cnt[ntiles * 16] and per-group sums added into grp (as emurx_launch_route's first pass).
// kind: 0 parse only, 1 parse + classify, 2 parse + lookup keys.
// rt (optional): kind 1: the route count pass fused in (per-(tile, owner) counts into cnt,
// per-group sums added into grp, as emurx_launch_route's first pass); kind 2 (required): the
// owner counts cnt / group offsets goff of k_owner_count + k_route_scan, and every frame's
// 32-byte emurx_lookup_rec head (emurx_parse.h pack_lookup) packed into region `owner` of send
// (EMURX_LOOKUP_REGION_BYTES(cap, tcap) bytes each), its tail units at the units its wave took
// from tcur[(owner * EMURX_TAIL_SHARDS + shard) * EMURX_TAIL_CURSOR_STRIDE] (a line each: the
// atomics of different cursors do not serialise on one line); count: the send counts (stride 2), where an
// overflowing tail shard records the units it needed.
struct emurx_route_args {
    uint32_t parts, rank, cap;
    uint32_t* cnt;
    uint32_t* grp;
    const uint32_t* goff;
    emurx_lookup_rec* send;
    uint32_t tcap;
    uint32_t* tcur;
    uint32_t* count;
    uint32_t tup_on;  // some client has a TransportCtx: tcp / udp heads carry their c5tuplekey tail
};
int emurx_launch_batch(const uint8_t* frames, const emurx_desc* desc, uint32_t n,
                       const emurx_dev_tables& T, int kind, const emurx_dev_out& out,
                       hipStream_t st, const hipEvent_t* ev, bool narrow, uint32_t* fb, uint32_t gen,
                       const emurx_route_args* rt = nullptr);

// One edited 64-byte table block (emurx_api.cpp ship_tables): k_apply copies w to dst.
struct emurx_delta {
    uint64_t dst;   // device address of the block (64-byte aligned)
    uint64_t pad;
    uint32_t w[16];
};  // 80 bytes
int emurx_launch_apply(const emurx_delta* d, uint32_t n, hipStream_t st);

// Enqueue the Namespace-partition packing of a classified batch (emurx_route.hip): three
// launches on `st`.  Scratch: tile_cnt [ceil(n / 256) * 16]; grp, grp_off [groups * 16] with
// groups = ceil(n / 16384) <= 1024 (n <= 16M); grp must be zero (the launches leave it zero).
int emurx_launch_route(const emurx_rec* rec, uint32_t n, uint32_t n_parts, uint32_t my_rank, uint32_t cap,
                       emurx_route_rec* send, uint32_t* send_count, uint32_t* tile_cnt, uint32_t* grp,
                       uint32_t* grp_off, hipStream_t st, bool counted = false);
// The owner counts of the partitioned source (emurx_parse_route_dev): k_owner_count (the
// CTunnelKey of every frame from its L2 header alone, counted per (tile, owner) and per group)
// + k_route_scan -> tile_cnt, grp_off, send_count; k_rx kind 2 then packs.  Two launches.
// send_count: [2 n_parts] {heads, tail overflow}; tcur [n_parts * EMURX_TAIL_SHARDS] cleared.
int emurx_launch_owner_count(const uint8_t* frames, const emurx_desc* desc, uint32_t n, uint32_t n_parts,
                             uint32_t* send_count, uint32_t* tile_cnt, uint32_t* grp, uint32_t* grp_off,
                             uint32_t* tcur, hipStream_t st);
// The owner keys of device-resident descriptors (emurx_desc_keys_dev), in place.  One launch.
int emurx_launch_desc_keys(const uint8_t* frames, emurx_desc* desc, uint32_t n, hipStream_t st);
// The owner side (emurx_lookup_dev): one lane per received head, n_parts regions of
// EMURX_LOOKUP_REGION_BYTES(cap, tcap) bytes; recv_count stride 2 (heads, tail overflow).
int emurx_launch_lookup(const emurx_lookup_rec* recv, const uint32_t* recv_count, uint32_t n_parts, uint32_t cap,
                        uint32_t tcap, const emurx_dev_tables& T, emurx_route_rec* out, uint32_t* flow,
                        hipStream_t st);

// Batched ZMQ ingest (emurx_ingest.hip).  zmq_walk: one lane per message; ctl = emurx_msg[nmsg]
// then slot_base[nmsg + 1]; writes desc[slot_base[m] ..) (holes marked EMURX_DESC_HOLE) and
// msg_stat[m] = frames | EMURX_MSG_* << 24.  The buffer must be readable 32 bytes past every message.
// keys = false: descriptors without owner keys (the measurement of their cost only).
int emurx_launch_zmq_walk(const uint8_t* buf, const uint32_t* ctl, uint32_t nmsg, emurx_desc* desc,
                          uint32_t* msg_stat, hipStream_t st, bool keys = true);
// A small batch (at most EMURX_SMALL_TILES tiles, EMURX_SMALL_MSGS messages, every tile's messages within the
// kernel's LDS budget: emurx_ingest_small_fits) in ONE launch: messages and control words read
// from pinned host memory, walk + parse + classify + queue packing, every result written into
// pinned host memory (h_*: the layout of the pipeline's D2H copies).  Device scratch: d_qseg
// [EMURX_SMALL_TILES * 13 * 256], d_tcnt [EMURX_SMALL_TILES * 16], d_hist [128] and d_ticket [3] (ticket,
// arrivals, degraded),
// zero before the first launch (each launch leaves them zero).  h_done (pinned host): seq
// (< 2^31) is written there after every result, bit 31 set when the batch was degraded (the
// host may spin on it instead of the stream).  spin_ticks: the 100 MHz wall-clock ticks a
// workgroup waits for every tile's arrival before it takes the degraded pack (0: at once).  trange[t]
// (emurx_ingest_tile_ranges): tile t's first message | its message count << 16.
#ifndef EMURX_SMALL_TILES
#define EMURX_SMALL_TILES 256
#endif
#define EMURX_SMALL_LDS 40960
#define EMURX_SMALL_MSGS 1024
int emurx_launch_ingest_small(const uint8_t* h_buf, const uint32_t* h_ctl, uint32_t nmsg, uint32_t n,
                              const emurx_dev_tables& T, emurx_rec* h_rec, emurx_desc* h_desc, uint32_t* h_qlist,
                              uint32_t* h_stat, uint32_t* h_qoff, uint64_t* h_hist, uint32_t* d_qseg, uint32_t* d_tcnt,
                              uint64_t* d_hist, uint32_t* d_ticket, uint32_t* h_done, uint32_t seq,
                              uint32_t spin_ticks, const uint32_t* trange, hipStream_t st);
// k_ingest_small's workgroups resident at once on `device` (0 when unknown)
uint32_t emurx_ingest_small_capacity(int device);
// Concatenate k_rx's per-tile queue segments (queue-major, frame order) into `packed`, write
// qoff[EMURX_NUM_QUEUES + 1], fold the histogram shards into hist_out[2 * EMURX_HIST_BINS] and
// clear the shards.  Scratch seg_off: [ceil(n / 256) * 16].  Two launches.
int emurx_launch_queue_pack(const uint32_t* qlist, uint32_t qcap, const uint32_t* tile_cnt, uint32_t n,
                            uint32_t* seg_off, uint32_t* packed, uint32_t* qoff, uint64_t* hist,
                            uint64_t* hist_out, hipStream_t st);

// The handle internals the communicator (emurx_comm.cpp) uses; defined in emurx_api.cpp.
struct emurx_comm_state;
int emurx_handle_bind(emurx_t* h);           // make the handle's device current (EMURX_OK / error)
int emurx_handle_device(const emurx_t* h);   // its device ordinal (< 0: host-only handle)
hipStream_t emurx_handle_stream(emurx_t* h);  // its own stream
emurx_comm_state*& emurx_handle_comm(emurx_t* h);
void emurx_comm_free(emurx_comm_state* c);   // emurx_comm.cpp: destroy a communicator

// Tx checksum generation (emurx_tx.hip): one launch, in place; status may be null.
int emurx_launch_tx_csum(uint8_t* frames, const emurx_tx_desc* desc, uint32_t n, uint8_t* status,
                         hipStream_t st);

// Tx ZMQ framing (emurx_txzmq.hip): see emurx_tx_zmq_dev.  scratch: emurx_txz_scratch_bytes(n).
size_t emurx_txz_scratch_bytes(uint32_t n);
// variant: the write kernel's image (EMURX_TXZ_*, emurx_tx_zmq_dev's feedback choice); feedback:
// the chain kernel also folds the bounds of its tiles' output rows into scratch words 0 (largest
// upper bound, atomicMax) and 1 (~ the smallest lower bound), which the caller copies back and
// clears (emurx_txz_feedback_words)
enum { EMURX_TXZ_WIDE = 0, EMURX_TXZ_NARROW = 1, EMURX_TXZ_LONG = 2 };
constexpr uint32_t emurx_txz_img_narrow_rows = 4608 / 16, emurx_txz_img_wide_rows = 6144 / 16;
int emurx_launch_tx_zmq(const uint8_t* frames, const emurx_desc* desc, uint32_t n, uint8_t* out, uint64_t cap,
                        uint64_t* msg_off, uint64_t* info, void* scratch, hipStream_t st, int variant = EMURX_TXZ_WIDE,
                        bool feedback = false);
