// emurx_comm.cpp — the library-owned communicator of the Namespace-owner exchange.
//
// The reference has no collective: one process, one main goroutine owns every table
// (src/emu/core/thread_ctx.go:139 MapNsT, :397-419 MainLoop, :772-784 GetNs; the single-goroutine
// assert parser.go:986-991).  Sharding the receive path over the GPUs of a node adds one exchange
// step: every frame's lookup record travels to the GPU that owns its Namespace partition.  This
// file puts that step behind the C-ABI so that a Go caller (cgo) drives it like every other
// entry point, with no Python or torch.distributed in between:
//
//   one process per GPU   emurx_comm_unique_id on one rank, the 128 bytes sent out of band,
//                         emurx_comm_init(h, id, nranks, rank) on every rank (ncclCommInitRank)
//   one process, N GPUs   emurx_comm_init_all(handles, n) (ncclCommInitAll over the handles'
//                         devices): the reference's process model; the exchanges of the N
//                         handles then go between emurx_group_start / emurx_group_end
//
// emurx_exchange_dev moves the regions emurx_parse_route_dev (or emurx_classify_route_dev)
// packed: RCCL point-to-point over xGMI (ncclSend / ncclRecv to every peer inside one
// ncclGroupStart / ncclGroupEnd, so the seven links of an MI355X run at once), the own region by
// a device copy.  EMURX_XCH_EQUAL (default) sends whole regions and never waits on the host;
// EMURX_XCH_PAYLOAD exchanges the counts first, waits for them, then sends only the spans that
// carry data (SURVEY §8e's all-to-all-v).
//
// RCCL is bound at the first communicator call (dlopen of librccl.so.1, the one already in the
// process if any), not when libemurx.so is loaded: linked as a load-time dependency, librccl
// pulled ROCm's own rocm-smi / roctx / HIP runtime into every process that loaded libemurx.so
// ahead of torch's bundled copies, and such a process aborted at exit (a double free in the
// mixed runtime libraries).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <type_traits>
#include <vector>

#include "../../include/emu_rx.h"
#include "emurx_kernels.h"

// Every RCCL operation of a communicator runs on its own stream (`st`), joined to the caller's
// stream by events both ways: two exchanges the caller issues on different streams (the bench's
// two buffer sets) then reach RCCL in issue order and never run side by side on one
// communicator, as every rank must see them.
struct emurx_comm_state {
    emurx_t* h = nullptr;
    ncclComm_t comm = nullptr;
    uint32_t nranks = 0, rank = 0;
    bool self_rccl = false;     // the own region through RCCL too (EMURX_COMM_SELF=rccl: a 1-rank
                                // communicator then drives RCCL's send / receive path)
    uint32_t* h_counts = nullptr;  // pinned: send + receive counts (payload mode)
    hipStream_t st = nullptr;      // the communicator's stream
    hipEvent_t ev = nullptr;       // counts landed (payload mode)
    hipEvent_t ev_in = nullptr;    // the caller's stream up to the exchange
    hipEvent_t ev_out = nullptr;   // the exchange done
};

namespace {

// the RCCL entry points this file calls, resolved once
struct Rccl {
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    char path[512] = {0};
};
const Rccl* rccl() {
    static Rccl r;
    static bool ok = false;
    static std::once_flag once;
    std::call_once(once, [] {
        void* so = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!so) so = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!so) return;
        bool all = true;
        auto get = [&](auto& f, const char* name) {
            f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(so, name));
            all = all && f != nullptr;
        };
        get(r.GetUniqueId, "ncclGetUniqueId");
        get(r.CommInitRank, "ncclCommInitRank");
        get(r.CommInitAll, "ncclCommInitAll");
        get(r.CommDestroy, "ncclCommDestroy");
        get(r.GetErrorString, "ncclGetErrorString");
        get(r.GroupStart, "ncclGroupStart");
        get(r.GroupEnd, "ncclGroupEnd");
        get(r.Send, "ncclSend");
        get(r.Recv, "ncclRecv");
        Dl_info di;
        if (all && dladdr(reinterpret_cast<void*>(r.GetUniqueId), &di) && di.dli_fname)
            snprintf(r.path, sizeof(r.path), "%s", di.dli_fname);
        ok = all;
    });
    return ok ? &r : nullptr;
}

thread_local int g_group_depth = 0;  // emurx_group_start nesting on this thread
// exchanges issued inside an open group: their RCCL kernels are launched by the outermost
// emurx_group_end, so the caller's stream is joined to the communicator's stream there
struct Pending {
    emurx_comm_state* c;
    hipStream_t user;
};
thread_local std::vector<Pending> g_pending;

// the caller's stream waits for everything enqueued so far on the communicator's stream
int join_back(emurx_comm_state* c, hipStream_t user) {
    if (emurx_handle_bind(c->h)) return EMURX_EDEVICE;
    return EMURX_HIP_OK(hipEventRecord(c->ev_out, c->st)) && EMURX_HIP_OK(hipStreamWaitEvent(user, c->ev_out, 0))
               ? EMURX_OK
               : EMURX_EDEVICE;
}

bool nccl_ok(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return true;
    static const bool dbg = getenv("EMURX_DEBUG") != nullptr;
    if (dbg) fprintf(stderr, "emurx: RCCL %s: %s\n", what, rccl() ? rccl()->GetErrorString(r) : "?");
    return false;
}

int new_state(emurx_t* h, uint32_t nranks, uint32_t rank, emurx_comm_state** out) {
    auto* c = new (std::nothrow) emurx_comm_state();
    if (!c) return EMURX_ENOMEM;
    c->h = h;
    c->nranks = nranks;
    c->rank = rank;
    const char* e = getenv("EMURX_COMM_SELF");
    c->self_rccl = e && !strcmp(e, "rccl");
    // ev_in / ev_out order two streams of one device (the caller's and the communicator's): a
    // device-scope release is enough, and the default system-scope one writes back and
    // invalidates the caches at every exchange (EMURX_COMM_FENCE=system restores it).  The
    // counts event (payload mode) is waited for by the host after a copy to pinned memory:
    // system scope
    const char* f = getenv("EMURX_COMM_FENCE");
    const unsigned order = hipEventDisableTiming | (f && !strcmp(f, "system") ? 0u : hipEventDisableSystemFence);
    if (!EMURX_HIP_OK(hipHostMalloc((void**)&c->h_counts, 4 * EMURX_MAX_PARTS * sizeof(uint32_t), hipHostMallocDefault)) ||
        !EMURX_HIP_OK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking)) ||
        !EMURX_HIP_OK(hipEventCreateWithFlags(&c->ev, hipEventDisableTiming)) ||
        !EMURX_HIP_OK(hipEventCreateWithFlags(&c->ev_in, order)) ||
        !EMURX_HIP_OK(hipEventCreateWithFlags(&c->ev_out, order))) {
        emurx_comm_free(c);
        return EMURX_EDEVICE;
    }
    *out = c;
    return EMURX_OK;
}

// one region's spans that carry data: the first min(count, cap) records and, for lookup
// regions, the tail shards (their units are taken by atomics: which are used is known on the
// device only)
int spans(uint32_t count, uint32_t cap, uint64_t rb, uint64_t heads_end, uint64_t region, uint64_t a[2], uint64_t b[2]) {
    int k = 0;
    const uint64_t h = (uint64_t)(count < cap ? count : cap) * rb;
    if (h) a[k] = 0, b[k++] = h;
    if (region > heads_end) a[k] = heads_end, b[k++] = region;
    return k;
}

}  // namespace

void emurx_comm_free(emurx_comm_state* c) {
    if (!c) return;
    const Rccl* R = rccl();  // loaded: a state exists only after an RCCL call
    if (c->st) (void)hipStreamSynchronize(c->st);
    for (size_t k = 0; k < g_pending.size();)  // an exchange of a group never ended
        if (g_pending[k].c == c) g_pending.erase(g_pending.begin() + k);
        else ++k;
    if (c->comm && R) (void)R->CommDestroy(c->comm);
    if (c->h_counts) (void)hipHostFree(c->h_counts);
    for (hipEvent_t e : {c->ev, c->ev_in, c->ev_out})
        if (e) (void)hipEventDestroy(e);
    if (c->st) (void)hipStreamDestroy(c->st);
    delete c;
}

extern "C" {

int emurx_comm_unique_id(uint8_t id[EMURX_COMM_ID_BYTES]) {
    static_assert(EMURX_COMM_ID_BYTES == sizeof(ncclUniqueId), "ncclUniqueId size");
    if (!id) return EMURX_EINVAL;
    const Rccl* R = rccl();
    if (!R) return EMURX_ECOMM;
    ncclUniqueId u;
    if (!nccl_ok(R->GetUniqueId(&u), "ncclGetUniqueId")) return EMURX_ECOMM;
    memcpy(id, &u, sizeof(u));
    return EMURX_OK;
}

int emurx_comm_init(emurx_t* h, const uint8_t id[EMURX_COMM_ID_BYTES], uint32_t nranks, uint32_t rank) {
    if (!h || !id || nranks == 0 || nranks > EMURX_MAX_PARTS || rank >= nranks) return EMURX_EINVAL;
    int rc = emurx_handle_bind(h);
    if (rc) return rc;
    const Rccl* R = rccl();
    if (!R) return EMURX_ECOMM;
    emurx_comm_state*& slot = emurx_handle_comm(h);
    if (slot) return EMURX_EEXIST;
    emurx_comm_state* c = nullptr;
    if ((rc = new_state(h, nranks, rank, &c))) return rc;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    if (!nccl_ok(R->CommInitRank(&c->comm, (int)nranks, u, (int)rank), "ncclCommInitRank")) {
        c->comm = nullptr;
        emurx_comm_free(c);
        return EMURX_ECOMM;
    }
    slot = c;
    return EMURX_OK;
}

int emurx_comm_init_all(emurx_t* const* hs, uint32_t n) {
    if (!hs || n == 0 || n > EMURX_MAX_PARTS) return EMURX_EINVAL;
    int dev[EMURX_MAX_PARTS];
    for (uint32_t k = 0; k < n; ++k) {
        if (!hs[k] || emurx_handle_comm(hs[k])) return hs[k] ? EMURX_EEXIST : EMURX_EINVAL;
        dev[k] = emurx_handle_device(hs[k]);
        if (dev[k] < 0) return EMURX_EDEVICE;
        for (uint32_t j = 0; j < k; ++j)
            if (dev[j] == dev[k]) return EMURX_EINVAL;  // one rank per GPU
    }
    const Rccl* R = rccl();
    if (!R) return EMURX_ECOMM;
    ncclComm_t comms[EMURX_MAX_PARTS] = {};
    if (!nccl_ok(R->CommInitAll(comms, (int)n, dev), "ncclCommInitAll")) return EMURX_ECOMM;
    int rc = EMURX_OK;
    emurx_comm_state* st[EMURX_MAX_PARTS] = {};
    for (uint32_t k = 0; k < n && !rc; ++k) {
        if (!(rc = emurx_handle_bind(hs[k]))) rc = new_state(hs[k], n, k, &st[k]);
    }
    if (rc) {
        for (uint32_t k = 0; k < n; ++k) {
            if (st[k]) emurx_comm_free(st[k]);
            else if (comms[k]) (void)R->CommDestroy(comms[k]);
        }
        return rc;
    }
    for (uint32_t k = 0; k < n; ++k) {
        st[k]->comm = comms[k];
        emurx_handle_comm(hs[k]) = st[k];
    }
    return EMURX_OK;
}

int emurx_comm_library(char* path, size_t cap) {
    if (!path || cap == 0) return EMURX_EINVAL;
    const Rccl* R = rccl();
    if (!R) return EMURX_ECOMM;
    snprintf(path, cap, "%s", R->path);
    return strlen(R->path) < cap ? EMURX_OK : EMURX_ENOSPC;
}

int emurx_comm_destroy(emurx_t* h) {
    if (!h) return EMURX_EINVAL;
    emurx_comm_state*& slot = emurx_handle_comm(h);
    if (!slot) return EMURX_ENOENT;
    int rc = emurx_handle_bind(h);
    if (rc) return rc;
    emurx_comm_free(slot);
    slot = nullptr;
    return EMURX_OK;
}

int emurx_comm_info(emurx_t* h, uint32_t* nranks, uint32_t* rank) {
    if (!h) return EMURX_EINVAL;
    emurx_comm_state* c = emurx_handle_comm(h);
    if (!c) return EMURX_ENOENT;
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    return EMURX_OK;
}

int emurx_group_start(void) {
    const Rccl* R = rccl();
    if (!R) return EMURX_ECOMM;
    if (!nccl_ok(R->GroupStart(), "ncclGroupStart")) return EMURX_ECOMM;
    ++g_group_depth;
    return EMURX_OK;
}

int emurx_group_end(void) {
    if (g_group_depth <= 0) return EMURX_EINVAL;
    const Rccl* R = rccl();  // loaded by emurx_group_start
    --g_group_depth;
    const bool ok = nccl_ok(R->GroupEnd(), "ncclGroupEnd");
    if (g_group_depth > 0) return ok ? EMURX_OK : EMURX_ECOMM;
    // the outermost end launched the group's kernels: now join every exchange's caller stream
    int rc = ok ? EMURX_OK : EMURX_ECOMM;
    for (const Pending& p : g_pending) {
        const int r = join_back(p.c, p.user);
        if (!rc) rc = r;
    }
    g_pending.clear();
    return rc;
}

int emurx_exchange_dev(emurx_t* h, const void* d_send, const uint32_t* d_send_count, void* d_recv,
                       uint32_t* d_recv_count, uint32_t cap, uint32_t tail_cap, uint32_t flags, uint64_t* bytes_moved,
                       void* stream) {
    if (!h || !d_send || !d_send_count || !d_recv || !d_recv_count || cap == 0 ||
        (flags & ~(EMURX_XCH_PAYLOAD | EMURX_XCH_ROUTE)) || ((uintptr_t)d_send & 15) || ((uintptr_t)d_recv & 15) ||
        ((uintptr_t)d_send_count & 3) || ((uintptr_t)d_recv_count & 3))
        return EMURX_EINVAL;
    emurx_comm_state* c = emurx_handle_comm(h);
    if (!c) return EMURX_ENOENT;
    const Rccl* R = rccl();  // loaded: the communicator exists
    const bool payload = flags & EMURX_XCH_PAYLOAD, route = flags & EMURX_XCH_ROUTE;
    if (payload && g_group_depth > 0) return EMURX_EINVAL;  // it waits on the host between its phases
    int rc = emurx_handle_bind(h);
    if (rc) return rc;
    hipStream_t user = stream ? (hipStream_t)stream : emurx_handle_stream(h);
    // the communicator's stream continues from the caller's (its packing of d_send)
    if (!EMURX_HIP_OK(hipEventRecord(c->ev_in, user)) || !EMURX_HIP_OK(hipStreamWaitEvent(c->st, c->ev_in, 0)))
        return EMURX_EDEVICE;
    hipStream_t st = c->st;
    // whole regions: the own region's device copy goes on the caller's stream, beside the
    // peers' transfers on the communicator's (the caller's stream waits for those anyway
    // before it reads the receive buffer); payload mode copies its spans on the communicator's
    // stream, behind the counts the host waits for
    hipStream_t self_st = payload ? st : user;
    const uint32_t P = c->nranks, me = c->rank, cs = route ? 1u : 2u;
    const uint64_t rb = route ? sizeof(emurx_route_rec) : sizeof(emurx_lookup_rec);
    const uint64_t heads_end = (uint64_t)cap * rb;
    const uint64_t region = route ? heads_end : EMURX_LOOKUP_REGION_BYTES(cap, tail_cap);
    auto sb = [&](uint32_t p) { return (const uint8_t*)d_send + p * region; };
    auto rbp = [&](uint32_t p) { return (uint8_t*)d_recv + p * region; };
    uint64_t moved = 0;
    const auto D2D = hipMemcpyDeviceToDevice;

    // the counts (and, whole-region mode, the regions) in one group
    if (!nccl_ok(R->GroupStart(), "ncclGroupStart")) return EMURX_ECOMM;
    bool ok = true;
    for (uint32_t p = 0; p < P && ok; ++p) {
        const bool self = p == me;
        if (self && !c->self_rccl) {
            ok = EMURX_HIP_OK(hipMemcpyAsync(d_recv_count + p * cs, d_send_count + p * cs, cs * 4, D2D, self_st));
            if (ok && !payload) ok = EMURX_HIP_OK(hipMemcpyAsync(rbp(p), sb(p), region, D2D, self_st));
            continue;
        }
        ok = nccl_ok(R->Send(d_send_count + p * cs, cs, ncclUint32, (int)p, c->comm, st), "ncclSend") &&
             nccl_ok(R->Recv(d_recv_count + p * cs, cs, ncclUint32, (int)p, c->comm, st), "ncclRecv");
        if (ok && !payload)
            ok = nccl_ok(R->Send(sb(p), region, ncclUint8, (int)p, c->comm, st), "ncclSend") &&
                 nccl_ok(R->Recv(rbp(p), region, ncclUint8, (int)p, c->comm, st), "ncclRecv");
        if (!self) moved += cs * 4 + (payload ? 0 : region);
    }
    const bool ended = nccl_ok(R->GroupEnd(), "ncclGroupEnd");
    if (!ok || !ended) return EMURX_ECOMM;
    if (payload) {
        // the counts to the host (this waits for the caller's stream: the batch's packing), then
        // the spans that carry data
        uint32_t* hc = c->h_counts;
        if (!EMURX_HIP_OK(hipMemcpyAsync(hc, d_send_count, P * cs * 4, hipMemcpyDeviceToHost, st)) ||
            !EMURX_HIP_OK(hipMemcpyAsync(hc + 2 * EMURX_MAX_PARTS, d_recv_count, P * cs * 4, hipMemcpyDeviceToHost, st)) ||
            !EMURX_HIP_OK(hipEventRecord(c->ev, st)) || !EMURX_HIP_OK(hipEventSynchronize(c->ev)))
            return EMURX_EDEVICE;
        const uint32_t* sc = hc;
        const uint32_t* rcn = hc + 2 * EMURX_MAX_PARTS;
        if (!nccl_ok(R->GroupStart(), "ncclGroupStart")) return EMURX_ECOMM;
        for (uint32_t p = 0; p < P && ok; ++p) {
            uint64_t a[2], b[2];
            const int ks = spans(sc[p * cs], cap, rb, heads_end, region, a, b);
            if (p == me && !c->self_rccl) {
                for (int k = 0; k < ks && ok; ++k) ok = EMURX_HIP_OK(hipMemcpyAsync(rbp(p) + a[k], sb(p) + a[k], b[k] - a[k], D2D, st));
                continue;
            }
            for (int k = 0; k < ks && ok; ++k) {
                ok = nccl_ok(R->Send(sb(p) + a[k], b[k] - a[k], ncclUint8, (int)p, c->comm, st), "ncclSend");
                if (p != me) moved += b[k] - a[k];
            }
            const int kr = spans(rcn[p * cs], cap, rb, heads_end, region, a, b);
            for (int k = 0; k < kr && ok; ++k)
                ok = nccl_ok(R->Recv(rbp(p) + a[k], b[k] - a[k], ncclUint8, (int)p, c->comm, st), "ncclRecv");
        }
        const bool e2 = nccl_ok(R->GroupEnd(), "ncclGroupEnd");
        if (!ok || !e2) return EMURX_ECOMM;
    }
    if (bytes_moved) *bytes_moved = moved;
    if (g_group_depth > 0) {  // launched by the group's end
        g_pending.push_back(Pending{c, user});
        return EMURX_OK;
    }
    return join_back(c, user);
}

}  // extern "C"
