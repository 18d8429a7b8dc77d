// test_exchange.cpp — the Namespace-owner exchange driven from a compiled caller through the
// C-ABI alone (include/emu_rx.h + the HIP runtime for device buffers), the way the cgo shim of
// INTEGRATION.md drives it: no Python, no torch in the process.  One GPU, so one rank:
//   TestExchangeOneProcess  emurx_comm_init_all over the process's handle (the reference's
//                           one-process model, thread_ctx.go:139,397-419), whole regions between
//                           emurx_group_start / emurx_group_end
//   TestExchangeCommInit    emurx_comm_unique_id + emurx_comm_init (one process per GPU), the
//                           payload-sized transfer
// Each: emurx_parse_route_dev -> emurx_exchange_dev -> emurx_lookup_dev, the owner's records
// compared byte for byte with the oracle's classification of the same frames, written into the
// fixture by tests/test_host_mirror.py (CLookupBy* ns_ctx.go:262-329, GetNs thread_ctx.go:772-784).
//
//   test_exchange <fixture.bin>       exit 0 and "PASS <name>" per test
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/emu_rx.h"

namespace {

struct Fixture {
    uint32_t n = 0, max_ns = 0, max_clients = 0;
    std::vector<uint8_t> buf;
    std::vector<emurx_desc> desc;
    std::vector<std::pair<std::vector<uint8_t>, uint32_t>> ns;  // CTunnelKey bytes, ns id
    std::vector<emurx_client_spec> clients;
    std::vector<emurx_route_rec> want;  // the oracle's records, frame order, source rank 0
} F;

void load(const char* path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error(std::string("cannot open ") + path);
    auto rd = [&](void* p, size_t k) {
        if (!f.read((char*)p, k)) throw std::runtime_error("short fixture");
    };
    uint32_t h[6];
    rd(h, sizeof(h));  // n, buffer bytes, Namespaces, clients, max_ns, max_clients
    F.n = h[0];
    F.max_ns = h[4];
    F.max_clients = h[5];
    F.buf.resize(h[1] + 64);
    rd(F.buf.data(), h[1]);
    F.desc.resize(F.n);
    rd(F.desc.data(), F.n * sizeof(emurx_desc));
    for (uint32_t k = 0; k < h[2]; ++k) {
        std::vector<uint8_t> key(12);
        uint32_t id;
        rd(key.data(), 12);
        rd(&id, 4);
        F.ns.emplace_back(key, id);
    }
    F.clients.resize(h[3]);
    rd(F.clients.data(), h[3] * sizeof(emurx_client_spec));
    F.want.resize(F.n);
    rd(F.want.data(), F.n * sizeof(emurx_route_rec));
}

#define CHECK(x)                                                                                          \
    do {                                                                                                  \
        const int rc_ = (x);                                                                              \
        if (rc_ != EMURX_OK) throw std::runtime_error(std::string(#x) + ": " + emurx_strerror(rc_));   \
    } while (0)
#define HIPCHECK(x)                                                                                       \
    do {                                                                                                  \
        if ((x) != hipSuccess) throw std::runtime_error(std::string(#x) + " failed");                   \
    } while (0)

template <class T>
struct Dev {
    T* p = nullptr;
    explicit Dev(size_t count) { HIPCHECK(hipMalloc((void**)&p, count * sizeof(T) + 64)); }
    ~Dev() { (void)hipFree(p); }
};

emurx_t* open_handle() {
    emurx_cfg cfg{0, F.max_ns, F.max_clients, F.n, 0};
    emurx_t* h = nullptr;
    CHECK(emurx_open(&cfg, &h));
    for (const char* p : {"arp", "icmp", "igmp", "dhcp", "dhcpsrv", "icmpv6", "dhcpv6", "dot1x", "mdns", "ppp",
                          "transport"})
        CHECK(emurx_register(h, p));
    for (auto& e : F.ns) CHECK(emurx_ns_add(h, e.first.data(), e.second, EMURX_PLUG_ALL));
    uint32_t added = 0;
    CHECK(emurx_clients_add(h, F.clients.data(), (uint32_t)F.clients.size(), &added));
    return h;
}

// parse + pack, the exchange (inside a group when `group`), the owner's lookups; the records
// compared with the oracle's
void owner_step(emurx_t* h, uint32_t flags, bool group) {
    const uint32_t n = F.n, cap = n, tcap = n / 16 / EMURX_TAIL_SHARDS + 32;
    const size_t region = EMURX_LOOKUP_REGION_BYTES(cap, tcap);
    const uint32_t qcap = (n + EMURX_QUEUE_TILE - 1) / EMURX_QUEUE_TILE * EMURX_QUEUE_TILE;
    Dev<uint8_t> frames(F.buf.size()), send(region), recv(region);
    Dev<emurx_desc> desc(n);
    Dev<uint32_t> qlist(EMURX_NUM_QUEUES * (size_t)qcap), tile_cnt(qcap / EMURX_QUEUE_TILE * 16), sc(2), rc(2);
    Dev<uint64_t> hist((size_t)EMURX_HIST_SHARDS * 2 * EMURX_HIST_BINS);
    Dev<emurx_route_rec> out(cap);
    HIPCHECK(hipMemcpy(frames.p, F.buf.data(), F.buf.size(), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(desc.p, F.desc.data(), n * sizeof(emurx_desc), hipMemcpyHostToDevice));
    HIPCHECK(hipMemset(hist.p, 0, (size_t)EMURX_HIST_SHARDS * 2 * EMURX_HIST_BINS * 8));
    HIPCHECK(hipMemset(recv.p, 0x5A, region));
    hipStream_t st;
    HIPCHECK(hipStreamCreate(&st));
    const emurx_dev_out o{nullptr, qlist.p, qcap, tile_cnt.p, hist.p, nullptr};
    CHECK(emurx_parse_route_dev(h, frames.p, desc.p, n, &o, 1, 0, cap, tcap, (emurx_lookup_rec*)send.p, sc.p, st));
    uint64_t moved = ~0ull;
    if (group) CHECK(emurx_group_start());
    CHECK(emurx_exchange_dev(h, send.p, sc.p, recv.p, rc.p, cap, tcap, flags, &moved, st));
    if (group) CHECK(emurx_group_end());
    CHECK(emurx_lookup_dev(h, (const emurx_lookup_rec*)recv.p, rc.p, 1, cap, tcap, out.p, nullptr, st));
    HIPCHECK(hipStreamSynchronize(st));
    HIPCHECK(hipStreamDestroy(st));
    uint32_t cnt[2];
    HIPCHECK(hipMemcpy(cnt, rc.p, 8, hipMemcpyDeviceToHost));
    std::vector<emurx_route_rec> got(n);
    HIPCHECK(hipMemcpy(got.data(), out.p, n * sizeof(emurx_route_rec), hipMemcpyDeviceToHost));
    if (cnt[0] != n || cnt[1] != 0) throw std::runtime_error("received counts " + std::to_string(cnt[0]));
    if (moved != 0) throw std::runtime_error("a 1-rank exchange moved bytes to another rank");
    for (uint32_t i = 0; i < n; ++i)
        if (memcmp(&got[i], &F.want[i], sizeof(emurx_route_rec)))
            throw std::runtime_error("record " + std::to_string(i) + " differs from the oracle's");
}

void TestExchangeOneProcess() {
    emurx_t* h = open_handle();
    try {
        emurx_t* hs[1] = {h};
        CHECK(emurx_comm_init_all(hs, 1));
        uint32_t nr = 0, r = 9;
        CHECK(emurx_comm_info(h, &nr, &r));
        if (nr != 1 || r != 0) throw std::runtime_error("comm_info");
        owner_step(h, EMURX_XCH_EQUAL, true);
        owner_step(h, EMURX_XCH_EQUAL, false);
    } catch (...) {
        emurx_close(h);
        throw;
    }
    emurx_close(h);  // destroys the communicator
}

void TestExchangeCommInit() {
    emurx_t* h = open_handle();
    try {
        uint8_t id[EMURX_COMM_ID_BYTES];
        CHECK(emurx_comm_unique_id(id));
        CHECK(emurx_comm_init(h, id, 1, 0));
        if (emurx_comm_init(h, id, 1, 0) != EMURX_EEXIST) throw std::runtime_error("second communicator accepted");
        owner_step(h, EMURX_XCH_PAYLOAD, false);
        CHECK(emurx_comm_destroy(h));
        if (emurx_comm_info(h, nullptr, nullptr) != EMURX_ENOENT) throw std::runtime_error("destroyed comm still there");
    } catch (...) {
        emurx_close(h);
        throw;
    }
    emurx_close(h);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s fixture.bin\n", argv[0]);
        return 2;
    }
    try {
        load(argv[1]);
    } catch (const std::exception& e) {
        fprintf(stderr, "%s\n", e.what());
        return 2;
    }
    char lib[512] = {0};
    const std::vector<std::pair<const char*, std::function<void()>>> tests = {
        {"TestExchangeOneProcess", TestExchangeOneProcess}, {"TestExchangeCommInit", TestExchangeCommInit}};
    int failed = 0;
    for (auto& t : tests) {
        try {
            t.second();
            printf("PASS %s\n", t.first);
        } catch (const std::exception& e) {
            printf("FAIL %s: %s\n", t.first, e.what());
            failed++;
        }
    }
    if (emurx_comm_library(lib, sizeof(lib)) == EMURX_OK) printf("rccl: %s\n", lib);
    printf("%s: %zu tests, %d failed\n", failed ? "FAIL" : "ok", tests.size(), failed);
    return failed ? 1 : 0;
}
