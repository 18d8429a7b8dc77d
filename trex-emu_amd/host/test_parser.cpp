// test_parser.cpp — the reference's parser tests (src/emu/core/parser_test.go), restated over
// the C++ host mirror (emu_core.h) and therefore over the HIP path behind the C-ABI.
// Frames: tests/golden/kat_frames.bin (rebuilt byte-for-byte from the Go tests by
// tests/golden/make_kat_frames.py).  Needs a GPU; run by tests/test_host_mirror.py.
//
//   test_parser <kat_frames.bin>      exit 0 and "PASS <name>" per test
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "emu_core.h"

using namespace emu;

namespace {

struct Kat {
    uint16_t vport;
    std::vector<uint8_t> data;
};
std::map<std::string, Kat> g_kat;

void load(const char* path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error(std::string("cannot open ") + path);
    auto rd = [&](void* p, size_t n) {
        if (!f.read((char*)p, n)) throw std::runtime_error("short fixture");
    };
    uint32_t count;
    rd(&count, 4);
    for (uint32_t i = 0; i < count; ++i) {
        uint16_t nl;
        rd(&nl, 2);
        std::string name(nl, '\0');
        rd(&name[0], nl);
        Kat k;
        uint32_t len;
        rd(&k.vport, 2);
        rd(&len, 4);
        k.data.resize(len);
        rd(k.data.data(), len);
        g_kat[name] = k;
    }
}

Mbuf frame(const std::string& name) {
    const Kat& k = g_kat.at(name);
    Mbuf m;
    m.Append(k.data);
    m.SetVPort(k.vport);
    return m;
}

struct Fatal : std::runtime_error {
    using std::runtime_error::runtime_error;
};
#define FATALF(...)                                     \
    do {                                                \
        char b_[256];                                   \
        snprintf(b_, sizeof b_, __VA_ARGS__);           \
        throw Fatal(b_);                                \
    } while (0)

// parser_test.go:14-33
int arp = 0;
CTunnelKey lastTun;
uint16_t lastL3, lastL4, lastL7;
uint32_t lastNs, lastClient;
uint8_t lastLookup;
int arpSupported(ParserPacketState* ps) {
    arp++;
    lastL3 = ps->L3;
    lastL4 = ps->L4;
    lastL7 = ps->L7;
    lastTun = *ps->Tun;
    lastNs = ps->NsId;
    lastClient = ps->ClientId;
    lastLookup = ps->Lookup;
    return -1;
}

CTunnelKey tunOf(uint16_t vport, uint32_t v0, uint32_t v1) {
    CTunnelData d;
    d.Vport = vport;
    d.Vlans[0] = v0;
    d.Vlans[1] = v1;
    CTunnelKey k;
    k.Set(d);
    return k;
}

// ---- parser_test.go ---------------------------------------------------------------------
void TestParserDot1Q_PPP() {  // :35-75
    CThreadCtx tctx;
    Parser parser;
    parser.Init(&tctx);
    Mbuf m1 = frame("test_parser_dot1q_ppp");
    if (parser.ParsePacket(&m1) != PARSER_ERR) FATALF("ppp is parserNotSupported after Init");
}

void TestParser_PPP() {  // :77-112
    CThreadCtx tctx;
    Parser parser;
    parser.Init(&tctx);
    Mbuf m1 = frame("test_parser_ppp");
    if (parser.ParsePacket(&m1) != PARSER_ERR) FATALF("ppp is parserNotSupported after Init");
}

void TestParserArp() {  // :114-171
    CThreadCtx tctx;
    Parser parser;
    parser.tctx = &tctx;
    parser.arp = arpSupported;
    Mbuf m1 = frame("test_parser_arp");
    arp = 0;
    parser.ParsePacket(&m1);
    if (arp != 0) FATALF(" arp cb should not be called (three tags)");
    if (parser.stats.get("errToManyDot1q") != 1) FATALF(" errToManyDot1q should be 1 ");
}

void TestParserArp1() {  // :173-234
    CThreadCtx tctx;
    Parser parser;
    parser.tctx = &tctx;
    parser.arp = arpSupported;
    Mbuf m1 = frame("test_parser_arp1");
    arp = 0;
    parser.ParsePacket(&m1);
    if (arp != 1) FATALF(" arp cb should be called ");
    if (lastTun != tunOf(7, 0x81000007, 0x81000fff)) FATALF(" ERROR expected last tun is not right %s", lastTun.String().c_str());
}

void TestParserIcmp() {  // :236-303
    CThreadCtx tctx;
    Parser parser;
    parser.tctx = &tctx;
    parser.icmp = arpSupported;
    Mbuf m1 = frame("test_parser_icmp");
    arp = 0;
    parser.ParsePacket(&m1);
    if (arp != 1) FATALF(" cb should be called ");
    if (lastTun != tunOf(7, 0x81000007, 0x81000fff)) FATALF(" ERROR expected last tun is not right ");
    if (lastL3 != 22 || lastL4 != 42 || lastL7 != 50) FATALF(" ERROR expected [22 42 50] != [%u %u %u] ", lastL3, lastL4, lastL7);
}

void TestParserDhcp1() {  // :305-388
    CThreadCtx tctx;
    Parser parser;
    parser.tctx = &tctx;
    parser.dhcp = arpSupported;
    Mbuf m1 = frame("test_parser_dhcp1");
    arp = 0;
    parser.ParsePacket(&m1);
    if (arp != 1) FATALF(" cb should be called ");
    if (lastTun != tunOf(7, 0x81000007, 0x81000001)) FATALF(" ERROR expected last tun is not right ");
    if (lastL3 != 22 || lastL4 != 42 || lastL7 != 50) FATALF(" ERROR expected [22 42 50] != [%u %u %u] ", lastL3, lastL4, lastL7);
}

void TestParserDhcpInvalidCs() {  // :390-454
    CThreadCtx tctx;
    Parser parser;
    parser.tctx = &tctx;
    parser.dhcp = arpSupported;
    Mbuf m1 = frame("test_parser_dhcp_invalid_cs");
    arp = 0;
    parser.ParsePacket(&m1);
    if (parser.stats.get("errIPv4cs") != 1) FATALF(" ipv4 checksum should be wrong ");
}

void TestParserIpv6Option() {  // :465-491 (the Go test asserts nothing; SURVEY.md §8c: RA flag, L4 66, bad csum)
    CThreadCtx tctx;
    Parser parser;
    parser.tctx = &tctx;
    parser.icmpv6 = arpSupported;
    Mbuf m1 = frame("test_parser_ipv6_option");
    arp = 0;
    parser.ParsePacket(&m1);
    if (arp != 0 || parser.stats.get("errIcmpv6Cse") != 1) FATALF(" icmpv6 checksum of the capture is wrong ");
}

// ---- beyond parser_test.go: the lookups and the batch entry point -----------------------
void TestNsClientLookup() {  // GetNs + CLookupByIPv4 + IsUnicastToMe (icmp.go:396-427)
    CThreadCtx tctx;
    Parser parser;
    parser.tctx = &tctx;
    parser.icmp = arpSupported;
    const int ns = tctx.AddNs(tunOf(7, 0x81000007, 0x81000fff));
    const uint8_t mac[6] = {0, 2, 2, 2, 2, 2}, ip[4] = {48, 0, 0, 1};
    const int cid = tctx.AddClient((uint32_t)ns, mac, ip);
    if (ns < 0 || cid < 0) FATALF(" AddNs / AddClient failed %d %d", ns, cid);
    Mbuf m1 = frame("test_parser_icmp");
    arp = 0;
    parser.ParsePacket(&m1);
    if (arp != 1 || lastNs != (uint32_t)ns || lastClient != (uint32_t)cid || lastLookup != EMURX_LK_CLIENT)
        FATALF(" lookup ns %u client %u lk %u ", lastNs, lastClient, lastLookup);
    // RemoveNs refuses while clients are active (thread_ctx.go:803-805); then GetNs == nil
    if (tctx.RemoveNs(tunOf(7, 0x81000007, 0x81000fff)) != EMURX_EEXIST) FATALF(" RemoveNs with clients ");
    if (tctx.RemoveClient((uint32_t)ns, mac) != EMURX_OK) FATALF(" RemoveClient ");
    parser.ParsePacket(&m1);
    if (lastNs != (uint32_t)ns || lastLookup != EMURX_LK_NO_CLIENT) FATALF(" removed client still found ");
    if (tctx.RemoveNs(tunOf(7, 0x81000007, 0x81000fff)) != EMURX_OK) FATALF(" RemoveNs ");
    parser.ParsePacket(&m1);
    if (lastNs != EMURX_ID_NONE || lastLookup != EMURX_LK_NO_NS) FATALF(" removed ns still found ");
}

void TestOnRxStream() {  // veth_zmq.go:277-320 + HandleRxPacket, callbacks in frame order
    CThreadCtx tctx;
    tctx.parser.Init(&tctx);
    std::vector<std::string> order;
    tctx.parser.icmp = [&](ParserPacketState* ps) { order.push_back("icmp"); return arpSupported(ps); };
    tctx.parser.dhcp = [&](ParserPacketState* ps) { order.push_back("dhcp"); return 0; };
    tctx.parser.arp = [&](ParserPacketState*) { order.push_back("arp"); return -2; };
    const char* names[] = {"test_parser_icmp", "test_parser_arp1", "test_parser_dhcp1", "test_parser_arp",
                           "test_parser_dhcp_invalid_cs", "test_parser_ppp", "test_parser_icmp"};
    std::vector<std::vector<uint8_t>> fr;
    std::vector<uint16_t> vp;
    uint64_t bytes = 0;
    for (const char* n : names) {
        fr.push_back(g_kat.at(n).data);
        vp.push_back(g_kat.at(n).vport);
        bytes += g_kat.at(n).data.size();
    }
    tctx.veth.OnRxStream(ZmqPack(fr, vp));
    const std::vector<std::string> want = {"icmp", "arp", "dhcp", "icmp"};
    if (order != want) FATALF(" callback order ");
    const VethStats& s = tctx.veth.stats;
    if (s.RxBatch != 1 || s.RxPkts != 7 || s.RxBytes != bytes || s.RxParseErr != 0) FATALF(" veth stats ");
    const ParserStats& p = tctx.parser.stats;
    // errParser: 2 icmp callbacks returning -1, the too-many-dot1q and bad-csum frames, the
    // ppp frame (parserNotSupported); errInternalHandler: the arp callback's -2
    if (p.get("errParser") != 5 || p.get("errInternalHandler") != 1) FATALF(" errParser %lu errInternalHandler %lu",
        (unsigned long)p.get("errParser"), (unsigned long)p.get("errInternalHandler"));
    if (p.get("icmpPkts") != 2 || p.get("errToManyDot1q") != 1 || p.get("errIPv4cs") != 1) FATALF(" counters ");
    // a truncated message: RxParseErr, the walk stops (veth_zmq.go:296-312)
    std::vector<uint8_t> bad = ZmqPack(fr, vp);
    bad.resize(bad.size() - 5);
    order.clear();
    tctx.veth.OnRxStream(bad);
    if (tctx.veth.stats.RxParseErr != 1 || order.size() != 3) FATALF(" truncated message ");
}

// RFC 1071 over big-endian byte pairs (layers/tcpip.go:76-94), folded and inverted
uint16_t csum16(const uint8_t* p, size_t n, uint32_t s = 0) {
    for (size_t i = 0; i + 1 < n; i += 2) s += (p[i] << 8) | p[i + 1];
    if (n & 1) s += p[n - 1] << 8;
    while (s > 0xffff) s = (s & 0xffff) + (s >> 16);
    return (uint16_t)~s;
}
// Ethernet + tags 0x8100/1, 0x8100/2 + IPv4 + UDP with valid checksums (the simulation layout)
std::vector<uint8_t> udp4(const uint8_t dst[6], const uint8_t src_ip[4], const uint8_t dst_ip[4], uint16_t sport,
                          uint16_t dport, size_t payload) {
    std::vector<uint8_t> f = {dst[0], dst[1], dst[2], dst[3], dst[4], dst[5], 0, 0, 1, 0, 0, 0x63,
                              0x81, 0, 0, 1, 0x81, 0, 0, 2, 0x08, 0};
    const uint16_t tot = (uint16_t)(20 + 8 + payload);
    const uint8_t ip[20] = {0x45, 0, (uint8_t)(tot >> 8), (uint8_t)tot, 0, 1, 0x40, 0, 64, 17, 0, 0,
                            src_ip[0], src_ip[1], src_ip[2], src_ip[3], dst_ip[0], dst_ip[1], dst_ip[2], dst_ip[3]};
    f.insert(f.end(), ip, ip + 20);
    const uint16_t hc = csum16(&f[22], 20);
    f[22 + 10] = hc >> 8;
    f[22 + 11] = hc & 0xff;
    const uint16_t ul = (uint16_t)(8 + payload);
    const uint8_t udp[8] = {(uint8_t)(sport >> 8), (uint8_t)sport, (uint8_t)(dport >> 8), (uint8_t)dport,
                            (uint8_t)(ul >> 8), (uint8_t)ul, 0, 0};
    f.insert(f.end(), udp, udp + 8);
    for (size_t i = 0; i < payload; ++i) f.push_back((uint8_t)(i * 7 + sport));
    uint32_t ps = 17 + ul;  // pseudo header: src, dst, 0 | proto, udp length
    for (int i = 0; i < 4; i += 2) ps += ((src_ip[i] << 8) | src_ip[i + 1]) + ((dst_ip[i] << 8) | dst_ip[i + 1]);
    uint16_t uc = csum16(&f[42], ul, ps);
    if (uc == 0) uc = 0xffff;
    f[42 + 6] = uc >> 8;
    f[42 + 7] = uc & 0xff;
    return f;
}

// The memo (emu_core.h): a transport handler's GetNs(ps.Tun) + CLookupByMac(dst MAC) per frame
// (plugin_transport.go:83-115) is answered from the frame's pre-resolved record, with the
// map's answer; through the batched binding (OnRxBatch, one GPU round trip for many messages);
// and when a callback removes a later frame's client mid-batch, that frame's record is stale
// and its lookups fall back to the maps.
void TestMemoLookups() {
    CThreadCtx tctx;
    tctx.parser.Init(&tctx);
    CTunnelKey key = tunOf(1, 0x81000001, 0x81000002);
    const int ns = tctx.AddNs(key);
    if (ns < 0) FATALF(" AddNs ");
    const int kClients = 16;
    std::vector<std::array<uint8_t, 6>> macs;
    std::map<uint64_t, int> truth;  // MAC -> client id the maps hold
    for (int c = 0; c < kClients; ++c) {
        std::array<uint8_t, 6> m = {0, 0, 1, 0, 0, (uint8_t)(c + 1)};
        const uint8_t ip[4] = {16, 0, 0, (uint8_t)(c + 1)};
        const int id = tctx.AddClient((uint32_t)ns, m.data(), ip);
        if (id < 0) FATALF(" AddClient ");
        macs.push_back(m);
        truth[m[5]] = id;
    }
    int victim = -1, victim_at = -1;  // the client a callback removes, and at which frame
    int frame_no = 0, bad = 0;
    tctx.parser.udp = [&](ParserPacketState* ps) {
        CThreadCtx* t = ps->Tctx;
        const int n = t->GetNs(*ps->Tun);
        const uint8_t* dst = ps->M->GetData();
        const int c = t->CLookupByMac((uint32_t)n, dst);
        const auto it = truth.find(dst[5]);
        const int want = (dst[0] == 0 && dst[1] == 0 && dst[2] == 1 && it != truth.end()) ? it->second : -1;
        if (n != ns || c != want) bad++;
        if (frame_no++ == victim_at && victim >= 0) {  // plugin code mutating the maps mid-batch
            if (t->RemoveClient((uint32_t)ns, macs[victim].data()) != EMURX_OK) bad++;
            truth.erase(macs[victim][5]);
        }
        return 0;
    };
    // 8 messages of 16 frames: every client, plus an unknown MAC per message
    std::vector<std::vector<uint8_t>> msgs;
    const uint8_t sip[4] = {48, 0, 0, 1};
    int frames = 0;
    for (int m = 0; m < 8; ++m) {
        std::vector<std::vector<uint8_t>> fr;
        std::vector<uint16_t> vp;
        for (int k = 0; k < 16; ++k) {
            const uint8_t unknown[6] = {0, 0, 1, 0, 0, 0xEE};
            const uint8_t* dst = k == 15 ? unknown : macs[(m + k) % kClients].data();
            const uint8_t dip[4] = {16, 0, 0, dst[5]};
            fr.push_back(udp4(dst, sip, dip, (uint16_t)(40000 + m * 16 + k), 5000, 22 + k));
            vp.push_back(1);
            frames++;
        }
        msgs.push_back(ZmqPack(fr, vp));
    }
    tctx.veth.OnRxBatch(msgs);
    const auto& s = tctx.memo_stats;
    if (bad || frame_no != frames) FATALF(" lookups differ from the maps: %d bad, %d frames", bad, frame_no);
    if (s.hits != 2u * frames || s.probes != 0 || s.stale != 0)
        FATALF(" memo hits %lu probes %lu stale %lu", (unsigned long)s.hits, (unsigned long)s.probes,
               (unsigned long)s.stale);
    if (tctx.veth.stats.RxBatch != 8 || tctx.veth.stats.RxPkts != (uint64_t)frames) FATALF(" veth stats ");
    if (tctx.parser.stats.get("udpPkts") != (uint64_t)frames) FATALF(" udpPkts ");
    // the same batch again; the callback of frame 40 removes client 3: later frames of that
    // Namespace are stale (their memo is off), the lookups go to the maps and see the removal
    tctx.memo_stats = {};
    frame_no = 0;
    victim = 3;
    victim_at = 40;
    tctx.veth.OnRxBatch(msgs);
    if (bad) FATALF(" lookups after the mid-batch removal differ from the maps: %d", bad);
    if (s.stale == 0 || s.probes != 2 * s.stale || s.hits != 2u * (frames - s.stale))
        FATALF(" stale %lu probes %lu hits %lu", (unsigned long)s.stale, (unsigned long)s.probes,
               (unsigned long)s.hits);
    // a key the GPU did not resolve for this frame goes to the maps
    tctx.memo_stats = {};
    tctx.parser.udp = [&](ParserPacketState* ps) {
        const uint8_t o5 = ps->M->GetData()[5] == 5 ? 6 : 5;  // never the frame's own destination
        const uint8_t other[6] = {0, 0, 1, 0, 0, o5};
        if (ps->Tctx->CLookupByMac((uint32_t)ns, other) != truth.at(o5)) bad++;
        return 0;
    };
    tctx.veth.OnRxBatch({msgs[0]});
    if (bad || s.probes != 16 || s.hits != 0) FATALF(" other keys: bad %d probes %lu", bad, (unsigned long)s.probes);
    // a callback that edits the maps (dhcp.go:718 updates its own client) and then looks its own
    // frame's key up again: the edit turned the memo off, the answer comes from the maps
    tctx.memo_stats = {};
    tctx.parser.udp = [&](ParserPacketState* ps) {
        CThreadCtx* t = ps->Tctx;
        const uint8_t* dst = ps->M->GetData();
        const int c = t->CLookupByMac((uint32_t)ns, dst);
        if (c >= 0 && dst[5] == macs[5][5]) {
            if (t->RemoveClient((uint32_t)ns, dst) != EMURX_OK) bad++;
            truth.erase(dst[5]);
            if (t->CLookupByMac((uint32_t)ns, dst) != -1) bad++;  // not the pre-edit GPU answer
        }
        return 0;
    };
    tctx.veth.OnRxBatch({msgs[0]});
    if (bad || truth.count(macs[5][5])) FATALF(" a lookup after an edit in its own callback: bad %d", bad);
    // a callback that throws (a Go panic): the memo does not outlive it, so a lookup made after
    // the batch (the frame's Mbuf gone) goes to the maps
    tctx.parser.udp = [&](ParserPacketState*) -> int { throw std::runtime_error("plugin panic"); };
    bool threw = false;
    try {
        tctx.veth.OnRxBatch({msgs[1]});
    } catch (const std::runtime_error&) {
        threw = true;
    }
    tctx.memo_stats = {};
    if (!threw || tctx.GetNs(key) != ns || s.hits != 0 || s.probes != 1)
        FATALF(" memo after a throwing callback: threw %d hits %lu", (int)threw, (unsigned long)s.hits);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s kat_frames.bin\n", argv[0]);
        return 2;
    }
    load(argv[1]);
    const std::vector<std::pair<const char*, std::function<void()>>> tests = {
        {"TestParserDot1Q_PPP", TestParserDot1Q_PPP}, {"TestParser_PPP", TestParser_PPP},
        {"TestParserArp", TestParserArp},             {"TestParserArp1", TestParserArp1},
        {"TestParserIcmp", TestParserIcmp},           {"TestParserDhcp1", TestParserDhcp1},
        {"TestParserDhcpInvalidCs", TestParserDhcpInvalidCs},
        {"TestParserIpv6Option", TestParserIpv6Option}, {"TestNsClientLookup", TestNsClientLookup},
        {"TestOnRxStream", TestOnRxStream}, {"TestMemoLookups", TestMemoLookups}};
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
    printf("%s: %zu tests, %d failed\n", failed ? "FAIL" : "ok", tests.size(), failed);
    return failed ? 1 : 0;
}
