// emu_core.cpp — C++ host mirror of the TRex-EMU rx operator surface (see emu_core.h).
#include "emu_core.h"

#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>

namespace emu {

namespace {
uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
void put_le32(uint8_t* p, uint32_t v) {
    p[0] = v & 0xff; p[1] = (v >> 8) & 0xff; p[2] = (v >> 16) & 0xff; p[3] = v >> 24;
}
void check(int rc, const char* what) {
    if (rc != EMURX_OK) throw std::runtime_error(std::string(what) + ": " + emurx_strerror(rc));
}
std::map<std::string, ParserCb>& proto_db() {
    static std::map<std::string, ParserCb> db;
    return db;
}
const char* kCounterNames[EMURX_NUM_PARSER_COUNTERS] = {
    "errInternalHandler", "errParser", "errEAPolTooShort", "errArpTooShort", "errIcmpv4TooShort",
    "errIgmpv4TooShort", "errUdpTooShort", "errTcpTooShort", "errDot1qTooShort", "errToManyDot1q",
    "errIPv4TooShort", "errIPv4HeaderTooShort", "errIPv4Fragment", "errIPv4cs", "errTCP", "errUDP",
    "eapolPkts", "eapolBytes", "arpPkts", "arpBytes", "icmpPkts", "icmpBytes", "igmpPkts",
    "igmpBytes", "dhcpPkts", "dhcpBytes", "dhcpSrvPkts", "dhcpSrvBytes", "mDnsPkts", "mDnsBytes",
    "tcpPkts", "tcpBytes", "udpPkts", "udpBytes", "udpCsErr", "tcpCsErr", "errIPv6TooShort",
    "errIPv6HopLimitDrop", "errIPv6Empty", "errIPv6OptJumbo", "errIPv6Fragment",
    "errIcmpv6TooShort", "errIcmpv6Cse", "errIcmpv4Cse", "errIcmpv6Unsupported", "Icmpv6Pkt",
    "Icmpv6Bytes", "errL4ProtoUnsupported", "errL3ProtoUnsupported", "errPacketIsTooShort"};
}  // namespace

// ---- CTunnelKey thread_ctx.go:92-136 ------------------------------------------------------
void CTunnelKey::Set(const CTunnelData& d) {
    b[0] = d.Vport & 0xff;
    b[1] = d.Vport >> 8;
    b[2] = b[3] = 0;
    put_le32(b + 4, d.Vlans[0]);
    put_le32(b + 8, d.Vlans[1]);
}
void CTunnelKey::Get(CTunnelData& d) const {
    d.Vport = (uint16_t)(b[0] | (b[1] << 8));
    d.Vlans[0] = le32(b + 4);
    d.Vlans[1] = le32(b + 8);
}
bool CTunnelKey::operator==(const CTunnelKey& o) const { return memcmp(b, o.b, 12) == 0; }
std::string CTunnelKey::String() const {
    CTunnelData d;
    Get(d);
    char s[64];
    snprintf(s, sizeof s, "%u-%x-%x", d.Vport, d.Vlans[0], d.Vlans[1]);
    return s;
}

// ---- getProto / parserNotSupported parser.go:524-526, 961-991 ----------------------------
void RegisterProto(const std::string& name, ParserCb cb) { proto_db()[name] = std::move(cb); }
int parserNotSupported(ParserPacketState*) { return PARSER_ERR; }

uint64_t ParserStats::get(const std::string& name) const {
    for (int i = 0; i < EMURX_NUM_PARSER_COUNTERS; ++i)
        if (name == kCounterNames[i]) return c[i];
    throw std::out_of_range("ParserStats: no counter " + name);
}

// ---- Parser -----------------------------------------------------------------------------
ParserCb* Parser::callback(uint32_t cb) {
    ParserCb* t[EMURX_NUM_CB] = {&arp, &icmp, &igmp, &dhcp, &dhcpsrv, &dhcpv6, &mdns, &tcp, &udp, &icmpv6, &eapol, &ppp};
    return cb < EMURX_NUM_CB ? t[cb] : nullptr;
}
uint32_t Parser::mask() const {
    const ParserCb* t[EMURX_NUM_CB] = {&arp, &icmp, &igmp, &dhcp, &dhcpsrv, &dhcpv6, &mdns, &tcp, &udp, &icmpv6, &eapol, &ppp};
    uint32_t m = 0;
    for (uint32_t i = 0; i < EMURX_NUM_CB; ++i)
        if (*t[i]) m |= 1u << i;
    return m;
}
void Parser::Init(CThreadCtx* t) {
    tctx = t;
    arp = icmp = igmp = dhcp = dhcpsrv = dhcpv6 = mdns = tcp = udp = icmpv6 = ppp = parserNotSupported;
    eapol = nullptr;  // parser.go:567-581: no default, an EAPOL frame then panics in Go
}
void Parser::Register(const std::string& protocol) {
    auto get = [&](const char* name) {
        auto it = proto_db().find(name);
        return it == proto_db().end() ? ParserCb(parserNotSupported) : it->second;
    };
    if (protocol == "arp") arp = get("arp");
    else if (protocol == "icmp") icmp = get("icmp");
    else if (protocol == "igmp") igmp = get("igmp");
    else if (protocol == "dhcp") dhcp = get("dhcp");
    else if (protocol == "dhcpsrv") dhcpsrv = get("dhcpsrv");
    else if (protocol == "ipv6") icmpv6 = get("ipv6");
    else if (protocol == "dhcpv6") dhcpv6 = get("dhcpv6");
    else if (protocol == "dot1x") eapol = get("dot1x");
    else if (protocol == "mdns") mdns = get("mdns");
    else if (protocol == "transport") { tcp = get("transport"); udp = get("transport"); }
    else if (protocol == "ppp") ppp = get("ppp");
}

int Parser::dispatch(const emurx_rec& r, Mbuf* m, CTunnelKey* tun) {
    CTunnelData d;
    d.Vport = r.vport;
    d.Vlans[0] = r.vlan[0];
    d.Vlans[1] = r.vlan[1];
    tun->Set(d);
    ParserPacketState ps;
    ps.Tctx = tctx;
    ps.Tun = tun;
    ps.M = m;
    ps.L3 = r.l3;
    ps.L4 = r.l4;
    ps.L7 = r.l7;
    ps.L7Len = r.l7_len;
    ps.Flags = r.flags & IPV6_M_RTALERT_ML;
    ps.NextHeader = r.next_hdr;
    ps.NsId = r.ns_id;
    ps.ClientId = r.client_id;
    ps.Lookup = (r.flags & EMURX_FLAG_LK_MASK) >> EMURX_FLAG_LK_SHIFT;
    ParserCb* cb = callback(r.proto);
    if (!cb || !*cb) throw std::runtime_error("emu: nil ParserCb");  // Go: nil func call
    return (*cb)(&ps);
}

int Parser::ParsePacket(Mbuf* m) {
    if (!tctx) throw std::runtime_error("Parser.tctx not set");
    std::vector<uint8_t> frame(m->GetData(), m->GetData() + m->PktLen());
    std::vector<uint8_t> msg = ZmqPack({frame}, {m->VPort()});
    emurx_t* h = tctx->rx();
    check(emurx_set_callbacks_mask(h, mask()), "set_callbacks_mask");
    emurx_rec rec{};
    uint32_t q[1], n = 0, qoff[EMURX_NUM_QUEUES + 1];
    emurx_counters d{};
    check(emurx_rx_stream(h, msg.data(), msg.size(), &rec, q, 1, &n, qoff, &d), "rx_stream");
    if (n != 1) throw std::runtime_error("ParsePacket: frame not decoded");
    for (int i = 0; i < EMURX_NUM_PARSER_COUNTERS; ++i)
        if (i != EMURX_PC_errParser) stats[i] += d.parser[i];  // errParser is HandleRxPacket's
    if (rec.status >= EMURX_ST_PANIC_L4LEN) throw std::runtime_error("emu: the Go parser panics on this frame");
    if (rec.status != EMURX_ST_OK) return PARSER_ERR;
    CTunnelKey tun;
    return dispatch(rec, m, &tun);
}

// ---- VethIFZmq::OnRxStream veth_zmq.go:277-320 -------------------------------------------
void VethIFZmq::OnRxStream(const uint8_t* stream, size_t len) {
    emurx_t* h = tctx->rx();
    Parser& p = tctx->parser;
    check(emurx_set_callbacks_mask(h, p.mask()), "set_callbacks_mask");
    const uint32_t cap = 1u << 16;
    std::vector<emurx_rec> rec(cap);
    std::vector<uint32_t> ql(cap);
    std::vector<emurx_desc> desc(cap);
    uint32_t n = 0, qoff[EMURX_NUM_QUEUES + 1];
    emurx_counters d{};
    check(emurx_rx_stream(h, stream, len, rec.data(), ql.data(), cap, &n, qoff, &d), "rx_stream");
    stats.RxBatch += d.rx_batch;
    stats.RxParseErr += d.rx_parse_err;
    stats.RxPkts += d.rx_pkts;
    stats.RxBytes += d.rx_bytes;
    stats.RefPanic += d.ref_panic;
    for (int i = 0; i < EMURX_NUM_PARSER_COUNTERS; ++i) p.stats[i] += d.parser[i];
    uint32_t nd = 0;
    int perr = 0;
    check(emurx_zmq_descriptors(stream, len, desc.data(), cap, &nd, &perr), "zmq_descriptors");
    CTunnelKey tun;
    for (uint32_t i = 0; i < n; ++i) {  // frame order, as the Go loop
        if (rec[i].status != EMURX_ST_OK) continue;  // counted in d (incl. HandleRxPacket's errParser)
        Mbuf m;
        m.Append(stream + desc[i].off, desc[i].len);
        m.SetVPort(desc[i].vport);
        const int r = p.dispatch(rec[i], &m, &tun);
        if (r < 0) {  // HandleRxPacket thread_ctx.go:367-372
            if (r == PARSER_ERR) p.stats[EMURX_PC_errParser]++;
            else p.stats[EMURX_PC_errInternalHandler]++;
        }
    }
}

// ---- CThreadCtx --------------------------------------------------------------------------
CThreadCtx::CThreadCtx(uint32_t max_ns, uint32_t max_clients, uint32_t max_frames, int device) {
    emurx_cfg cfg{};
    cfg.device = (uint32_t)device;
    cfg.max_ns = max_ns;
    cfg.max_clients = max_clients;
    cfg.max_frames = max_frames;
    check(emurx_open(&cfg, &h_), "emurx_open");
    parser.tctx = this;
    veth.tctx = this;
}
CThreadCtx::~CThreadCtx() { emurx_close(h_); }

int CThreadCtx::AddNs(const CTunnelKey& key, uint32_t plugins) {
    const uint32_t id = next_ns_;
    const int rc = emurx_ns_add(h_, key.b, id, plugins);
    if (rc) return rc;
    ++next_ns_;
    return (int)id;
}
int CThreadCtx::RemoveNs(const CTunnelKey& key) { return emurx_ns_remove(h_, key.b); }
int CThreadCtx::AddClient(uint32_t ns, const uint8_t mac[6], const uint8_t ipv4[4], const uint8_t ipv6[16],
                          uint32_t plugins) {
    const uint32_t id = next_client_;
    const int rc = emurx_client_add(h_, ns, id, mac, ipv4, ipv6, nullptr, plugins);
    if (rc) return rc;
    ++next_client_;
    return (int)id;
}
int CThreadCtx::RemoveClient(uint32_t ns, const uint8_t mac[6]) { return emurx_client_remove(h_, ns, mac); }
void CThreadCtx::HandleRxPacket(Mbuf* m) {
    const int r = parser.ParsePacket(m);
    if (r < 0) {
        if (r == PARSER_ERR) parser.stats[EMURX_PC_errParser]++;
        else parser.stats[EMURX_PC_errInternalHandler]++;
    }
}

std::vector<uint8_t> ZmqPack(const std::vector<std::vector<uint8_t>>& frames, const std::vector<uint16_t>& vports) {
    std::vector<uint8_t> m;
    const uint32_t hdr = (0xBEEFu << 16) | (uint32_t)frames.size();
    auto be32 = [&](uint32_t v) {
        m.push_back(v >> 24); m.push_back((v >> 16) & 0xff); m.push_back((v >> 8) & 0xff); m.push_back(v & 0xff);
    };
    be32(hdr);
    for (size_t i = 0; i < frames.size(); ++i) {
        be32(0xAA000000u | ((uint32_t)(vports[i] & 0xff) << 16) | (uint32_t)frames[i].size());
        m.insert(m.end(), frames[i].begin(), frames[i].end());
    }
    return m;
}

}  // namespace emu
