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

int Parser::dispatch(const emurx_rec& r, Mbuf* m, CTunnelKey* tun, bool memo) {
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
    CThreadCtx::Memo& mo = tctx->memo_;
    // the memo lives exactly as long as the callback: off again on return AND when the callback
    // throws (a Go panic), so no later lookup compares against this frame's freed Mbuf
    struct Off {
        CThreadCtx::Memo& m;
        ~Off() { m.on = false; }
    } off{mo};
    mo.on = memo;
    if (!memo) tctx->memo_stats.stale++;
    mo.tun = *tun;
    mo.ns = r.ns_id;
    mo.client = r.client_id;
    mo.lookup = ps.Lookup;
    mo.proto = r.proto;
    mo.frame = m->GetData();
    mo.len = m->PktLen();
    mo.l3 = r.l3;
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
    return dispatch(rec, m, &tun, true);
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
    const uint64_t gen = emurx_table_gen(h);
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
        uint8_t stale = 0;
        if (emurx_table_gen(h) != gen) check(emurx_recs_stale(h, &rec[i], 1, gen, &stale), "recs_stale");
        const int r = p.dispatch(rec[i], &m, &tun, !stale);
        if (r < 0) {  // HandleRxPacket thread_ctx.go:367-372
            if (r == PARSER_ERR) p.stats[EMURX_PC_errParser]++;
            else p.stats[EMURX_PC_errInternalHandler]++;
        }
    }
}

void VethIFZmq::OnRxBatch(const std::vector<std::vector<uint8_t>>& msgs) {
    emurx_t* h = tctx->rx();
    Parser& p = tctx->parser;
    check(emurx_set_callbacks_mask(h, p.mask()), "set_callbacks_mask");
    size_t bytes = 0;
    for (const auto& m : msgs) bytes += m.size();
    uint8_t* buf = nullptr;
    check(emurx_ingest_buffer(h, 0, bytes, &buf), "ingest_buffer");
    std::vector<emurx_msg> mv(msgs.size());
    size_t at = 0;
    for (size_t k = 0; k < msgs.size(); ++k) {  // the receive copy into the pinned slot
        if (!msgs[k].empty()) memcpy(buf + at, msgs[k].data(), msgs[k].size());
        mv[k] = emurx_msg{(uint32_t)at, (uint32_t)msgs[k].size()};
        at += msgs[k].size();
    }
    const uint64_t gen = emurx_table_gen(h);  // the tables this batch is classified against
    check(emurx_ingest_submit(h, 0, mv.data(), (uint32_t)mv.size()), "ingest_submit");
    emurx_ingest_result res;
    check(emurx_ingest_wait(h, 0, &res), "ingest_wait");
    const emurx_counters& d = res.delta;
    stats.RxBatch += d.rx_batch;
    stats.RxParseErr += d.rx_parse_err;
    stats.RxPkts += d.rx_pkts;
    stats.RxBytes += d.rx_bytes;
    stats.RefPanic += d.ref_panic;
    for (int i = 0; i < EMURX_NUM_PARSER_COUNTERS; ++i) p.stats[i] += d.parser[i];
    CTunnelKey tun;
    for (uint32_t i = 0; i < res.n_frames; ++i) {  // message order, then wire order
        const emurx_rec& r = res.rec[i];
        if (r.status != EMURX_ST_OK) continue;
        Mbuf m;
        m.Append(buf + res.desc[i].off, res.desc[i].len);
        m.SetVPort(res.desc[i].vport);
        uint8_t stale = 0;  // a callback of an earlier frame mutated this frame's Namespace
        if (emurx_table_gen(h) != gen) check(emurx_recs_stale(h, &r, 1, gen, &stale), "recs_stale");
        const int rv = p.dispatch(r, &m, &tun, !stale);
        if (rv < 0) {  // HandleRxPacket thread_ctx.go:367-372
            if (rv == PARSER_ERR) p.stats[EMURX_PC_errParser]++;
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

namespace {
std::array<uint8_t, 12> key12(const CTunnelKey& k) {
    std::array<uint8_t, 12> a;
    memcpy(a.data(), k.b, 12);
    return a;
}
uint64_t mac48(const uint8_t* m) {
    uint64_t v = 0;
    for (int i = 0; i < 6; ++i) v |= (uint64_t)m[i] << (8 * i);
    return v;
}
}  // namespace

int CThreadCtx::AddNs(const CTunnelKey& key, uint32_t plugins) {
    memo_.on = false;  // an edit from inside a callback: the frame's GPU answer may be stale
    const uint32_t id = next_ns_;
    const int rc = emurx_ns_add(h_, key.b, id, plugins);
    if (rc) return rc;
    ns_map_[key12(key)] = id;
    ++next_ns_;
    return (int)id;
}
int CThreadCtx::RemoveNs(const CTunnelKey& key) {
    memo_.on = false;  // an edit from inside a callback: the frame's GPU answer may be stale
    const int rc = emurx_ns_remove(h_, key.b);
    if (rc == EMURX_OK) ns_map_.erase(key12(key));
    return rc;
}
int CThreadCtx::AddClient(uint32_t ns, const uint8_t mac[6], const uint8_t ipv4[4], const uint8_t ipv6[16],
                          uint32_t plugins) {
    memo_.on = false;  // an edit from inside a callback: the frame's GPU answer may be stale
    const uint32_t id = next_client_;
    const int rc = emurx_client_add(h_, ns, id, mac, ipv4, ipv6, nullptr, plugins);
    if (rc) return rc;
    mac_map_[{ns, mac48(mac)}] = id;
    const uint32_t ip = ipv4 ? le32(ipv4) : 0;
    if (ip) ip4_map_[{ns, ip}] = id;
    client_keys_[id] = {mac48(mac), ip};
    ++next_client_;
    return (int)id;
}
int CThreadCtx::RemoveClient(uint32_t ns, const uint8_t mac[6]) {
    memo_.on = false;  // an edit from inside a callback: the frame's GPU answer may be stale
    const int rc = emurx_client_remove(h_, ns, mac);
    if (rc != EMURX_OK) return rc;
    auto it = mac_map_.find({ns, mac48(mac)});
    if (it != mac_map_.end()) {
        const auto ck = client_keys_[it->second];
        if (ck.second) ip4_map_.erase({ns, ck.second});
        client_keys_.erase(it->second);
        mac_map_.erase(it);
    }
    return rc;
}
int CThreadCtx::UpdateClientIpv4(uint32_t ns, uint32_t client, const uint8_t ipv4[4]) {
    memo_.on = false;  // an edit from inside a callback: the frame's GPU answer may be stale
    const int rc = emurx_client_update_ipv4(h_, client, ipv4);
    if (rc != EMURX_OK) return rc;
    auto& ck = client_keys_[client];
    if (ck.second) ip4_map_.erase({ns, ck.second});
    ck.second = le32(ipv4);
    if (ck.second) ip4_map_[{ns, ck.second}] = client;
    return rc;
}

// ---- the lookups plugins make, answered from the frame's memo when they can ---------------
int CThreadCtx::GetNs(const CTunnelKey& key) {
    // GetNs(ps.Tun) of the frame being dispatched: the Namespace the GPU found for it
    if (memo_.on && key == memo_.tun && memo_.lookup != EMURX_LK_NONE) {
        memo_stats.hits++;
        return memo_.ns == EMURX_ID_NONE ? -1 : (int)memo_.ns;
    }
    memo_stats.probes++;
    auto it = ns_map_.find(key12(key));
    return it == ns_map_.end() ? -1 : (int)it->second;
}
int CThreadCtx::CLookupByMac(uint32_t ns, const uint8_t mac[6]) {
    // the MAC[dst] rule (transport, dhcpv6, ppp, unicast dhcp / dhcpsrv / eapol): the GPU looked
    // this key up in this Namespace when the outcome is a client, a client without the plugin,
    // or no client
    const Memo& mo = memo_;
    const bool mac_rule = mo.proto == EMURX_CB_TCP || mo.proto == EMURX_CB_UDP || mo.proto == EMURX_CB_DHCPV6 ||
                          mo.proto == EMURX_CB_PPP;
    const bool probed = mo.lookup == EMURX_LK_CLIENT || mo.lookup == EMURX_LK_CLIENT_NO_PLUGIN ||
                        mo.lookup == EMURX_LK_NO_CLIENT;
    if (mo.on && mac_rule && probed && ns == mo.ns && mo.len >= 6 && memcmp(mac, mo.frame, 6) == 0) {
        memo_stats.hits++;
        return mo.client == EMURX_ID_NONE ? -1 : (int)mo.client;
    }
    memo_stats.probes++;
    auto it = mac_map_.find({ns, mac48(mac)});
    return it == mac_map_.end() ? -1 : (int)it->second;
}
int CThreadCtx::CLookupByIPv4(uint32_t ns, const uint8_t ip[4]) {
    // an ARP request's target (arp.go:912-925): the GPU's IPv4 lookup of that address
    const Memo& mo = memo_;
    const bool arp_req = mo.proto == EMURX_CB_ARP && mo.len >= (uint32_t)mo.l3 + 28u && mo.frame[mo.l3 + 6] == 0 &&
                         mo.frame[mo.l3 + 7] == 1;
    const bool probed = mo.lookup == EMURX_LK_CLIENT || mo.lookup == EMURX_LK_CLIENT_NO_PLUGIN ||
                        mo.lookup == EMURX_LK_NO_CLIENT;
    if (mo.on && arp_req && probed && ns == mo.ns && memcmp(ip, mo.frame + mo.l3 + 24, 4) == 0) {
        memo_stats.hits++;
        return mo.client == EMURX_ID_NONE ? -1 : (int)mo.client;
    }
    memo_stats.probes++;
    auto it = ip4_map_.find({ns, le32(ip)});
    return it == ip4_map_.end() ? -1 : (int)it->second;
}
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
