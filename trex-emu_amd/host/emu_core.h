// emu_core.h — C++ host mirror of TRex-EMU's receive-path operator surface over the C-ABI
// (include/emu_rx.h).  The reference's host language (Go) is not available here, so this
// is the drop-in shape a C++ caller (and the host parity tests, host/test_parser.cpp) use:
// the same type and method names as src/emu/core, the same argument meaning and the same
// error behaviour, with the parse / checksum / Namespace / Client work done by the HIP path.
//
//   CTunnelData / CTunnelKey      thread_ctx.go:37-136
//   Mbuf (data + vport only)      mbuf.go
//   ParserPacketState, ParserCb   parser.go:51-61, 503
//   Parser (callback fields, Init, Register, ParsePacket, stats)   parser.go:503-991
//   CThreadCtx (AddNs/RemoveNs/GetNs, AddClient, HandleRxPacket)   thread_ctx.go:139-812
//   VethIFZmq::OnRxStream          veth_zmq.go:277-320
//   GetNs / CLookupByMac / CLookupByIPv4   thread_ctx.go:777-784, ns_ctx.go:262-285
//
// The lookups plugins make keep their Go signatures and answer from the frame being
// dispatched when they ask for the key the GPU resolved (the frame's memo: its tunnel key,
// Namespace, client and lookup outcome), so a plugin's GetNs + CLookupBy* per frame costs no
// map probe; any other key, or a frame whose Namespace a callback of an earlier frame of the
// batch has mutated (emurx_recs_stale), falls back to the host maps.  No plugin code changes.
#pragma once
#include <array>
#include <cstdint>
#include <functional>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/emu_rx.h"

namespace emu {

constexpr int PARSER_OK = 0;
constexpr int PARSER_ERR = -1;
constexpr uint32_t IPV6_M_RTALERT_ML = 0x1;  // parser.go:48

struct CTunnelData {
    uint16_t Vport = 0;
    uint32_t Vlans[2] = {0, 0};
};

// 12-byte Namespace key: [0:2] vport LE, [2:4] 0, [4:8] Vlans[0] LE, [8:12] Vlans[1] LE
struct CTunnelKey {
    uint8_t b[12] = {};
    void Set(const CTunnelData& d);
    void Get(CTunnelData& d) const;
    bool operator==(const CTunnelKey& o) const;
    bool operator!=(const CTunnelKey& o) const { return !(*this == o); }
    std::string String() const;
};

class Mbuf {
public:
    void Append(const uint8_t* p, size_t n) { data_.insert(data_.end(), p, p + n); }
    void Append(const std::vector<uint8_t>& v) { Append(v.data(), v.size()); }
    void SetVPort(uint16_t v) { vport_ = v; }
    uint16_t VPort() const { return vport_; }
    const uint8_t* GetData() const { return data_.data(); }
    uint32_t PktLen() const { return (uint32_t)data_.size(); }

private:
    std::vector<uint8_t> data_;
    uint16_t vport_ = 0;
};

class CThreadCtx;

struct ParserPacketState {
    CThreadCtx* Tctx = nullptr;
    CTunnelKey* Tun = nullptr;
    Mbuf* M = nullptr;
    uint16_t L3 = 0, L4 = 0, L7 = 0, L7Len = 0;
    uint32_t Flags = 0;
    uint8_t NextHeader = 0;
    // resolved on the GPU (what GetNs / the callback's CLookupBy* would return)
    uint32_t NsId = EMURX_ID_NONE, ClientId = EMURX_ID_NONE;
    uint8_t Lookup = EMURX_LK_NONE;  // enum emurx_lookup
};
using ParserCb = std::function<int(ParserPacketState*)>;

// getProto registry (parser.go:961-991): plugins register their rx handler by name
void RegisterProto(const std::string& name, ParserCb cb);
int parserNotSupported(ParserPacketState* ps);

struct ParserStats {
    std::array<uint64_t, EMURX_NUM_PARSER_COUNTERS> c{};
    uint64_t& operator[](int i) { return c[i]; }
    uint64_t get(const std::string& name) const;  // ParserStats field name, parser.go:67-119
};

class Parser {
public:
    CThreadCtx* tctx = nullptr;
    ParserStats stats;
    // parser.go:509-520, in emurx_cb order
    ParserCb arp, icmp, igmp, dhcp, dhcpsrv, dhcpv6, mdns, tcp, udp, icmpv6, eapol, ppp;

    void Init(CThreadCtx* t);                    // parser.go:567-581 (eapol stays unset)
    void Register(const std::string& protocol);  // parser.go:528-565
    // One frame through the device path; returns the callback's value or PARSER_ERR.
    // Adds the ParserStats increments the Go ParsePacket makes (errParser is HandleRxPacket's).
    int ParsePacket(Mbuf* m);

    ParserCb* callback(uint32_t cb);
    uint32_t mask() const;  // callbacks set -> registered mask of the device path
    // dispatch one device record (status OK) to its callback; memo: the record may answer the
    // callback's GetNs / CLookupBy* (it is not stale)
    int dispatch(const emurx_rec& r, Mbuf* m, CTunnelKey* tun, bool memo);
};

struct VethStats {
    uint64_t RxPkts = 0, RxBytes = 0, RxBatch = 0, RxParseErr = 0, RefPanic = 0;
};

class VethIFZmq {
public:
    CThreadCtx* tctx = nullptr;
    VethStats stats;
    // veth_zmq.go:277-320 + per frame HandleRxPacket, callbacks in frame order.  One message
    // per call (emurx_rx_stream): a fallback, slower than the CPU per message
    void OnRxStream(const uint8_t* stream, size_t len);
    void OnRxStream(const std::vector<uint8_t>& s) { OnRxStream(s.data(), s.size()); }
    // The primary binding: the messages MainLoop has queued (thread_ctx.go:409-410), all in one
    // GPU round trip (emurx_ingest_*: pinned staging, framing walk, parse + classify and queue
    // packing on the device), then OnRxStream's per-frame dispatch in message and wire order,
    // each callback seeing its frame's memo.  Same counters as OnRxStream once per message.
    void OnRxBatch(const std::vector<std::vector<uint8_t>>& msgs);
};

class CThreadCtx {
public:
    explicit CThreadCtx(uint32_t max_ns = 4096, uint32_t max_clients = 65536, uint32_t max_frames = 4096,
                        int device = 0);
    ~CThreadCtx();
    CThreadCtx(const CThreadCtx&) = delete;
    CThreadCtx& operator=(const CThreadCtx&) = delete;

    Parser parser;
    VethIFZmq veth;

    // ids are dense and owned here, as the Go side assigns them (thread_ctx.go:786, ns_ctx.go:332)
    int AddNs(const CTunnelKey& key, uint32_t plugins = 0x7FF);  // -> ns id, or EMURX_E*
    int RemoveNs(const CTunnelKey& key);  // EMURX_EEXIST while it has clients (thread_ctx.go:803)
    int AddClient(uint32_t ns, const uint8_t mac[6], const uint8_t ipv4[4] = nullptr,
                  const uint8_t ipv6[16] = nullptr, uint32_t plugins = 0x7FF);  // -> client id
    int RemoveClient(uint32_t ns, const uint8_t mac[6]);  // ns_ctx.go RemoveClient
    int UpdateClientIpv4(uint32_t ns, uint32_t client, const uint8_t ipv4[4]);  // ns_ctx.go:442-471
    void HandleRxPacket(Mbuf* m);  // thread_ctx.go:365-375
    emurx_t* rx() const { return h_; }

    // The lookups plugins make (thread_ctx.go:777-784, ns_ctx.go:262-285): -1 for nil.  While a
    // frame is dispatched they answer from its memo when asked for the key the GPU resolved.
    int GetNs(const CTunnelKey& key);
    int CLookupByMac(uint32_t ns, const uint8_t mac[6]);
    int CLookupByIPv4(uint32_t ns, const uint8_t ip[4]);
    struct MemoStats {
        uint64_t hits = 0;    // answered from the frame's pre-resolved record
        uint64_t probes = 0;  // answered from the host maps
        uint64_t stale = 0;   // frames whose memo was off (mid-batch mutation)
    } memo_stats;

private:
    friend class Parser;
    friend class VethIFZmq;
    struct Memo {
        bool on = false;
        CTunnelKey tun;
        uint32_t ns = EMURX_ID_NONE, client = EMURX_ID_NONE;
        uint8_t lookup = EMURX_LK_NONE, proto = EMURX_CB_NONE;
        const uint8_t* frame = nullptr;
        uint32_t len = 0;
        uint16_t l3 = 0;
    } memo_;
    // the Go maps as the host keeps them (the memo's fallback; the device tables mirror them)
    std::map<std::array<uint8_t, 12>, uint32_t> ns_map_;
    std::map<std::pair<uint32_t, uint64_t>, uint32_t> mac_map_;
    std::map<std::pair<uint32_t, uint32_t>, uint32_t> ip4_map_;
    std::map<uint32_t, std::pair<uint64_t, uint32_t>> client_keys_;  // id -> (mac, ipv4)
    emurx_t* h_ = nullptr;
    uint32_t next_ns_ = 0, next_client_ = 0;
};

// ZMQ wire framing (veth_zmq.go:8-22, 149-178): header + per frame 0xAA|vport|len
std::vector<uint8_t> ZmqPack(const std::vector<std::vector<uint8_t>>& frames, const std::vector<uint16_t>& vports);

}  // namespace emu
