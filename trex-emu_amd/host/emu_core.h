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
#pragma once
#include <array>
#include <cstdint>
#include <functional>
#include <string>
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
    // dispatch one device record (status OK) to its callback
    int dispatch(const emurx_rec& r, Mbuf* m, CTunnelKey* tun);
};

struct VethStats {
    uint64_t RxPkts = 0, RxBytes = 0, RxBatch = 0, RxParseErr = 0, RefPanic = 0;
};

class VethIFZmq {
public:
    CThreadCtx* tctx = nullptr;
    VethStats stats;
    // veth_zmq.go:277-320 + per frame HandleRxPacket, callbacks in frame order
    void OnRxStream(const uint8_t* stream, size_t len);
    void OnRxStream(const std::vector<uint8_t>& s) { OnRxStream(s.data(), s.size()); }
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
    void HandleRxPacket(Mbuf* m);  // thread_ctx.go:365-375
    emurx_t* rx() const { return h_; }

private:
    emurx_t* h_ = nullptr;
    uint32_t next_ns_ = 0, next_client_ = 0;
};

// ZMQ wire framing (veth_zmq.go:8-22, 149-178): header + per frame 0xAA|vport|len
std::vector<uint8_t> ZmqPack(const std::vector<std::vector<uint8_t>>& frames, const std::vector<uint16_t>& vports);

}  // namespace emu
