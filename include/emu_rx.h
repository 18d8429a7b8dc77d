/*
 * emu_rx.h — C-ABI of the MI355X receive path (parse + Namespace/Client classify).
 *
 * Drop-in boundary for TRex-EMU's rx hot path.  The entry points replace, one for one,
 * the Go surface listed below (paths relative to the reference tree):
 *
 *   emurx_rx_stream()        VethIFZmq.OnRxStream         src/emu/core/veth_zmq.go:277-320
 *                            + per frame CThreadCtx.HandleRxPacket  src/emu/core/thread_ctx.go:365-375
 *                            + Parser.ParsePacket / parsePacketL4   src/emu/core/parser.go:583-959
 *                            + CThreadCtx.GetNs                     src/emu/core/thread_ctx.go:772-784
 *                            + CNSCtx.CLookupBy{Mac,IPv4,IPv6,IPv6LocalGlobal} src/emu/core/ns_ctx.go:262-329
 *                            (down to, not including, the ParserCb call: plugins stay in Go)
 *   emurx_classify_dev()     the same, device-resident (frames + descriptors already in HBM)
 *   emurx_register()         Parser.Register               src/emu/core/parser.go:528-565
 *   emurx_ns_add/remove()    CThreadCtx.AddNs/RemoveNs      src/emu/core/thread_ctx.go:786-812
 *   emurx_ns_set_plugins()   ns.PluginCtx presence          src/emu/core/plugin_ctx.go:257-265
 *   emurx_client_add/remove  CNSCtx.AddClient/RemoveClient  src/emu/core/ns_ctx.go:332-440
 *   emurx_client_update_*    CNSCtx.UpdateClientIpv4/Ipv6/DIpv6 src/emu/core/ns_ctx.go:442-533
 *   emurx_client_set_ra()    CClient.Ipv6Router prefix      src/emu/core/client_ctx.go:60-66,279-295
 *   emurx_hist_to_counters() ParserStats accumulation       src/emu/core/parser.go:67-119
 *   emurx_comm_* / emurx_exchange_dev   no Go counterpart: the one MapNsT of the single main
 *                            goroutine (thread_ctx.go:139,397-419,772-784) split by Namespace
 *                            owner over the GPUs, joined by an RCCL exchange
 *
 * Conventions: plain C types, no exceptions or aborts cross the ABI; every call returns
 * EMURX_OK (0) or a negative EMURX_E* code (mirrors PARSER_OK/PARSER_ERR, parser.go:41-44).
 * Single caller thread per handle (the Go main goroutine, thread_ctx.go:397-419); every entry
 * point re-binds the handle's device, so goroutine OS-thread migration is harmless.
 */
#ifndef EMU_RX_H
#define EMU_RX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EMURX_ABI_VERSION 6

/* ---- return codes -------------------------------------------------------------------- */
#define EMURX_OK 0
#define EMURX_EINVAL (-22)   /* bad argument */
#define EMURX_ENOMEM (-12)   /* host or device allocation failed / capacity exceeded */
#define EMURX_EEXIST (-17)   /* key already present (AddNs / AddClient duplicate) */
#define EMURX_ENOENT (-2)    /* key not present */
#define EMURX_EDEVICE (-5)   /* HIP runtime error */
#define EMURX_ENOSPC (-28)   /* output buffer too small */

#define EMURX_ID_NONE 0xFFFFFFFFu

/* ---- limits (src/emu/core/mbuf.go:44-56, veth_zmq.go:8-22) ----------------------------- */
#define EMURX_MAX_FRAME 9216u      /* MAX_PACKET_SIZE: MbufPoll.Alloc panics above */
#define EMURX_ZMQ_MAGIC 0xBEEFu    /* ZMQ_PACKET_HEADER_MAGIC */

/* ---- parser callbacks: order of the Parser struct fields, parser.go:509-520 ------------ */
enum emurx_cb {
    EMURX_CB_ARP = 0,
    EMURX_CB_ICMP = 1,
    EMURX_CB_IGMP = 2,
    EMURX_CB_DHCP = 3,
    EMURX_CB_DHCPSRV = 4,
    EMURX_CB_DHCPV6 = 5,
    EMURX_CB_MDNS = 6,
    EMURX_CB_TCP = 7,
    EMURX_CB_UDP = 8,
    EMURX_CB_ICMPV6 = 9,
    EMURX_CB_EAPOL = 10,
    EMURX_CB_PPP = 11,
    EMURX_NUM_CB = 12,
    EMURX_CB_NONE = 0xFF
};
/* output queues: one per callback + one for every frame that reaches no callback */
#define EMURX_Q_DROP 12
#define EMURX_NUM_QUEUES 13

/* ---- plugins whose per-Namespace / per-Client presence gates a callback --------------- */
enum emurx_plugin {
    EMURX_PLUG_ARP = 0,       /* "arp"       */
    EMURX_PLUG_ICMP = 1,      /* "icmp"      */
    EMURX_PLUG_IGMP = 2,      /* "igmp"      */
    EMURX_PLUG_DHCP = 3,      /* "dhcp"      */
    EMURX_PLUG_DHCPSRV = 4,   /* "dhcpsrv"   */
    EMURX_PLUG_DHCPV6 = 5,    /* "dhcpv6"    */
    EMURX_PLUG_MDNS = 6,      /* "mdns"      */
    EMURX_PLUG_TRANSPORT = 7, /* "transport" */
    EMURX_PLUG_IPV6 = 8,      /* "ipv6"      */
    EMURX_PLUG_DOT1X = 9,     /* "dot1x"     */
    EMURX_PLUG_PPP = 10,      /* "ppp"       */
    EMURX_NUM_PLUG = 11
};
#define EMURX_PLUG_ALL ((1u << EMURX_NUM_PLUG) - 1u)

/* ---- per-frame parse outcome (one per distinct return path of ParsePacket) ------------ */
enum emurx_status {
    EMURX_ST_OK = 0,                 /* callback `proto` invoked                             */
    EMURX_ST_NOT_SUPPORTED = 1,      /* callback unregistered -> parserNotSupported, :524     */
    EMURX_ST_PACKET_TOO_SHORT = 2,   /* errPacketIsTooShort        :770                       */
    EMURX_ST_EAPOL_TOO_SHORT = 3,    /* errEAPolTooShort           :781                       */
    EMURX_ST_ARP_TOO_SHORT = 4,      /* errArpTooShort             :792                       */
    EMURX_ST_DOT1Q_TOO_SHORT = 5,    /* errDot1qTooShort           :802                       */
    EMURX_ST_TOO_MANY_DOT1Q = 6,     /* errToManyDot1q             :806                       */
    EMURX_ST_IPV4_TOO_SHORT = 7,     /* errIPv4TooShort            :824,846                   */
    EMURX_ST_IPV4_HDR_TOO_SHORT = 8, /* errIPv4HeaderTooShort      :829,838,842               */
    EMURX_ST_IPV4_FRAGMENT = 9,      /* errIPv4Fragment            :833                       */
    EMURX_ST_IPV4_CS = 10,           /* errIPv4cs                  :854                       */
    EMURX_ST_IPV6_TOO_SHORT = 11,    /* errIPv6TooShort            :866-877,894-926           */
    EMURX_ST_IPV6_HOPLIMIT = 12,     /* errIPv6HopLimitDrop        :879                       */
    EMURX_ST_IPV6_EMPTY = 13,        /* errIPv6Empty               :943                       */
    EMURX_ST_IPV6_JUMBO = 14,        /* errIPv6OptJumbo            :938                       */
    EMURX_ST_IPV6_FRAGMENT = 15,     /* errIPv6Fragment            :934                       */
    EMURX_ST_ICMPV4_TOO_SHORT = 16,  /* errIcmpv4TooShort (ICMP and IGMP) :592,607            */
    EMURX_ST_ICMPV4_CS = 17,         /* errIcmpv4Cse               :597                       */
    EMURX_ST_TCP_TOO_SHORT = 18,     /* errTcpTooShort             :615,621                   */
    EMURX_ST_TCP_CS = 19,            /* tcpCsErr                   :628                       */
    EMURX_ST_UDP_TOO_SHORT = 20,     /* errUdpTooShort             :637                       */
    EMURX_ST_UDP_CS = 21,            /* udpCsErr                   :644                       */
    EMURX_ST_ICMPV6_TOO_SHORT = 22,  /* errIcmpv6TooShort          :685                       */
    EMURX_ST_ICMPV6_CS = 23,         /* errIcmpv6Cse               :689                       */
    EMURX_ST_ICMPV6_UNSUPPORTED = 24,/* errIcmpv6Unsupported       :715                       */
    EMURX_ST_L4_UNSUPPORTED = 25,    /* errL4ProtoUnsupported      :720                       */
    EMURX_ST_L3_UNSUPPORTED = 26,    /* errL3ProtoUnsupported      :954                       */
    /* inputs on which the reference Go code panics: defined here, no counters */
    EMURX_ST_PANIC_L4LEN = 27,       /* IPv4 totlen < IHL, span slice p[L4:L4+l4len] :597,628,644,689 */
    EMURX_ST_PANIC_IPV6_OPT = 28,    /* processIpv6Options reads p[i+1] past the header :738  */
    EMURX_ST_PANIC_NIL_EAPOL = 29,   /* EAPOL with dot1x unregistered: nil ParserCb :789       */
    EMURX_ST_PANIC_MBUF = 30,        /* ZMQ frame > 9216 B: MbufPoll.Alloc panics, mbuf.go:106 */
    EMURX_NUM_STATUS = 31
};
/* status of the record written for an empty descriptor slot (EMURX_DESC_HOLE): no frame, no
   Namespace (ns_id = client_id = EMURX_ID_NONE), proto EMURX_CB_NONE, not counted */
#define EMURX_ST_HOLE 0xFFu

/* ---- lookup outcome of the callback's Namespace/Client rule (record.flags bits 4..6) -- */
enum emurx_lookup {
    EMURX_LK_NONE = 0,             /* not attempted: no callback is invoked for the frame */
    EMURX_LK_NO_NS = 1,            /* GetNs(ps.Tun) == nil                                */
    EMURX_LK_NS_NO_PLUGIN = 2,     /* ns.PluginCtx.Get(<plugin>) == nil                   */
    EMURX_LK_NS_LEVEL = 3,         /* namespace-level dispatch, no client key (igmp, mdns,
                                      ipv6 non-echo, arp reply)                           */
    EMURX_LK_NO_CLIENT = 4,        /* the rule's key resolved no (acceptable) client     */
    EMURX_LK_CLIENT_NO_PLUGIN = 5, /* client found, client.PluginCtx.Get(<plugin>) == nil */
    EMURX_LK_CLIENT = 6            /* client_id is valid                                  */
};
#define EMURX_FLAG_RTALERT 0x01u   /* IPV6_M_RTALERT_ML, parser.go:48 */
#define EMURX_FLAG_LK_SHIFT 4
#define EMURX_FLAG_LK_MASK 0x70u

/* ---- wire/device data structures ------------------------------------------------------ */
/* frame descriptor: byte offset of the frame in the batch buffer, its length and vport.
   (The ZMQ per-frame header 0xAA|vport|len, veth_zmq.go:296-305, carries the same fields.) */
typedef struct emurx_desc {
    uint32_t off;
    uint16_t len;
    uint8_t vport;
    uint8_t pad;   /* 0, EMURX_DESC_HOLE, or the frame's owner key (EMURX_DESC_KEYED) */
} emurx_desc;
/* pad value of an empty descriptor slot: no frame, no record, no queue entry, not counted
   (the batched ingest leaves one for every frame a message announced but did not carry) */
#define EMURX_DESC_HOLE 0xFFu
/* pad = EMURX_DESC_KEYED | k (k <= 126): the frame's Namespace-owner key, a 7-bit digest of
   the CTunnelKey its parse leaves (vport and the dot1q / QinQ words of its first 22 bytes,
   parser.go:801-818).  The device framing walk of the batched ingest writes it with every
   descriptor (it reads the frame's header there anyway); emurx_desc_keys_dev writes it for
   descriptors built elsewhere; emurx_owner_key gives it for a key.  With keyed descriptors
   emurx_parse_route_dev counts the owners from the descriptors alone instead of re-reading
   every frame's header.  A key that does not match the frame misroutes that frame. */
#define EMURX_DESC_KEYED 0x80u

/* 32-byte record, one per frame, in frame order.  The numeric fields are exactly the
   ParserPacketState the reference hands to a ParserCb (parser.go:51-61) plus the
   CTunnelData that makes ps.Tun (thread_ctx.go:37-40), the callback tag, the outcome and
   the resolved Namespace / Client ids. */
typedef struct emurx_rec {
    uint32_t ns_id;     /* id given at emurx_ns_add, or EMURX_ID_NONE                      */
    uint32_t client_id; /* id given at emurx_client_add, or EMURX_ID_NONE                  */
    uint32_t vlan[2];   /* CTunnelData.Vlans: (TPID<<16)|VID, PCP/DEI cleared, 0 if absent */
    uint16_t vport;     /* CTunnelData.Vport                                               */
    uint16_t l3;        /* ParserPacketState.L3                                            */
    uint16_t l4;        /* ParserPacketState.L4                                            */
    uint16_t l7;        /* ParserPacketState.L7                                            */
    uint16_t l7_len;    /* ParserPacketState.L7Len (uint16 wraparound preserved)           */
    uint8_t next_hdr;   /* ParserPacketState.NextHeader                                    */
    uint8_t proto;      /* enum emurx_cb of the callback reached, EMURX_CB_NONE on errors  */
    uint8_t status;     /* enum emurx_status                                               */
    uint8_t flags;      /* bit0 EMURX_FLAG_RTALERT (ps.Flags); bits 4..6 enum emurx_lookup */
    uint16_t rsv;
} emurx_rec;

/* Outcome histogram: EMURX_HIST_BINS × {pkts, bytes}.  Bin = hist_bin(status, proto).
   Counter deltas are derived from it by emurx_hist_to_counters(). */
#define EMURX_HIST_BINS 64
#define EMURX_HIST_BIN(status, proto) \
    ((status) <= EMURX_ST_NOT_SUPPORTED ? (unsigned)(status) * EMURX_NUM_CB + (unsigned)(proto) \
                                        : 2u * EMURX_NUM_CB + (unsigned)(status) - 2u)

/* ParserStats in declaration order, parser.go:67-119 (all uint64). */
enum emurx_parser_counter {
    EMURX_PC_errInternalHandler = 0, EMURX_PC_errParser, EMURX_PC_errEAPolTooShort,
    EMURX_PC_errArpTooShort, EMURX_PC_errIcmpv4TooShort, EMURX_PC_errIgmpv4TooShort,
    EMURX_PC_errUdpTooShort, EMURX_PC_errTcpTooShort, EMURX_PC_errDot1qTooShort,
    EMURX_PC_errToManyDot1q, EMURX_PC_errIPv4TooShort, EMURX_PC_errIPv4HeaderTooShort,
    EMURX_PC_errIPv4Fragment, EMURX_PC_errIPv4cs, EMURX_PC_errTCP, EMURX_PC_errUDP,
    EMURX_PC_eapolPkts, EMURX_PC_eapolBytes, EMURX_PC_arpPkts, EMURX_PC_arpBytes,
    EMURX_PC_icmpPkts, EMURX_PC_icmpBytes, EMURX_PC_igmpPkts, EMURX_PC_igmpBytes,
    EMURX_PC_dhcpPkts, EMURX_PC_dhcpBytes, EMURX_PC_dhcpSrvPkts, EMURX_PC_dhcpSrvBytes,
    EMURX_PC_mDnsPkts, EMURX_PC_mDnsBytes, EMURX_PC_tcpPkts, EMURX_PC_tcpBytes,
    EMURX_PC_udpPkts, EMURX_PC_udpBytes, EMURX_PC_udpCsErr, EMURX_PC_tcpCsErr,
    EMURX_PC_errIPv6TooShort, EMURX_PC_errIPv6HopLimitDrop, EMURX_PC_errIPv6Empty,
    EMURX_PC_errIPv6OptJumbo, EMURX_PC_errIPv6Fragment, EMURX_PC_errIcmpv6TooShort,
    EMURX_PC_errIcmpv6Cse, EMURX_PC_errIcmpv4Cse, EMURX_PC_errIcmpv6Unsupported,
    EMURX_PC_Icmpv6Pkt, EMURX_PC_Icmpv6Bytes, EMURX_PC_errL4ProtoUnsupported,
    EMURX_PC_errL3ProtoUnsupported, EMURX_PC_errPacketIsTooShort,
    EMURX_NUM_PARSER_COUNTERS
};

typedef struct emurx_counters {
    uint64_t parser[EMURX_NUM_PARSER_COUNTERS]; /* ParserStats deltas (parse-side errParser
                                                   included; callback returns are added by
                                                   the caller, thread_ctx.go:365-375)      */
    uint64_t rx_pkts;      /* VethStats.RxPkts    veth_zmq.go:233 */
    uint64_t rx_bytes;     /* VethStats.RxBytes   veth_zmq.go:234 */
    uint64_t rx_batch;     /* VethStats.RxBatch   veth_zmq.go:278 */
    uint64_t rx_parse_err; /* VethStats.RxParseErr veth_zmq.go:281-312 */
    uint64_t ref_panic;    /* frames with an EMURX_ST_PANIC_* status (reference would abort) */
} emurx_counters;

typedef struct emurx_cfg {
    int device;            /* HIP device ordinal; < 0: a host-only handle (the table mirror,
                              generations and image queries, no device: data-path calls
                              return EMURX_EDEVICE) */
    uint32_t max_ns;       /* ns ids must be < max_ns */
    uint32_t max_clients;  /* client ids must be < max_clients.  The device tables are sized
                              for max_ns / max_clients and kept sparse so that a lookup
                              almost always ends in its home bucket (one memory trip for a
                              wave of 64 lookups): about 128 B of device memory per Namespace
                              and 1.7 KB per client (MAC, IPv4, IPv6, client info), 1/n_parts
                              of that when partitioned.  The memory is traded for lookup
                              latency: a table that would pass 2 GiB, or whose device
                              allocation fails, is built at half the spread (down to 2 slots
                              per entry: more probe trips) instead of failing;
                              env EMURX_TABLE_SPREAD="ns,mac,ip,ci" (slots per entry, powers of
                              two >= 2; default 8,8,16,16) sets the spreads */
    uint32_t max_frames;   /* frames per batch (device scratch is sized for it) */
    uint32_t max_bytes;    /* bytes per host batch (emurx_rx_stream staging) */
} emurx_cfg;

/* Device-resident outputs of one batch (all pointers are device memory).
   Frames are processed in tiles of EMURX_QUEUE_TILE (frame i is in tile i / TILE).  Each
   callback owns a region of qlist, and each tile a segment of that region: the indices of
   tile t's frames that reach callback q are, in frame order,
       qlist[q*qcap + t*TILE .. q*qcap + t*TILE + tile_cnt[t*16 + q])
   so queue q (EMURX_Q_DROP = no callback) is the concatenation of its segments over t.
   The histogram is kept as EMURX_HIST_SHARDS accumulating copies (fold them with
   emurx_hist_fold).  rec / qlist / tile_cnt may individually be NULL; hist is required. */
#define EMURX_QUEUE_TILE 256
#define EMURX_HIST_SHARDS 64
typedef struct emurx_dev_out {
    emurx_rec* rec;        /* [n] records, frame order                                     */
    uint32_t* qlist;       /* [EMURX_NUM_QUEUES * qcap] frame indices                       */
    uint32_t qcap;         /* per-queue region, >= ceil(n / TILE) * TILE                    */
    uint32_t* tile_cnt;    /* [ceil(n / TILE) * 16] frames per (tile, queue), 13 used of 16  */
    uint64_t* hist;        /* [EMURX_HIST_SHARDS * 2 * EMURX_HIST_BINS], ACCUMULATED         */
    uint32_t* flow;        /* [n] transport flow outcome (EMURX_FLOW_* / flow id), or NULL   */
} emurx_dev_out;

/* Transport flow outcome per frame (emurx_dev_out.flow), the decision
   TransportCtx.handleRxPacket (src/emu/plugins/transport/client_ctx.go:912-969) takes before
   any socket code runs.  Only frames that reach a client's transport handler get one of these
   (tcp / udp callback, lookup EMURX_LK_CLIENT); the key is the reference's c5tuplekey
   (client_ctx.go:44-112): src, dst, src port, dst port, protocol (IPv4: the header's protocol
   field; IPv6: ParserPacketState.NextHeader). */
#define EMURX_FLOW_NONE 0xFFFFFFFFu      /* the transport handler is not reached              */
#define EMURX_FLOW_NO_CTX 0xFFFFFFF0u    /* client without a TransportCtx: handler returns -1
                                            (PluginTransClient.handleRxTransPacket :73-80)     */
#define EMURX_FLOW_NO_SYN 0xFFFFFFF1u    /* new TCP flow without a bare SYN (ft_new_tcp_no_syn) :840-844 */
#define EMURX_FLOW_NO_SERVER 0xFFFFFFF2u /* new flow, no listener on the port (ft_new_no_cb) :848-853,884-887 */
#define EMURX_FLOW_NEW 0xFFFFFFF3u       /* new flow with a listener: OnAccept runs in Go :855-868,890-903 */
#define EMURX_FLOW_UNKNOWN 0xFFFFFFF4u   /* emurx_lookup_dev only: the handler is reached but the head came
                                            without its c5tuplekey (the source's handle saw no TransportCtx,
                                            or the tuple did not fit its tail shard): the caller decides */
#define EMURX_FLOW_ID_MAX 0xFFFFFFEFu    /* flow ids are 0 .. EMURX_FLOW_ID_MAX                */

typedef struct emurx_ctx emurx_t;

/* ---- lifecycle --------------------------------------------------------------------- */
int emurx_abi_version(void);
int emurx_open(const emurx_cfg* cfg, emurx_t** out);
void emurx_close(emurx_t* h);
const char* emurx_strerror(int code);

/* ---- parser registration (Parser.Register / Init, parser.go:528-581) ------------------ */
int emurx_register(emurx_t* h, const char* protocol);     /* "arp","icmp",...,"transport" */
int emurx_set_callbacks_mask(emurx_t* h, uint32_t mask);  /* bit i = enum emurx_cb i live */
uint32_t emurx_get_callbacks_mask(const emurx_t* h);

/* ---- table sync (control plane runs on the same goroutine as rx) ---------- */
/* key = CTunnelKey bytes (thread_ctx.go:58,92-97): [0:2] vport LE, [2:4] 0, [4:8] Vlans[0] LE,
   [8:12] Vlans[1] LE. */
int emurx_ns_add(emurx_t* h, const uint8_t key[12], uint32_t ns_id, uint32_t plugin_mask);
int emurx_ns_remove(emurx_t* h, const uint8_t key[12]);
int emurx_ns_set_plugins(emurx_t* h, uint32_t ns_id, uint32_t plugin_mask);
/* ipv4 / ipv6 / dhcpv6 may be NULL or all-zero (= absent, as Ipv4Key.IsZero etc.). */
int emurx_client_add(emurx_t* h, uint32_t ns_id, uint32_t client_id, const uint8_t mac[6],
                     const uint8_t ipv4[4], const uint8_t ipv6[16], const uint8_t dhcpv6[16],
                     uint32_t plugin_mask);
/* ctx_client_add (ApiClientAddHandler rpc_base_cmds.go:350-406): a list of clients, each
   through CNSCtx.AddClient in order; stops at the first error and returns it, *n_added =
   clients added before it.  Zero address fields mean absent. */
typedef struct emurx_client_spec {
    uint32_t ns_id, client_id, plugin_mask;
    uint8_t mac[6], ipv4[4], ipv6[16], dhcpv6[16];
    uint8_t pad[2];
} emurx_client_spec; /* 56 bytes */
int emurx_clients_add(emurx_t* h, const emurx_client_spec* clients, uint32_t n, uint32_t* n_added);
int emurx_client_remove(emurx_t* h, uint32_t ns_id, const uint8_t mac[6]);
int emurx_client_set_plugins(emurx_t* h, uint32_t client_id, uint32_t plugin_mask);
int emurx_client_update_ipv4(emurx_t* h, uint32_t client_id, const uint8_t ipv4[4]);
int emurx_client_update_ipv6(emurx_t* h, uint32_t client_id, const uint8_t ipv6[16]);
int emurx_client_update_dipv6(emurx_t* h, uint32_t client_id, const uint8_t dhcpv6[16]);
int emurx_client_set_ra(emurx_t* h, uint32_t client_id, const uint8_t prefix[16],
                        uint8_t prefix_len);
/* Transport flow tables.  A flow key is the reference's tuple bytes: 13 for IPv4
   (c5tuplekeyv4: src[4] dst[4] sport BE dport BE proto), 37 for IPv6 (c5tuplekeyv6: src[16]
   dst[16] sport dport next header), as buildTuplev4/v6 (client_ctx.go:89-112) builds it from a
   received frame.  flow_add / flow_remove mirror TransportCtx.addFlowv4/6 / removeFlowv4/6
   (client_ctx.go:597-651); server_add / server_remove the listener map serverCb
   (lookupServerPort :1142-1155, proto 6 or 17).  Adding either marks the client as having a
   TransportCtx (created on first use, socketApi.go:174-193); client_set_transport sets or
   clears that mark directly.  Removing a client drops its flows and listeners. */
int emurx_flow_add(emurx_t* h, uint32_t client_id, const uint8_t* tuple, uint32_t tuple_len, uint32_t flow_id);
int emurx_flow_remove(emurx_t* h, uint32_t client_id, const uint8_t* tuple, uint32_t tuple_len);
int emurx_server_add(emurx_t* h, uint32_t client_id, uint16_t port, uint8_t proto);
int emurx_server_remove(emurx_t* h, uint32_t client_id, uint16_t port, uint8_t proto);
int emurx_client_set_transport(emurx_t* h, uint32_t client_id, int has_ctx);
/* Table edits reach the device incrementally: every call above edits the slots of the
   device table image it changes (deleted slots become tombstones) and marks the 64-byte
   blocks it touched.  Before the next launch that reads the tables, the edited blocks are
   copied to the device and scattered by one kernel on that launch's stream, ordered after
   every launch on any stream that read the tables since the previous shipment (stream
   events, no host synchronisation) and before every later reader.  A table that outgrows
   its load factor is rebuilt larger and shipped whole (then the host waits for the device
   once).  Streams given to the library must outlive the handle.
   emurx_sync ships pending edits now, on `stream` (NULL = the handle's stream). */
int emurx_sync(emurx_t* h, void* stream);
/* diagnostics: 64-byte blocks shipped as deltas and whole tables uploaded since emurx_open,
   and the bytes of this handle's device tables (any pointer may be NULL) */
int emurx_table_stats(const emurx_t* h, uint64_t* delta_blocks, uint64_t* whole_tables, uint64_t* image_bytes);

/* Partitioned tables (multi-GPU, one handle per GPU): with n_parts > 1 this handle's device
   tables hold only the Namespaces with emurx_ns_owner(key, n_parts) == part and their
   clients, flows and listeners; the host maps stay complete, so every table call keeps Go's
   semantics and return codes.  Device memory per handle ~ 1/n_parts of the tables.
   Rebuilds and ships every table.  (1, 0) = replicated (the default). */
int emurx_set_partition(emurx_t* h, uint32_t n_parts, uint32_t part);

/* ---- mid-batch table mutations ---------------------------------------
   A batch is classified against the tables as they stand when it is launched (a snapshot);
   the Go loop dispatches its records in frame order, and a callback may mutate the maps
   (DHCP's UpdateClientIpv4 dhcp.go:718, a TCP accept adding a flow) before later frames of
   the same batch are dispatched, which Go would classify against the mutated maps.
   emurx_table_gen() is the generation of the tables (it advances on every mutation); read it
   when launching a batch.  While dispatching, a record whose emurx_recs_stale flag is set
   may differ from what the live maps give (its Namespace was added, removed or mutated --
   any of its clients, addresses, plugins, RA prefix, flows -- after that generation): the
   caller re-probes it in its own maps.  Unflagged records equal the live classification. */
uint64_t emurx_table_gen(const emurx_t* h);
int emurx_recs_stale(const emurx_t* h, const emurx_rec* rec, uint32_t n, uint64_t gen, uint8_t* stale);

/* The device tables' answer for a key, computed on the host image by the kernels' bucket walk
   (tests of the incremental maintenance).  table: 0 ns {vport, vlan0, vlan1} -> ns id,
   1 mac {ns, mac lo, mac hi} -> client, 2 ipv4 {ns, ip} -> client, 3 ipv6 {ns, ip[4]} -> client,
   4 client info {client} -> plugin mask, 5 flow4 {client, src, dst, ports, proto} -> flow,
   6 flow6 {client, src[4], dst[4], ports, nh} -> flow, 7 listener {client, port | proto << 16} -> 1
   (words little-endian as in the tables).  EMURX_ENOENT when absent. */
int emurx_image_lookup(emurx_t* h, uint32_t table, const uint32_t* key, uint32_t* value);
/* Compare the device tables with the host image after a shipment (synchronises the handle's
   stream): *mismatched = 32-bit words that differ. */
int emurx_image_check(emurx_t* h, uint64_t* mismatched);

/* ---- data path ---------------------------------------------------------------------- */
/* Host batch, ZMQ wire format (veth_zmq.go:8-22).  Decodes the stream exactly like
   OnRxStream (uint16 running offset, abort-on-header-error), stages it in pinned memory,
   parses + classifies on the GPU and returns records in frame order plus per-queue frame
   index lists.  out_qoff[q]..out_qoff[q+1] indexes out_qlist for queue q
   (out_qoff has EMURX_NUM_QUEUES+1 entries).  *n_out = frames decoded.  `delta` receives
   the ParserStats + VethStats deltas of this batch. */
int emurx_rx_stream(emurx_t* h, const uint8_t* msg, size_t len, emurx_rec* out_rec,
                    uint32_t* out_qlist, uint32_t out_cap, uint32_t* n_out,
                    uint32_t out_qoff[EMURX_NUM_QUEUES + 1], emurx_counters* delta);

/* Device-resident batch: frames (d_frames) and descriptors (d_desc) already in HBM.
   Enqueues parse+classify+compaction on `stream` (hipStream_t, NULL = handle stream) and
   returns without synchronising.  out->hist is accumulated into (zero it to reset).
   n <= cfg.max_frames, out->qcap >= ceil(n / EMURX_QUEUE_TILE) * EMURX_QUEUE_TILE.
   d_frames must be 16-byte aligned and d_desc 8-byte aligned (EMURX_EINVAL otherwise), and
   the frame buffer must stay readable up to the next 64-byte boundary past its last byte
   (frames are staged with 16-byte loads).  One k_rx launch; when table edits are pending
   (emurx_ns_* / emurx_client_* since the last launch) a k_apply launch and cross-stream
   events go ahead of it, and a whole-table or growing shipment synchronises the host with
   the stream (or the device).  Not capturable in a hipGraph: the kernel arguments carry the
   table addresses, which a later table growth reallocates; a capturing stream gets
   EMURX_EINVAL before anything is enqueued (the same for emurx_classify_route_dev,
   emurx_parse_route_dev, emurx_lookup_dev and emurx_route_dev, whose scratch may be allocated
   or change streams behind an event).  Call emurx_sync first to take the shipment out of a
   latency-critical call.  No emurx_* call reads or clears the thread's last HIP error
   (hipGetLastError): a launch's status is hipLaunchKernel's return value, so an error a
   caller's earlier HIP call left pending is still pending after the call (the one exception:
   the out-of-memory status of a table allocation the library recovered from, emurx_cfg). */
int emurx_classify_dev(emurx_t* h, const uint8_t* d_frames, const emurx_desc* d_desc,
                       uint32_t n, const emurx_dev_out* out, void* stream);

/* Device-resident, parse only (no table lookups): records with ns_id/client_id NONE and
   lookup EMURX_LK_NONE (ParsePacket alone).  The multi-GPU path uses emurx_parse_route_dev,
   which parses and packs the lookup records for the Namespace owners in the same pass. */
int emurx_parse_dev(emurx_t* h, const uint8_t* d_frames, const emurx_desc* d_desc,
                    uint32_t n, const emurx_dev_out* out, void* stream);

/* Build descriptors for a ZMQ message on the host (the sequential offset walk of
   OnRxStream).  Returns frames decoded in *n_out; *parse_err = 1 when the walk stopped on a
   header error (RxParseErr).  Frames longer than EMURX_MAX_FRAME stop the walk with
   *parse_err = 2 (the reference panics there). */
int emurx_zmq_descriptors(const uint8_t* msg, size_t len, emurx_desc* out, uint32_t cap,
                          uint32_t* n_out, int* parse_err);

/* ---- batched host ingest: many ZMQ messages per GPU round trip -------
   The per-message loop of VethIFZmq.OnRxStream (veth_zmq.go:277-320) over a whole batch of
   messages, with the framing walk on the GPU (one lane per message, same uint16 offset and
   abort-on-header-error rules as emurx_zmq_descriptors), then parse + classify (k_rx), then
   the per-callback queues packed on the GPU.  Several slots let the caller fill one pinned
   staging buffer while the other slots' batches are in flight (a slot's buffers are allocated
   at its first emurx_ingest_buffer: unused slots cost nothing):

       buf = emurx_ingest_buffer(h, s, bytes)    pinned host memory owned by the library
       ... the caller writes ZMQ messages into buf (the receive copy it does anyway) ...
       emurx_ingest_submit(h, s, msgs, nmsg)     H2D + 4 launches + D2H, returns at once
       emurx_ingest_wait(h, s, &res)             results of slot s, valid until its next submit

   Frames are numbered in message order, then wire order (the order the Go loop handles
   them).  res.desc[i].off is the frame's offset in the slot's buffer.  Counters in res.delta
   are those of OnRxStream called once per message (RxBatch = nmsg). */
#define EMURX_INGEST_SLOTS 4
#define EMURX_MSG_OK 0u          /* every announced frame decoded                           */
#define EMURX_MSG_PARSE_ERR 1u   /* RxParseErr: the walk stopped on a header error           */
#define EMURX_MSG_PANIC 2u       /* the reference panics: frame > 9216 B or offset wrap      */
typedef struct emurx_msg {
    uint32_t off; /* message start in the slot buffer (any alignment) */
    uint32_t len; /* message bytes                                    */
} emurx_msg;
typedef struct emurx_ingest_result {
    const emurx_rec* rec;        /* [n_frames] records, frame order                         */
    const emurx_desc* desc;      /* [n_frames] frame offset / length / vport in the buffer  */
    const uint32_t* qlist;       /* [n_frames] frame indices grouped by queue (qoff)        */
    const uint32_t* msg_frames;  /* [n_msgs] frames decoded from each message               */
    const uint8_t* msg_status;   /* [n_msgs] EMURX_MSG_*                                    */
    uint32_t n_frames;
    uint32_t n_msgs;
    uint32_t qoff[EMURX_NUM_QUEUES + 1];
    emurx_counters delta;        /* ParserStats + VethStats deltas of the batch             */
    uint32_t one_launch;         /* 1: the batch ran as one kernel (k_ingest_small, the
                                    small-batch path), 0: the copy + four-launch pipeline     */
    uint32_t degraded;           /* 1: a one-launch batch whose workgroups did not all arrive
                                    within the wait bound (EMURX_INGEST_SPIN_US, default 200 us,
                                    read at emurx_open, plus 0.1 ns per byte of the batch's
                                    messages: at most 1.2 ms; 0 forces it): its queues were
                                    packed by the last workgroup from device scratch.  Same
                                    results.                                                    */
} emurx_ingest_result;
/* Pinned staging buffer of slot s (0 <= s < EMURX_INGEST_SLOTS) with room for `bytes`
   (grown on demand; not while the slot has a batch in flight). */
int emurx_ingest_buffer(emurx_t* h, uint32_t slot, size_t bytes, uint8_t** buf);
/* Enqueue the slot's messages.  EMURX_ENOSPC when the messages could announce more frames
   than cfg.max_frames (split the batch); EMURX_EINVAL for a message outside the buffer or a
   slot still in flight. */
int emurx_ingest_submit(emurx_t* h, uint32_t slot, const emurx_msg* msgs, uint32_t nmsg);
/* Wait for the slot's batch and point `res` at its results (library-owned pinned memory). */
int emurx_ingest_wait(emurx_t* h, uint32_t slot, emurx_ingest_result* res);
/* The framing walk alone on messages already in device memory (the first stage of the
   batched ingest, k_zmq_walk): one lane per message follows OnRxStream's offset chain
   (veth_zmq.go:277-320) and writes the descriptors of its frames, each with its Namespace-owner
   key (EMURX_DESC_KEYED, from the frame's bytes 12..19: what emurx_parse_route_dev's owner
   count reads instead of the frame), and msg_stat[m] = frames | EMURX_MSG_* << 24.  d_ctl:
   emurx_msg[nmsg] then slot_base[nmsg + 1] (message m's descriptor slots are
   [slot_base[m], slot_base[m + 1]); slots a message announced but did not carry become
   EMURX_DESC_HOLE).  The buffer must be readable 32 bytes past every message.  flags:
   EMURX_WALK_NO_KEYS leaves the pad byte 0 (for the measurement of what the keys cost; the
   bench folds the difference into the exchange's rate).  One launch, no host sync. */
#define EMURX_WALK_NO_KEYS 1u
int emurx_zmq_walk_dev(emurx_t* h, const uint8_t* d_buf, const uint32_t* d_ctl, uint32_t nmsg, emurx_desc* d_desc,
                       uint32_t* d_msg_stat, uint32_t flags, void* stream);
/* The slot's HIP stream (hipStream_t, created on first use), so that a caller can order its
   own work with the slot's batches: make the next batch wait for a device-side producer
   (hipStreamWaitEvent before emurx_ingest_submit), or chain a consumer after the D2H. */
int emurx_ingest_stream(emurx_t* h, uint32_t slot, void** stream);

/* ---- tx-side checksum generation -----------------------------------
   What the plugins' tx paths do to a frame before Veth.Send, for a batch of frames in
   device memory, in place.  Per frame, `ops` selects:
     EMURX_TX_IPV4_HDR   IPv4Header(p[l3:l3+IHL*4]).UpdateChecksum()         ip4.go:132-136
                   (the callers' slice is the whole header: 20 B in transport, tcp_output.go:110-112;
                   24 B with IGMP's router-alert option, igmp.go:1179-1186)
   and one L4 kind (ops >> EMURX_TX_L4_SHIFT), the field zeroed first, the span p[l4:len]:
     TCP4 / UDP4   p[l4+16 | l4+6] = PktChecksumTcpUdp(p[l4:], 0, IPv4Header(p[l3:l3+20]))
                   tcpip.go:38-40 + ip4.go:49-58 (callers tcp_output.go:64-70, udp.go:143-150)
     TCP6 / UDP6 / ICMP6   IPv6Header(p[l3:l3+40]).FixL4ChecksumOffset(p[l4:], osize, 16 | 6 | 2)
                   ip6.go:40-56,127-134 (tcp_output.go:71-76, udp.go:151-156, ipv6/nd.go:1111);
                   with EMURX_TX_V6_NH the pseudo header's next header is `nh` instead of
                   o.NextHeader(): PktChecksumTcpUdpV6(p[l4:], 0, ipv6, osize, nh) tcpip.go:34-36
                   (MLD reports behind a hop-by-hop header, ipv6/mld.go:1271)
     ICMP4         ICMPv4Header(p[l4:]).UpdateChecksum()                      icmp4.go:252-256
   A frame whose header or field would lie past `len` (the Go slices panic there) is left
   untouched and gets status EMURX_TX_RANGE. */
#define EMURX_TX_IPV4_HDR 0x01u
#define EMURX_TX_V6_NH 0x02u
#define EMURX_TX_L4_SHIFT 4
enum emurx_tx_l4 {
    EMURX_TX_L4_NONE = 0,
    EMURX_TX_L4_TCP4 = 1,
    EMURX_TX_L4_UDP4 = 2,
    EMURX_TX_L4_TCP6 = 3,
    EMURX_TX_L4_UDP6 = 4,
    EMURX_TX_L4_ICMP6 = 5,
    EMURX_TX_L4_ICMP4 = 6
};
#define EMURX_TX_OK 0u
#define EMURX_TX_RANGE 1u
typedef struct emurx_tx_desc {
    uint32_t off;      /* frame start in the buffer                              */
    uint16_t len;      /* frame length (the L4 span ends here)                   */
    uint16_t l3, l4;   /* header offsets in the frame                            */
    uint16_t osize;    /* IPv6 extension bytes given to FixL4ChecksumOffset      */
    uint8_t ops;       /* EMURX_TX_IPV4_HDR | EMURX_TX_V6_NH | kind << EMURX_TX_L4_SHIFT */
    uint8_t nh;        /* pseudo-header next header with EMURX_TX_V6_NH          */
    uint8_t pad[2];
} emurx_tx_desc;       /* 16 bytes */
/* d_frames: device buffer, rewritten in place; d_status: [n] EMURX_TX_* (may be NULL).
   One launch on `stream`, no host synchronisation. */
int emurx_tx_checksum_dev(emurx_t* h, uint8_t* d_frames, const emurx_tx_desc* d_desc, uint32_t n,
                          uint8_t* d_status, void* stream);

/* ---- tx framing: VethIFZmq.Send / FlushTx (src/emu/core/veth_zmq.go:149-200) ------------
   The n frames desc[i] = {off, len, vport} of d_frames, in order, are packed into ZMQ
   messages exactly as n consecutive Send calls followed by one FlushTx would pack them:
     a frame whose length would bring the open message's frame bytes to
     ZMQ_TX_MAX_BUFFER_SIZE or more first closes it (:186-188); a message closes at
     ZMQ_TX_PKT_BURST_SIZE frames (:198-200);
     message = BE32 EMURX_ZMQ_MAGIC << 16 | frames (:157-159), then per frame
     BE32 0xAA << 24 | vport << 16 | len (:167-169) and the frame's bytes.
   The messages land back to back in d_out.  d_msg_off[m] (u64) is message m's start and
   d_msg_off[n_msgs] the total; capacity n + 1.  d_info = {n_msgs, total bytes}.  Nothing is
   written at or past out_cap; out_cap >= 8 * n + sum(len) always suffices, and d_info
   tells the size needed when it did not.  d_out 16-byte aligned; the frames are read as
   the aligned 16-byte blocks that hold them.  n < EMURX_TX_ZMQ_MAX_FRAMES.  Two launches on
   `stream` (the chain scan, then the write), no host synchronisation; calls on different
   streams of one handle share its scratch, so they must not overlap.  Replaces
   VethIFZmq.FlushTx's per-frame append loop. */
#define EMURX_ZMQ_TX_BURST 64u            /* ZMQ_TX_PKT_BURST_SIZE  veth_zmq.go:36 */
#define EMURX_ZMQ_TX_MAX_BUFFER 32768u    /* ZMQ_TX_MAX_BUFFER_SIZE veth_zmq.go:37 */
#define EMURX_ZMQ_PKT_MAGIC 0xAAu         /* per-frame header tag   veth_zmq.go:167 */
#define EMURX_TX_ZMQ_MAX_FRAMES (1u << 26) /* n must be below it (else EMURX_EINVAL)       */
int emurx_tx_zmq_dev(emurx_t* h, const uint8_t* d_frames, const emurx_desc* d_desc, uint32_t n,
                     uint8_t* d_out, uint64_t out_cap, uint64_t* d_msg_off, uint64_t* d_info, void* stream);

/* ParserStats delta from an outcome histogram (pure host arithmetic). */
void emurx_hist_to_counters(const uint64_t hist[2 * EMURX_HIST_BINS], emurx_counters* out);
/* Sum the EMURX_HIST_SHARDS copies of a device histogram (after a D2H copy). */
void emurx_hist_fold(const uint64_t* shards, uint64_t out[2 * EMURX_HIST_BINS]);

/* Kernel timing with HIP events recorded on the launch stream around every batch.
   emurx_set_timing(h, slots, stride): slots > 0 keeps the last `slots` timed batches (ring),
   0 disables; every `stride`-th batch is timed (0 or 1 = every batch), so that a timed run
   can keep most launches free of event markers.
   emurx_kernel_times(): waits for the most recent timed batch and returns the device time in
   ms of every batch timed since the previous call (oldest first, at most min(cap, slots));
   then resets the ring. */
int emurx_set_timing(emurx_t* h, uint32_t slots, uint32_t stride);
int emurx_kernel_times(emurx_t* h, float* batch_ms, uint32_t cap, uint32_t* n_out);

/* The source tree this library was built from: the first 16 hex digits of the sha1 of its
   sources, headers and Makefile (trex-emu_amd/Makefile SRC_ID).  No ABI replacement: build
   provenance, printed by the Python binding when it loads the library. */
const char* emurx_build_id(void);

/* LDS staging slab (bytes per wave) of the most recent k_rx launch: 7168 or 6144 (0 before
   the first).  Chosen per launch from sampled feedback of earlier launches (a wave whose
   frames span 6-7 KiB fits only the wider slab); EMURX_STAGE=wide|narrow in the environment
   at emurx_open forces one.  Results never depend on it.  No ABI replacement: a tuning
   observable of this implementation. */
uint32_t emurx_last_stage(const emurx_t* h);
/* LDS image (bytes per wave) of the most recent tx framing write (emurx_tx_zmq_dev): 6144,
   4608 or 0 (every tile on the rows-over-lanes path); -1 before the first.  Chosen per call from
   the tile sizes an earlier call's chain kernel saw; EMURX_TXZ=wide|narrow|long at emurx_open
   forces one.  Results never depend on it.  A tuning observable, no ABI replacement. */
int32_t emurx_last_txz(const emurx_t* h);

/* HBM copy ceiling of this GPU for the roofline context (bench.py): a streaming 16-byte copy
   of `bytes` (a multiple of 16, 16-byte aligned device pointers) on `stream`, one launch.
   Not part of the receive path. */
int emurx_copy_ceiling_dev(void* d_dst, const void* d_src, size_t bytes, void* stream);

/* ---- Namespace-partitioned exchange (multi-GPU, one process per GPU) -------------------
   Frames shard by input offset across the GPUs of a node; each Namespace is owned by one
   partition, emurx_ns_owner(key) = a hash of its CTunnelKey (thread_ctx.go:92-97) mapped
   onto [0, n_parts).  After a batch is classified, emurx_route_dev packs every record whose
   Namespace was found (ns_id != EMURX_ID_NONE) into the send region of its owner:
       send[d * cap .. d * cap + send_count[d])   in frame order, as emurx_route_rec
   An equal-split all-to-all (RCCL over xGMI; n_parts regions of `cap` records) then delivers
   each record to the GPU that owns its Namespace, with send_count exchanged alongside so the
   receiver knows how many of each region are valid.  send_count[d] > cap means the region
   overflowed (records past cap were not written): the caller must raise cap and resend.
   Records without a Namespace stay with the receiving GPU (they are in its counters). */
#define EMURX_MAX_PARTS 8
typedef struct emurx_route_rec {
    emurx_rec rec;       /* the classified record                                        */
    uint32_t src_index;  /* frame index in the source GPU's batch                        */
    uint32_t src_rank;   /* source partition                                             */
} emurx_route_rec;       /* 40 bytes */

uint32_t emurx_ns_owner(const uint8_t key[12], uint32_t n_parts);
/* the descriptor owner key of a CTunnelKey (EMURX_DESC_KEYED | k); emurx_ns_owner(key, n) =
   ((k & 0x7f) * n) >> 7 for every n_parts <= EMURX_MAX_PARTS */
uint8_t emurx_owner_key(const uint8_t key[12]);
/* Write the owner key (EMURX_DESC_KEYED) of every frame into d_desc[i].pad, in place (holes
   stay holes): what the device framing walk does, for descriptors built without it.  Reads
   8 bytes of every frame.  One launch, no host synchronisation. */
int emurx_desc_keys_dev(emurx_t* h, const uint8_t* d_frames, emurx_desc* d_desc, uint32_t n, void* stream);
/* d_rec: the batch's records (device), n frames; d_send: [n_parts * cap] (device);
   d_send_count: [n_parts] (device).  Three kernel launches on `stream`, no host sync. */
int emurx_route_dev(emurx_t* h, const emurx_rec* d_rec, uint32_t n, uint32_t n_parts, uint32_t my_rank,
                    uint32_t cap, emurx_route_rec* d_send, uint32_t* d_send_count, void* stream);
/* Classify + route in one call: emurx_classify_dev of the batch (out->rec required) with the
   route's per-owner counts taken inside the k_rx launch, then the group scan and the packing
   of emurx_route_dev into d_send / d_send_count.  Equal to the two calls in sequence.  The
   route scratch is one set per stream (4 sets; a further stream takes a set over behind an
   event), so routes of batches pipelined over several streams run side by side. */
int emurx_classify_route_dev(emurx_t* h, const uint8_t* d_frames, const emurx_desc* d_desc, uint32_t n,
                             const emurx_dev_out* out, uint32_t n_parts, uint32_t my_rank, uint32_t cap,
                             emurx_route_rec* d_send, uint32_t* d_send_count, void* stream);

/* ---- owner-partitioned classification ---------------------------------
   With partitioned tables (emurx_set_partition) the lookups run on the GPU that owns the
   frame's Namespace.  The receiving GPU parses its shard and derives each frame's lookup key
   (emurx_parse_route_dev); every frame travels to the owner of its CTunnelKey as a 32-byte
   emurx_lookup_rec head, plus a tail of 16-byte units for the few classes whose key does not
   fit the head (an equal-split all-to-all of one region per owner, as for emurx_route_rec);
   the owner resolves Namespace, Client and flow against its partition for the frames that
   reached a callback (emurx_lookup_dev) and keeps the records of the others as parsed.  The
   owner's output for a frame equals emurx_classify_dev's record for it on replicated tables,
   bit for bit (the MapNsT / MapClient* maps thread_ctx.go:139, ns_ctx.go:110-112 split by
   owner).

   Region of one owner (EMURX_LOOKUP_REGION_BYTES(cap, tail_cap) bytes, 16-byte aligned):
     [0, 32 cap)                        heads, frame order: head j of the `count` valid ones
     [32 cap, + 16 EMURX_TAIL_SHARDS tail_cap)   tails: EMURX_TAIL_SHARDS shards of tail_cap
                                        16-byte units; a head's `x` names its tail's first unit
   Tails (the head's key kind / tuple bit say which):
     ICMPv6 echo, CLookupByIPv6 / LocalGlobal key (ns_ctx.go:288-329): 1 unit, the IPv6
       destination; the head carries the client-table hash of the key in place of L7 / L7Len
       (both 0 for ICMPv6, parser.go:684-717), so the owner issues the client probe without
       waiting for the tail
     tcp / udp while some client has a TransportCtx (client_ctx.go:46,78, the c5tuplekey):
       1 unit over IPv4 {ports, src, dst, 0}, 3 over IPv6 {ports, src[4], dst[4], 0, 0, 0}
   Every other frame is its head alone: config D's traffic averages 32.8 bytes per frame
   against the 64 of ABI version 4.  Tail units are taken per (wave, owner) by atomics on one
   of EMURX_TAIL_SHARDS cursors (spread so that no address serialises), so the ORDER of the
   tail units in a shard is not deterministic; what each head's tail holds is. */
#define EMURX_TAIL_SHARDS 64u
#define EMURX_TAIL_CURSOR_STRIDE 64u  /* words between two tail cursors: one per 256-byte line */
#define EMURX_LOOKUP_REGION_BYTES(cap, tail_cap) \
    ((uint64_t)(cap) * 32u + (uint64_t)EMURX_TAIL_SHARDS * (uint64_t)(tail_cap) * 16u)
#define EMURX_TAIL_NONE 0xFFFFFFFFu   /* head.x of a record whose tail did not fit its shard */
typedef struct emurx_lookup_rec {
    uint32_t frame;    /* source frame index (the source rank is the region it arrives in)  */
    uint32_t w[6];     /* the parse packed: CTunnelKey VLAN words (14-bit codes), vport, l3,
                          next header, l4, l7, l7_len, proto, status, RTALERT; the key kind,
                          the tuple bit; the destination MAC and TCP flags (emurx_parse.h)  */
    uint32_t x;        /* MAC key bytes 0..3 / IPv4 key, or the first tail unit's index     */
} emurx_lookup_rec;    /* 32 bytes */
/* Parse the batch (records without lookups into out->rec when non-NULL, queues, histogram as
   emurx_parse_dev) and pack the lookup record of every frame (holes excepted) into the region
   of its Namespace's owner: region d of d_send (EMURX_LOOKUP_REGION_BYTES(cap, tail_cap)
   bytes each) gets d_send_count[2 d] heads in frame order.  Three launches: the owner counts
   (from the descriptors' owner keys, EMURX_DESC_KEYED; a frame without one has its L2 header
   read, 8 bytes), their group scan (which also clears the tail cursors), and k_rx writing
   each head at its final place and each tail at the units its wave took.  Reads no table.
   d_send_count: [2 n_parts]; d_send_count[2 d] is the true head count (> cap: heads past cap
   were dropped); d_send_count[2 d + 1] is 0, or, when a tail did not fit its shard, the units
   the fullest shard of region d needed (> tail_cap; that head's x is EMURX_TAIL_NONE).  The
   caller must check both of every batch (after the count exchange, on every rank) and, on
   overflow, grow cap / tail_cap and route the batch again; the library raises no error of its
   own on the device path. */
int emurx_parse_route_dev(emurx_t* h, const uint8_t* d_frames, const emurx_desc* d_desc, uint32_t n,
                          const emurx_dev_out* out, uint32_t n_parts, uint32_t my_rank, uint32_t cap,
                          uint32_t tail_cap, emurx_lookup_rec* d_send, uint32_t* d_send_count, void* stream);
/* The owner's half: d_recv holds n_parts regions (EMURX_LOOKUP_REGION_BYTES(cap, tail_cap)
   bytes each, the all-to-all's receive buffer), d_recv_count[2 s] heads of them valid in region
   s.  Writes d_out[s * cap + j] (the classified record + source index / rank, emurx_route_rec)
   and d_flow (optional, the transport flow decision) for every valid slot.  One launch, no
   host synchronisation.  Counts must not exceed the capacities (the counts the sources
   reported; an overflow is for the sources to resolve first, emurx_parse_route_dev): slots past
   cap are not read, and a tail index past the shards is not read either. */
int emurx_lookup_dev(emurx_t* h, const emurx_lookup_rec* d_recv, const uint32_t* d_recv_count,
                     uint32_t n_parts, uint32_t cap, uint32_t tail_cap, emurx_route_rec* d_out,
                     uint32_t* d_flow, void* stream);

/* ---- the exchange behind the C-ABI: a library-owned communicator (RCCL over xGMI) -------
   The reference is one process whose main goroutine owns every table (MapNsT / GetNs
   thread_ctx.go:139,772-784, MainLoop :397-419).  Sharded over the GPUs of a node, the one new
   step is the exchange of every frame's lookup record to its Namespace owner; these calls run
   it from the caller's thread (cgo) with no Python or torch in between:
     one process per GPU:  rank 0 calls emurx_comm_unique_id and hands the 128 bytes to every
                           rank out of band; each rank calls emurx_comm_init(h, id, nranks, rank)
                           on its handle (ncclCommInitRank: blocks until every rank has joined)
     one process, N GPUs:  emurx_comm_init_all(handles, n) (ncclCommInitAll over the handles'
                           devices, one per GPU), the reference's process model; the exchanges of
                           the N handles are then issued between emurx_group_start and
                           emurx_group_end (whole-region mode only)
   The communicator's nranks is the n_parts of the exchange; handle k of emurx_comm_init_all is
   rank k.  emurx_close destroys it. */
#define EMURX_ECOMM (-71)          /* RCCL error (init, send / receive, group) */
#define EMURX_COMM_ID_BYTES 128    /* ncclUniqueId */
int emurx_comm_unique_id(uint8_t id[EMURX_COMM_ID_BYTES]);
int emurx_comm_init(emurx_t* h, const uint8_t id[EMURX_COMM_ID_BYTES], uint32_t nranks, uint32_t rank);
int emurx_comm_init_all(emurx_t* const* hs, uint32_t n);
int emurx_comm_destroy(emurx_t* h);
/* EMURX_ENOENT when the handle has no communicator */
int emurx_comm_info(emurx_t* h, uint32_t* nranks, uint32_t* rank);
/* The RCCL library the communicators use, bound at the first communicator call (dlopen of
   librccl.so.1: the copy already in the process if any, else the system's); its path into
   `path`.  EMURX_ECOMM when none loads. */
int emurx_comm_library(char* path, size_t cap);
/* A group is per OS thread (RCCL's ncclGroupStart / ncclGroupEnd are): emurx_group_start, the
   group's exchanges and emurx_group_end must run on one thread (from Go: between
   runtime.LockOSThread and runtime.UnlockOSThread).  emurx_group_end returns EMURX_EINVAL on a
   thread with no open group. */
int emurx_group_start(void);
int emurx_group_end(void);
/* One exchange of the regions emurx_parse_route_dev packed (lookup regions of
   EMURX_LOOKUP_REGION_BYTES(cap, tail_cap) bytes, two counts each) or, with EMURX_XCH_ROUTE,
   those emurx_classify_route_dev packed (cap emurx_route_rec, one count each): rank r receives
   region r of every source s into region s of d_recv, and its counts into d_recv_count, the
   layout emurx_lookup_dev reads.  Enqueued on `stream` (NULL = the handle's stream):
     EMURX_XCH_EQUAL    whole regions and counts in one group (ncclSend / ncclRecv to every
                        peer, the own region by a device copy); no host synchronisation
     EMURX_XCH_PAYLOAD  the counts first, then the host waits for them (the stream up to the
                        batch's packing) and only the spans that carry data travel: the first
                        min(count, cap) records and the tail shards (not inside a group)
   *bytes_moved (optional): bytes sent to other ranks by this call.  A count > cap (the sources'
   overflow, emurx_parse_route_dev) is delivered as is, so every rank sees it. */
#define EMURX_XCH_EQUAL 0u
#define EMURX_XCH_PAYLOAD 1u
#define EMURX_XCH_ROUTE 2u
int emurx_exchange_dev(emurx_t* h, const void* d_send, const uint32_t* d_send_count, void* d_recv,
                       uint32_t* d_recv_count, uint32_t cap, uint32_t tail_cap, uint32_t flags,
                       uint64_t* bytes_moved, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* EMU_RX_H */
