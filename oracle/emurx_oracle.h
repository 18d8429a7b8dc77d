/*
 * emurx_oracle.h — CPU ORACLE (test infrastructure ONLY).
 *
 * A single-threaded plain-C restatement of TRex-EMU's receive path, written to be read
 * line-by-line against the Go reference.  It is the checker for the HIP product path:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * Nothing in trex-emu_amd/ links or calls it.
 *
 * Parity pins: src/emu/core/parser_test.go KAT frames (rebuilt byte-for-byte),
 * gopacket layers/tcpip_test.go checksum KATs, and the 8,703-frame golden capture corpus
 * unit-test/exp JSON captures (see tests/golden/).
 */
#ifndef EMURX_ORACLE_H
#define EMURX_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/emu_rx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc orc_t;

orc_t* orc_new(void);
void orc_free(orc_t* o);

void orc_set_callbacks_mask(orc_t* o, uint32_t mask);
int orc_ns_add(orc_t* o, const uint8_t key[12], uint32_t ns_id, uint32_t plugin_mask);
int orc_ns_remove(orc_t* o, const uint8_t key[12]);
int orc_ns_set_plugins(orc_t* o, uint32_t ns_id, uint32_t plugin_mask);
int orc_client_add(orc_t* o, uint32_t ns_id, uint32_t client_id, const uint8_t mac[6],
                   const uint8_t ipv4[4], const uint8_t ipv6[16], const uint8_t dhcpv6[16],
                   uint32_t plugin_mask);
int orc_clients_add(orc_t* o, const emurx_client_spec* c, uint32_t n, uint32_t* n_added);
int orc_client_remove(orc_t* o, uint32_t ns_id, const uint8_t mac[6]);
int orc_client_set_plugins(orc_t* o, uint32_t client_id, uint32_t plugin_mask);
int orc_client_update_ipv4(orc_t* o, uint32_t client_id, const uint8_t ipv4[4]);
int orc_client_update_ipv6(orc_t* o, uint32_t client_id, const uint8_t ipv6[16]);
int orc_client_update_dipv6(orc_t* o, uint32_t client_id, const uint8_t dhcpv6[16]);
int orc_client_set_ra(orc_t* o, uint32_t client_id, const uint8_t prefix[16], uint8_t plen);

/* tcpipChecksum (layers/tcpip.go:76-94) */
uint16_t orc_checksum(const uint8_t* data, size_t len, uint32_t csum);

/* parse + classify ONE frame (ParsePacket + the callback's ns/client rule) */
void orc_parse_frame(const orc_t* o, const uint8_t* p, uint32_t len, uint16_t vport,
                     emurx_rec* r);

/* parse only (no tables): ns/client NONE, lookup NONE */
void orc_parse_only(uint32_t cb_mask, const uint8_t* p, uint32_t len, uint16_t vport,
                    emurx_rec* r);

/* batch over descriptors: records in frame order, per-queue lists (qoff[14]),
   counters (ParserStats deltas incl. parse-side errParser; rx_* left 0). */
void orc_rx_batch(const orc_t* o, const uint8_t* frames, const emurx_desc* desc, uint32_t n,
                  emurx_rec* rec, uint32_t* qlist, uint32_t qoff[EMURX_NUM_QUEUES + 1],
                  emurx_counters* cnt);

/* OnRxStream (veth_zmq.go:277-320) + HandleRxPacket per frame */
int orc_rx_stream(const orc_t* o, const uint8_t* msg, size_t len, emurx_rec* rec,
                  uint32_t* qlist, uint32_t cap, uint32_t* n_out,
                  uint32_t qoff[EMURX_NUM_QUEUES + 1], emurx_counters* cnt);

/* descriptor walk of OnRxStream only */
int orc_zmq_descriptors(const uint8_t* msg, size_t len, emurx_desc* out, uint32_t cap,
                        uint32_t* n_out, int* parse_err);

/* transport flow tables + the per-frame flow decision (see emu_rx.h emurx_flow_add) */
int orc_flow_add(orc_t* o, uint32_t cid, const uint8_t* tuple, uint32_t tlen, uint32_t flow);
int orc_flow_remove(orc_t* o, uint32_t cid, const uint8_t* tuple, uint32_t tlen);
int orc_server_add(orc_t* o, uint32_t cid, uint16_t port, uint8_t proto);
int orc_server_remove(orc_t* o, uint32_t cid, uint16_t port, uint8_t proto);
int orc_client_set_transport(orc_t* o, uint32_t cid, int has_ctx);
void orc_flows(const orc_t* o, const uint8_t* frames, const emurx_desc* desc, const emurx_rec* rec,
               uint32_t n, uint32_t* flow);

/* tx checksum generation over a batch, in place (see emu_rx.h emurx_tx_checksum_dev) */
uint8_t orc_tx_frame(uint8_t* p, uint32_t len, uint16_t l3, uint16_t l4, uint16_t osize, uint8_t ops, uint8_t nh);
void orc_tx_checksum(uint8_t* frames, const emurx_tx_desc* d, uint32_t n, uint8_t* status);
/* VethIFZmq.Send x n + FlushTx (veth_zmq.go:149-200) into out; returns the total bytes
   (written only below cap); msg_off[0..n_msgs] (capacity n + 1); *n_msgs */
uint64_t orc_tx_zmq(const uint8_t* frames, const emurx_desc* d, uint32_t n, uint8_t* out, uint64_t cap,
                    uint64_t* msg_off, uint64_t* n_msgs);

#ifdef __cplusplus
}
#endif
#endif
