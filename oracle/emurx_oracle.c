/*
 * emurx_oracle.c — CPU ORACLE, TEST INFRASTRUCTURE ONLY (never linked by the product).
 *
 * Plain-C restatement of the TRex-EMU receive path.  Every function cites the Go it
 * follows (paths relative to the reference tree).  Deliberately written as a sequential,
 * byte-by-byte transliteration of the Go control flow — it shares no code with the HIP
 * path it checks.  Integer widths follow Go: offsets are uint16 (wraparound preserved),
 * packet sizes uint32, checksum accumulators uint32.
 */
#include "emurx_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ===================================================================================== */
/* encoding/binary BigEndian                                                              */
/* ===================================================================================== */
static inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* ===================================================================================== */
/* Generic byte-keyed open-addressing map (stands in for the Go runtime maps; only the   */
/* exact-match semantics matter for parity).                                               */
/* ===================================================================================== */
#define KMAX 20
typedef struct {
    uint8_t* keys;   /* cap * ksz */
    uint32_t* vals;  /* cap */
    uint8_t* state;  /* 0 empty, 1 used, 2 deleted */
    uint32_t cap, used, tomb, ksz;
} bmap;

static uint32_t fnv1a(const uint8_t* k, uint32_t n) {
    uint32_t h = 2166136261u;
    for (uint32_t i = 0; i < n; i++) { h ^= k[i]; h *= 16777619u; }
    return h;
}
static void bmap_init(bmap* m, uint32_t ksz) {
    memset(m, 0, sizeof(*m));
    m->ksz = ksz;
}
static void bmap_free(bmap* m) { free(m->keys); free(m->vals); free(m->state); }
static int bmap_find(const bmap* m, const uint8_t* k, uint32_t* v) {
    if (!m->cap) return 0;
    uint32_t i = fnv1a(k, m->ksz) & (m->cap - 1);
    for (uint32_t n = 0; n < m->cap; n++, i = (i + 1) & (m->cap - 1)) {
        if (m->state[i] == 0) return 0;
        if (m->state[i] == 1 && !memcmp(m->keys + (size_t)i * m->ksz, k, m->ksz)) {
            if (v) *v = m->vals[i];
            return 1;
        }
    }
    return 0;
}
static void bmap_put(bmap* m, const uint8_t* k, uint32_t v);
static void bmap_grow(bmap* m) {
    bmap old = *m;
    uint32_t nc = old.cap ? old.cap * 2 : 64;
    while ((old.used + 1) * 2 > nc) nc *= 2;
    m->cap = nc; m->used = 0; m->tomb = 0;
    m->keys = (uint8_t*)calloc((size_t)nc, m->ksz);
    m->vals = (uint32_t*)calloc(nc, sizeof(uint32_t));
    m->state = (uint8_t*)calloc(nc, 1);
    for (uint32_t i = 0; i < old.cap; i++)
        if (old.state[i] == 1) bmap_put(m, old.keys + (size_t)i * old.ksz, old.vals[i]);
    bmap_free(&old);
}
/* map[k] = v (insert or overwrite) */
static void bmap_put(bmap* m, const uint8_t* k, uint32_t v) {
    if ((m->used + m->tomb + 1) * 2 > m->cap) bmap_grow(m);
    uint32_t i = fnv1a(k, m->ksz) & (m->cap - 1), first_del = 0xFFFFFFFFu;
    for (;; i = (i + 1) & (m->cap - 1)) {
        if (m->state[i] == 0) break;
        if (m->state[i] == 2) { if (first_del == 0xFFFFFFFFu) first_del = i; continue; }
        if (!memcmp(m->keys + (size_t)i * m->ksz, k, m->ksz)) { m->vals[i] = v; return; }
    }
    if (first_del != 0xFFFFFFFFu) { i = first_del; m->tomb--; }
    memcpy(m->keys + (size_t)i * m->ksz, k, m->ksz);
    m->vals[i] = v; m->state[i] = 1; m->used++;
}
/* delete(map, k) */
static void bmap_del(bmap* m, const uint8_t* k) {
    if (!m->cap) return;
    uint32_t i = fnv1a(k, m->ksz) & (m->cap - 1);
    for (uint32_t n = 0; n < m->cap; n++, i = (i + 1) & (m->cap - 1)) {
        if (m->state[i] == 0) return;
        if (m->state[i] == 1 && !memcmp(m->keys + (size_t)i * m->ksz, k, m->ksz)) {
            m->state[i] = 2; m->used--; m->tomb++;
            return;
        }
    }
}

/* ===================================================================================== */
/* Thread / Namespace / Client state (thread_ctx.go:139, ns_ctx.go:110-112, client_ctx.go) */
/* ===================================================================================== */
typedef struct {
    int alive;
    uint32_t ns_id;
    uint8_t mac[6];
    uint8_t ipv4[4];
    uint8_t ipv6[16];
    uint8_t dhcpv6[16];
    uint32_t plugins;
    int has_ra;              /* Ipv6Router != nil */
    int has_ctx;             /* GetTransportCtx() != nil (socketApi.go:174-193) */
    uint8_t ra_prefix[16];   /* Ipv6Router.PrefixIpv6 */
    uint8_t ra_plen;         /* Ipv6Router.PrefixLen */
} orc_client;

typedef struct {
    int alive;
    uint8_t key[12];
    uint32_t plugins;
    uint32_t* order;  /* clientHead dlist, insertion order */
    uint32_t norder, corder;
} orc_ns;

struct orc {
    uint32_t cb_mask;
    bmap ns_map;     /* CTunnelKey (12 B) -> ns_id   (MapNsT) */
    bmap mac_map;    /* ns_id|MAC (10 B)  -> client  (MapClientMAC) */
    bmap ip4_map;    /* ns_id|IPv4 (8 B)  -> client  (MapClientIPv4) */
    bmap ip6_map;    /* ns_id|IPv6 (20 B) -> client  (MapClientIPv6) */
    bmap ft4_map;    /* client|c5tuplekeyv4 (4+13 B) -> flow (TransportCtx.ftv4) */
    bmap ft6_map;    /* client|c5tuplekeyv6 (4+37 B) -> flow (TransportCtx.ftv6) */
    bmap srv_map;    /* client|port BE|proto (7 B) -> 1 (TransportCtx.serverCb)   */
    orc_ns* ns; uint32_t nns;
    orc_client* cl; uint32_t ncl;
};

static int is_zero(const uint8_t* p, int n) {
    for (int i = 0; i < n; i++) if (p[i]) return 0;
    return 1;
}
static void mk_key(uint8_t* k, uint32_t ns_id, const uint8_t* b, int n) {
    memcpy(k, &ns_id, 4);
    memcpy(k + 4, b, (size_t)n);
}

orc_t* orc_new(void) {
    orc_t* o = (orc_t*)calloc(1, sizeof(orc_t));
    bmap_init(&o->ns_map, 12);
    bmap_init(&o->mac_map, 10);
    bmap_init(&o->ip4_map, 8);
    bmap_init(&o->ip6_map, 20);
    bmap_init(&o->ft4_map, 17);
    bmap_init(&o->ft6_map, 41);
    bmap_init(&o->srv_map, 7);
    o->cb_mask = (1u << EMURX_NUM_CB) - 1u; /* production registers all 12 (trex-emu.go:47-67) */
    return o;
}
void orc_free(orc_t* o) {
    if (!o) return;
    bmap_free(&o->ns_map); bmap_free(&o->mac_map); bmap_free(&o->ip4_map); bmap_free(&o->ip6_map);
    bmap_free(&o->ft4_map); bmap_free(&o->ft6_map); bmap_free(&o->srv_map);
    for (uint32_t i = 0; i < o->nns; i++) free(o->ns[i].order);
    free(o->ns); free(o->cl); free(o);
}
void orc_set_callbacks_mask(orc_t* o, uint32_t mask) { o->cb_mask = mask; }

static orc_ns* ns_get(orc_t* o, uint32_t id) {
    if (id >= o->nns) {
        uint32_t n = id + 1 > o->nns * 2 ? id + 1 : o->nns * 2;
        o->ns = (orc_ns*)realloc(o->ns, n * sizeof(orc_ns));
        memset(o->ns + o->nns, 0, (n - o->nns) * sizeof(orc_ns));
        o->nns = n;
    }
    return &o->ns[id];
}
static orc_client* cl_get(orc_t* o, uint32_t id) {
    if (id >= o->ncl) {
        uint32_t n = id + 1 > o->ncl * 2 ? id + 1 : o->ncl * 2;
        o->cl = (orc_client*)realloc(o->cl, n * sizeof(orc_client));
        memset(o->cl + o->ncl, 0, (n - o->ncl) * sizeof(orc_client));
        o->ncl = n;
    }
    return &o->cl[id];
}

/* CThreadCtx.AddNs thread_ctx.go:786-795 */
int orc_ns_add(orc_t* o, const uint8_t key[12], uint32_t ns_id, uint32_t plugin_mask) {
    if (bmap_find(&o->ns_map, key, NULL)) return EMURX_EEXIST;
    orc_ns* n = ns_get(o, ns_id);
    if (n->alive) return EMURX_EEXIST;
    n->alive = 1; memcpy(n->key, key, 12); n->plugins = plugin_mask; n->norder = 0;
    bmap_put(&o->ns_map, key, ns_id);
    return EMURX_OK;
}
/* CThreadCtx.RemoveNs thread_ctx.go:797-812 (refuses while clients are active) */
int orc_ns_remove(orc_t* o, const uint8_t key[12]) {
    uint32_t id;
    if (!bmap_find(&o->ns_map, key, &id)) return EMURX_ENOENT;
    if (o->ns[id].norder) return EMURX_EEXIST;
    o->ns[id].alive = 0;
    bmap_del(&o->ns_map, key);
    return EMURX_OK;
}
int orc_ns_set_plugins(orc_t* o, uint32_t ns_id, uint32_t plugin_mask) {
    if (ns_id >= o->nns || !o->ns[ns_id].alive) return EMURX_ENOENT;
    o->ns[ns_id].plugins = plugin_mask;
    return EMURX_OK;
}

/* CNSCtx.AddClient ns_ctx.go:332-389 */
int orc_client_add(orc_t* o, uint32_t ns_id, uint32_t cid, const uint8_t mac[6],
                   const uint8_t ipv4[4], const uint8_t ipv6[16], const uint8_t dhcpv6[16],
                   uint32_t plugin_mask) {
    static const uint8_t z[16] = {0};
    if (ns_id >= o->nns || !o->ns[ns_id].alive) return EMURX_ENOENT;
    if (!ipv4) ipv4 = z;
    if (!ipv6) ipv6 = z;
    if (!dhcpv6) dhcpv6 = z;
    uint8_t k[KMAX];
    if (is_zero(mac, 6)) return EMURX_EINVAL;
    mk_key(k, ns_id, mac, 6);
    if (bmap_find(&o->mac_map, k, NULL)) return EMURX_EEXIST;
    int has4 = !is_zero(ipv4, 4), has6 = !is_zero(ipv6, 16), has6d = !is_zero(dhcpv6, 16);
    if (has4) { mk_key(k, ns_id, ipv4, 4); if (bmap_find(&o->ip4_map, k, NULL)) return EMURX_EEXIST; }
    if (has6) { mk_key(k, ns_id, ipv6, 16); if (bmap_find(&o->ip6_map, k, NULL)) return EMURX_EEXIST; }
    if (has6d) { mk_key(k, ns_id, dhcpv6, 16); if (bmap_find(&o->ip6_map, k, NULL)) return EMURX_EEXIST; }
    if (cid < o->ncl && o->cl[cid].alive) return EMURX_EEXIST;
    orc_client* c = cl_get(o, cid);
    memset(c, 0, sizeof(*c));
    c->alive = 1; c->ns_id = ns_id; c->plugins = plugin_mask;
    memcpy(c->mac, mac, 6); memcpy(c->ipv4, ipv4, 4); memcpy(c->ipv6, ipv6, 16);
    memcpy(c->dhcpv6, dhcpv6, 16);
    mk_key(k, ns_id, mac, 6); bmap_put(&o->mac_map, k, cid);
    if (has4) { mk_key(k, ns_id, ipv4, 4); bmap_put(&o->ip4_map, k, cid); }
    if (has6) { mk_key(k, ns_id, ipv6, 16); bmap_put(&o->ip6_map, k, cid); }
    if (has6d) { mk_key(k, ns_id, dhcpv6, 16); bmap_put(&o->ip6_map, k, cid); }
    orc_ns* n = &o->ns[ns_id];
    if (n->norder == n->corder) {
        n->corder = n->corder ? n->corder * 2 : 16;
        n->order = (uint32_t*)realloc(n->order, n->corder * sizeof(uint32_t));
    }
    n->order[n->norder++] = cid; /* clientHead.AddLast */
    return EMURX_OK;
}

/* ctx_client_add rpc_base_cmds.go:371-380: AddClient per listed client, stop at the first error */
int orc_clients_add(orc_t* o, const emurx_client_spec* c, uint32_t n, uint32_t* n_added) {
    uint32_t k = 0;
    int rc = EMURX_OK;
    for (; k < n; k++)
        if ((rc = orc_client_add(o, c[k].ns_id, c[k].client_id, c[k].mac, c[k].ipv4, c[k].ipv6, c[k].dhcpv6,
                                 c[k].plugin_mask)))
            break;
    if (n_added) *n_added = k;
    return rc;
}

/* CNSCtx.RemoveClient ns_ctx.go:392-440 */
int orc_client_remove(orc_t* o, uint32_t ns_id, const uint8_t mac[6]) {
    if (ns_id >= o->nns || !o->ns[ns_id].alive) return EMURX_ENOENT;
    if (is_zero(mac, 6)) return EMURX_EINVAL;
    uint8_t k[KMAX];
    uint32_t cid;
    mk_key(k, ns_id, mac, 6);
    if (!bmap_find(&o->mac_map, k, &cid)) return EMURX_ENOENT;
    orc_client* c = &o->cl[cid];
    bmap_del(&o->mac_map, k);
    orc_ns* n = &o->ns[ns_id];
    for (uint32_t i = 0; i < n->norder; i++)
        if (n->order[i] == cid) {
            memmove(n->order + i, n->order + i + 1, (n->norder - i - 1) * sizeof(uint32_t));
            n->norder--;
            break;
        }
    /* delete by key, whoever the entry points at (as the Go code does) */
    if (!is_zero(c->ipv4, 4)) { mk_key(k, ns_id, c->ipv4, 4); bmap_del(&o->ip4_map, k); }
    if (!is_zero(c->ipv6, 16)) { mk_key(k, ns_id, c->ipv6, 16); bmap_del(&o->ip6_map, k); }
    if (!is_zero(c->dhcpv6, 16)) { mk_key(k, ns_id, c->dhcpv6, 16); bmap_del(&o->ip6_map, k); }
    /* TransportCtx.onRemove client_ctx.go:579-595: the client's sockets go with it */
    bmap* tm[3] = {&o->ft4_map, &o->ft6_map, &o->srv_map};
    for (int t = 0; t < 3; t++)
        for (uint32_t i = 0; i < tm[t]->cap; i++)
            if (tm[t]->state[i] == 1 && !memcmp(tm[t]->keys + (size_t)i * tm[t]->ksz, &cid, 4)) {
                tm[t]->state[i] = 2; tm[t]->used--; tm[t]->tomb++;
            }
    c->has_ctx = 0;
    c->alive = 0;
    return EMURX_OK;
}
int orc_client_set_plugins(orc_t* o, uint32_t cid, uint32_t plugin_mask) {
    if (cid >= o->ncl || !o->cl[cid].alive) return EMURX_ENOENT;
    o->cl[cid].plugins = plugin_mask;
    return EMURX_OK;
}

/* CNSCtx.UpdateClientIpv4/Ipv6/DIpv6 ns_ctx.go:442-533 (shared shape) */
static int update_addr(orc_t* o, uint32_t cid, uint8_t* cur, const uint8_t* nw, int n,
                       bmap* m) {
    if (cid >= o->ncl || !o->cl[cid].alive) return EMURX_ENOENT;
    uint32_t ns_id = o->cl[cid].ns_id;
    uint8_t k[KMAX];
    if (!memcmp(cur, nw, (size_t)n)) return EMURX_OK;
    if (!is_zero(cur, n)) {
        mk_key(k, ns_id, cur, n);
        if (!bmap_find(m, k, NULL)) { memset(cur, 0, (size_t)n); return EMURX_ENOENT; }
        bmap_del(m, k);
    }
    if (!is_zero(nw, n)) {
        mk_key(k, ns_id, nw, n);
        if (bmap_find(m, k, NULL)) { memset(cur, 0, (size_t)n); return EMURX_EEXIST; }
        bmap_put(m, k, cid);
    }
    memcpy(cur, nw, (size_t)n);
    return EMURX_OK;
}
int orc_client_update_ipv4(orc_t* o, uint32_t cid, const uint8_t ipv4[4]) {
    if (cid >= o->ncl) return EMURX_ENOENT;
    return update_addr(o, cid, o->cl[cid].ipv4, ipv4, 4, &o->ip4_map);
}
int orc_client_update_ipv6(orc_t* o, uint32_t cid, const uint8_t ipv6[16]) {
    if (cid >= o->ncl) return EMURX_ENOENT;
    return update_addr(o, cid, o->cl[cid].ipv6, ipv6, 16, &o->ip6_map);
}
int orc_client_update_dipv6(orc_t* o, uint32_t cid, const uint8_t d[16]) {
    if (cid >= o->ncl) return EMURX_ENOENT;
    return update_addr(o, cid, o->cl[cid].dhcpv6, d, 16, &o->ip6_map);
}
int orc_client_set_ra(orc_t* o, uint32_t cid, const uint8_t prefix[16], uint8_t plen) {
    if (cid >= o->ncl || !o->cl[cid].alive) return EMURX_ENOENT;
    o->cl[cid].has_ra = 1;
    memcpy(o->cl[cid].ra_prefix, prefix, 16);
    o->cl[cid].ra_plen = plen;
    return EMURX_OK;
}

/* ===================================================================================== */
/* Checksums: gopacket layers/tcpip.go, ip4.go, ip6.go                                     */
/* ===================================================================================== */
/* tcpipChecksum tcpip.go:76-94 */
uint16_t orc_checksum(const uint8_t* data, size_t len, uint32_t csum) {
    long length = (long)len - 1;
    for (long i = 0; i < length; i += 2) {
        csum += (uint32_t)data[i] << 8;
        csum += (uint32_t)data[i + 1];
    }
    if (len % 2 == 1) csum += (uint32_t)data[length] << 8;
    while (csum > 0xffff) csum = (csum >> 16) + (csum & 0xffff);
    return (uint16_t)~csum;
}
/* getCs tcpip.go:22-32 / getCsv6 ip6.go:115-124: byte-pair sum of a pseudo header */
static uint32_t pair_sum(const uint8_t* d, int n) {
    uint32_t csum = 0;
    for (int i = 0; i < n; i += 2) { csum += (uint32_t)d[i] << 8; csum += (uint32_t)d[i + 1]; }
    return csum;
}
/* IPv4Header.GetPhCs ip4.go:49-58 */
static uint32_t ipv4_phcs(const uint8_t* ip) {
    uint8_t ph[12] = {0};
    memcpy(ph, ip + 12, 4);
    memcpy(ph + 4, ip + 16, 4);
    ph[9] = ip[9];
    uint16_t len = (uint16_t)(be16(ip + 2) - (uint16_t)((ip[0] & 0xf) << 2));
    ph[10] = (uint8_t)(len >> 8); ph[11] = (uint8_t)len;
    return pair_sum(ph, 12);
}
/* IPv6Header.GetPhCs ip6.go:126-134 */
static uint32_t ipv6_phcs(const uint8_t* ip, uint16_t osize, uint8_t nh) {
    uint8_t ph[40] = {0};
    memcpy(ph, ip + 8, 16);
    memcpy(ph + 16, ip + 24, 16);
    uint32_t l = (uint32_t)(uint16_t)(be16(ip + 4) - osize);
    ph[32] = (uint8_t)(l >> 24); ph[33] = (uint8_t)(l >> 16); ph[34] = (uint8_t)(l >> 8); ph[35] = (uint8_t)l;
    ph[39] = nh;
    return pair_sum(ph, 40);
}

/* ===================================================================================== */
/* Parser.ParsePacket / parsePacketL4 / processIpv6Options  parser.go:583-959             */
/* ===================================================================================== */
typedef struct {
    const uint8_t* p;
    uint32_t packetSize;
    uint32_t cb_mask;
    emurx_rec* r;
} pctx;

/* "return o.<cb>(ps)": the callback is reached */
static void invoke(pctx* c, int cb) {
    c->r->proto = (uint8_t)cb;
    if (c->cb_mask & (1u << cb)) c->r->status = EMURX_ST_OK;
    else if (cb == EMURX_CB_EAPOL) c->r->status = EMURX_ST_PANIC_NIL_EAPOL; /* nil func, :789 */
    else c->r->status = EMURX_ST_NOT_SUPPORTED; /* parserNotSupported :524 */
}
static void fail(pctx* c, int st) { c->r->status = (uint8_t)st; c->r->proto = EMURX_CB_NONE; }

/* processIpv6Options parser.go:726-746; returns 0 on a Go index-out-of-range panic */
static int ipv6_options(const uint8_t* p, int size, uint8_t* flags) {
    int i = 0;
    uint8_t nh = p[0];
    for (;;) {
        switch (nh) {
        case 0: i++; break;                                        /* IPV6_OPTION_NONE */
        case 5: *flags |= EMURX_FLAG_RTALERT; return 1;            /* IPV6_ROUTER_ALERT */
        default:
            if (i + 1 >= size) return 0;                           /* p[i+1] out of range */
            i = i + 2 + (int)p[i + 1];
        }
        if (i > size - 1) return 1;
        nh = p[i];
    }
}

/* the span p[L4:L4+l4len] of the L4 checksum; Go panics when the uint16 end wraps below L4 */
static int span_ok(uint16_t l4, uint16_t l4len) { return (uint16_t)(l4 + l4len) >= l4; }

/* Parser.parsePacketL4 parser.go:583-724 */
static void parse_l4(pctx* c, uint8_t nextHdr, uint32_t pcs, uint16_t l4len, uint16_t layer3) {
    const uint8_t* p = c->p;
    emurx_rec* ps = c->r;
    uint32_t packetSize = c->packetSize;
    ps->next_hdr = nextHdr;
    switch (nextHdr) {
    case 1: /* IPProtocolICMPv4 */
        if (packetSize < (uint32_t)(uint16_t)(ps->l4 + 8)) { fail(c, EMURX_ST_ICMPV4_TOO_SHORT); return; }
        if (!span_ok(ps->l4, l4len)) { fail(c, EMURX_ST_PANIC_L4LEN); return; }
        if (orc_checksum(p + ps->l4, l4len, 0) != 0) { fail(c, EMURX_ST_ICMPV4_CS); return; }
        ps->l7 = (uint16_t)(ps->l4 + 8);
        invoke(c, EMURX_CB_ICMP);
        return;
    case 2: /* IPProtocolIGMP */
        if (packetSize < (uint32_t)(uint16_t)(ps->l4 + 8)) { fail(c, EMURX_ST_ICMPV4_TOO_SHORT); return; }
        invoke(c, EMURX_CB_IGMP);
        return;
    case 6: { /* IPProtocolTCP */
        if (l4len < 20) { fail(c, EMURX_ST_TCP_TOO_SHORT); return; }
        if ((uint32_t)(uint16_t)(ps->l4 + 12) >= packetSize) { fail(c, EMURX_ST_PANIC_L4LEN); return; }
        uint8_t d = p[(uint16_t)(ps->l4 + 12)];
        uint8_t tcplen = (uint8_t)((d >> 4) << 2);
        if (l4len < tcplen) { fail(c, EMURX_ST_TCP_TOO_SHORT); return; }
        ps->l7 = (uint16_t)(ps->l4 + tcplen);
        ps->l7_len = (uint16_t)(l4len - tcplen);
        if (!span_ok(ps->l4, l4len)) { fail(c, EMURX_ST_PANIC_L4LEN); return; }
        if (orc_checksum(p + ps->l4, l4len, pcs) != 0) { fail(c, EMURX_ST_TCP_CS); return; }
        invoke(c, EMURX_CB_TCP);
        return;
    }
    case 17: { /* IPProtocolUDP */
        if (packetSize < (uint32_t)(uint16_t)(ps->l4 + 8)) { fail(c, EMURX_ST_UDP_TOO_SHORT); return; }
        ps->l7_len = (uint16_t)(l4len - 8);
        const uint8_t* udp = p + ps->l4;
        if (be16(udp + 6) > 0) {
            if (!span_ok(ps->l4, l4len)) { fail(c, EMURX_ST_PANIC_L4LEN); return; }
            if (orc_checksum(p + ps->l4, l4len, pcs) != 0) { fail(c, EMURX_ST_UDP_CS); return; }
        }
        ps->l7 = (uint16_t)(ps->l4 + 8);
        uint16_t src = be16(udp), dst = be16(udp + 2);
        if (dst == 5353) { invoke(c, EMURX_CB_MDNS); return; }
        if (layer3 == 0x86DD) {
            if (src == 547 && dst == 546) { invoke(c, EMURX_CB_DHCPV6); return; }
        } else {
            if (src == 67 && dst == 68) { invoke(c, EMURX_CB_DHCP); return; }
            if (dst == 67 && (src == 67 || src == 68)) { invoke(c, EMURX_CB_DHCPSRV); return; }
        }
        invoke(c, EMURX_CB_UDP);
        return;
    }
    case 58: { /* IPProtocolICMPv6 */
        if (packetSize < (uint32_t)(uint16_t)(ps->l4 + 4)) { fail(c, EMURX_ST_ICMPV6_TOO_SHORT); return; }
        if (!span_ok(ps->l4, l4len)) { fail(c, EMURX_ST_PANIC_L4LEN); return; }
        if (orc_checksum(p + ps->l4, l4len, pcs) != 0) { fail(c, EMURX_ST_ICMPV6_CS); return; }
        uint8_t t = p[ps->l4];
        switch (t) {
        case 1: case 2: case 3: case 4: case 128: case 129: case 130: case 131: case 132:
        case 133: case 134: case 135: case 136:
            invoke(c, EMURX_CB_ICMPV6);
            return;
        default:
            fail(c, EMURX_ST_ICMPV6_UNSUPPORTED);
            return;
        }
    }
    default:
        fail(c, EMURX_ST_L4_UNSUPPORTED);
        return;
    }
}

/* Parser.ParsePacket parser.go:756-959 */
static void parse_packet(uint32_t cb_mask, const uint8_t* p, uint32_t packetSize, uint16_t vport,
                         emurx_rec* ps) {
    pctx c = {p, packetSize, cb_mask, ps};
    memset(ps, 0, sizeof(*ps));
    ps->ns_id = EMURX_ID_NONE;
    ps->client_id = EMURX_ID_NONE;
    ps->proto = EMURX_CB_NONE;
    ps->vport = vport; /* d.Vport = m.port */
    int vlanIndex = 0;
    uint16_t offset = 14;

    if (packetSize < 14) { fail(&c, EMURX_ST_PACKET_TOO_SHORT); return; }
    uint16_t nextHdr = be16(p + 12);
    for (;;) {
        switch (nextHdr) {
        case 0x888E: /* EthernetTypeEAPOL */
            if (packetSize < (uint32_t)(uint16_t)(offset + 4)) { fail(&c, EMURX_ST_EAPOL_TOO_SHORT); return; }
            ps->l3 = offset;
            invoke(&c, EMURX_CB_EAPOL);
            return;
        case 0x0806: /* EthernetTypeARP, ARPHeaderSize = 28 */
            if (packetSize < (uint32_t)(uint16_t)(offset + 28)) { fail(&c, EMURX_ST_ARP_TOO_SHORT); return; }
            ps->l3 = offset;
            invoke(&c, EMURX_CB_ARP);
            return;
        case 0x8100: case 0x88A8: { /* Dot1Q, QinQ */
            if (packetSize < (uint32_t)(uint16_t)(offset + 4)) { fail(&c, EMURX_ST_DOT1Q_TOO_SHORT); return; }
            if (vlanIndex > 1) { fail(&c, EMURX_ST_TOO_MANY_DOT1Q); return; }
            uint32_t val = be32(p + offset - 2) & 0xffff0fffu;
            ps->vlan[vlanIndex] = val;
            vlanIndex++;
            nextHdr = be16(p + offset + 2);
            if (nextHdr == 0x8863 || nextHdr == 0x8864) { invoke(&c, EMURX_CB_PPP); return; }
            offset = (uint16_t)(offset + 4);
            break;
        }
        case 0x8863: case 0x8864: /* PPPoE discovery / session */
            invoke(&c, EMURX_CB_PPP);
            return;
        case 0x0800: { /* EthernetTypeIPv4 */
            ps->l3 = offset;
            if (packetSize < (uint32_t)(uint16_t)(offset + 20)) { fail(&c, EMURX_ST_IPV4_TOO_SHORT); return; }
            const uint8_t* ip = p + offset;
            if ((ip[0] & 0xf0) >> 4 != 4) { fail(&c, EMURX_ST_IPV4_HDR_TOO_SHORT); return; }
            uint16_t frag = be16(ip + 6);
            if ((frag & 0x1FFF) > 0 || (frag & 0x2000) == 0x2000) { fail(&c, EMURX_ST_IPV4_FRAGMENT); return; }
            uint16_t hdr = (uint16_t)((ip[0] & 0xf) << 2);
            if (hdr < 20) { fail(&c, EMURX_ST_IPV4_HDR_TOO_SHORT); return; }
            if (packetSize < (uint32_t)(uint16_t)(offset + hdr)) { fail(&c, EMURX_ST_IPV4_HDR_TOO_SHORT); return; }
            uint16_t totlen = be16(ip + 2);
            if (packetSize < (uint32_t)(uint16_t)(offset + totlen)) { fail(&c, EMURX_ST_IPV4_TOO_SHORT); return; }
            if (orc_checksum(ip, hdr, 0) != 0) { fail(&c, EMURX_ST_IPV4_CS); return; }
            uint16_t l4len = (uint16_t)(totlen - hdr);
            ps->l4 = (uint16_t)(offset + hdr);
            parse_l4(&c, ip[9], ipv4_phcs(ip), l4len, nextHdr);
            return;
        }
        case 0x86DD: { /* EthernetTypeIPv6 */
            ps->l3 = offset;
            if (packetSize < (uint32_t)(uint16_t)(offset + 40)) { fail(&c, EMURX_ST_IPV6_TOO_SHORT); return; }
            const uint8_t* ip = p + offset;
            if ((ip[0] & 0xf0) >> 4 != 6) { fail(&c, EMURX_ST_IPV6_TOO_SHORT); return; }
            uint16_t plen = be16(ip + 4);
            if (packetSize < (uint32_t)(uint16_t)(offset + 40 + plen)) { fail(&c, EMURX_ST_IPV6_TOO_SHORT); return; }
            if (ip[7] == 0) { fail(&c, EMURX_ST_IPV6_HOPLIMIT); return; }
            uint16_t l4 = (uint16_t)(ps->l3 + 40);
            uint16_t l4len = plen;
            uint8_t nh = ip[6];
            uint16_t osize = 0;
            for (int doloop = 1; doloop;) {
                switch (nh) {
                case 0: case 60: case 43: case 51: case 50: case 135: case 139: case 140: {
                    if (l4len < 8) { fail(&c, EMURX_ST_IPV6_TOO_SHORT); return; }
                    /* reads past the frame happen only after a uint16 payload-length wrap;
                       Go would read stale mbuf bytes or panic: undefined -> PANIC status */
                    if ((uint32_t)l4 + 2 > packetSize) { fail(&c, EMURX_ST_PANIC_L4LEN); return; }
                    uint16_t hl = (uint16_t)(((uint16_t)p[l4 + 1] << 3) + 8);
                    if (l4len < hl) { fail(&c, EMURX_ST_IPV6_TOO_SHORT); return; }
                    if ((uint32_t)l4 + hl > packetSize) { fail(&c, EMURX_ST_PANIC_L4LEN); return; }
                    nh = p[l4];
                    if (!ipv6_options(p + l4 + 2, hl - 2, &ps->flags)) { fail(&c, EMURX_ST_PANIC_IPV6_OPT); return; }
                    l4len = (uint16_t)(l4len - hl);
                    osize = (uint16_t)(osize + hl);
                    l4 = (uint16_t)(l4 + hl);
                    break;
                }
                case 44: fail(&c, EMURX_ST_IPV6_FRAGMENT); return;
                case 194: fail(&c, EMURX_ST_IPV6_JUMBO); return;
                case 59: fail(&c, EMURX_ST_IPV6_EMPTY); return;
                default: doloop = 0; break;
                }
            }
            ps->l4 = l4;
            parse_l4(&c, nh, ipv6_phcs(ip, osize, nh), l4len, nextHdr);
            return;
        }
        default:
            fail(&c, EMURX_ST_L3_UNSUPPORTED);
            return;
        }
    }
}

/* ===================================================================================== */
/* Namespace / Client rules of each callback (the emu/plugins rx handlers)    */
/* ===================================================================================== */
static const uint8_t cb_plugin[EMURX_NUM_CB] = {
    EMURX_PLUG_ARP, EMURX_PLUG_ICMP, EMURX_PLUG_IGMP, EMURX_PLUG_DHCP, EMURX_PLUG_DHCPSRV,
    EMURX_PLUG_DHCPV6, EMURX_PLUG_MDNS, EMURX_PLUG_TRANSPORT, EMURX_PLUG_TRANSPORT,
    EMURX_PLUG_IPV6, EMURX_PLUG_DOT1X, EMURX_PLUG_PPP};

/* CNSCtx.CLookupByMac ns_ctx.go:262-272 */
static uint32_t lookup_mac(const orc_t* o, uint32_t ns, const uint8_t* mac) {
    uint8_t k[KMAX]; uint32_t v;
    if (is_zero(mac, 6)) return EMURX_ID_NONE;
    mk_key(k, ns, mac, 6);
    return bmap_find(&o->mac_map, k, &v) ? v : EMURX_ID_NONE;
}
/* CNSCtx.CLookupByIPv4 ns_ctx.go:274-285 */
static uint32_t lookup_ip4(const orc_t* o, uint32_t ns, const uint8_t* ip) {
    uint8_t k[KMAX]; uint32_t v;
    if (is_zero(ip, 4)) return EMURX_ID_NONE;
    mk_key(k, ns, ip, 4);
    return bmap_find(&o->ip4_map, k, &v) ? v : EMURX_ID_NONE;
}
/* CNSCtx.CLookupByIPv6 ns_ctx.go:318-329 */
static uint32_t lookup_ip6(const orc_t* o, uint32_t ns, const uint8_t* ip) {
    uint8_t k[KMAX]; uint32_t v;
    if (is_zero(ip, 16)) return EMURX_ID_NONE;
    mk_key(k, ns, ip, 16);
    return bmap_find(&o->ip6_map, k, &v) ? v : EMURX_ID_NONE;
}
/* Go 1.18 net.IP.To4 != nil for a 16-byte address */
static int is_v4in6(const uint8_t* ip) {
    return is_zero(ip, 10) && ip[10] == 0xff && ip[11] == 0xff;
}
/* net.IP.IsLinkLocalUnicast (Go 1.18 src/net/ip.go) — parity unpinned (std lib) */
static int ip_is_link_local_unicast(const uint8_t* ip) {
    if (is_v4in6(ip)) return ip[12] == 169 && ip[13] == 254;
    return ip[0] == 0xfe && (ip[1] & 0xc0) == 0x80;
}
/* net.IP.IsGlobalUnicast (Go 1.18) */
static int ip_is_global_unicast(const uint8_t* ip) {
    if (is_v4in6(ip)) {
        const uint8_t* v4 = ip + 12;
        if (v4[0] == 255 && v4[1] == 255 && v4[2] == 255 && v4[3] == 255) return 0; /* IPv4bcast */
        if (is_zero(v4, 4)) return 0;                                               /* unspecified */
        if (v4[0] == 127) return 0;                                                 /* loopback */
        if ((v4[0] & 0xf0) == 0xe0) return 0;                                       /* multicast */
        return !ip_is_link_local_unicast(ip);
    }
    static const uint8_t loop6[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1};
    if (is_zero(ip, 16)) return 0;
    if (!memcmp(ip, loop6, 16)) return 0;
    if (ip[0] == 0xff) return 0;
    return !ip_is_link_local_unicast(ip);
}
/* CClient.IsValidPrefix client_ctx.go:279-295 (GetIpv6LocalLink :260-277) */
static int client_valid_prefix(const orc_client* c, const uint8_t* ip) {
    static const uint8_t ll[8] = {0xfe, 0x80, 0, 0, 0, 0, 0, 0};
    if (!memcmp(ip, ll, 8)) return 1;
    if (c->has_ra && c->ra_plen == 64 && !memcmp(c->ra_prefix, ip, 8)) return 1;
    return 0;
}
/* CNSCtx.CLookupByIPv6LocalGlobal ns_ctx.go:288-316 + ExtractOnlyMac client_ctx.go:314-329 */
static uint32_t lookup_ip6_local_global(const orc_t* o, uint32_t ns, const uint8_t* ip) {
    if (!(ip_is_link_local_unicast(ip) || ip_is_global_unicast(ip))) return EMURX_ID_NONE;
    if (ip[11] == 0xff && ip[12] == 0xfe) {
        uint8_t mac[6] = {(uint8_t)(ip[8] ^ 2), ip[9], ip[10], ip[13], ip[14], ip[15]};
        uint32_t cid = lookup_mac(o, ns, mac);
        if (cid != EMURX_ID_NONE && client_valid_prefix(&o->cl[cid], ip)) return cid;
        return EMURX_ID_NONE;
    }
    return lookup_ip6(o, ns, ip);
}
/* CNSCtx.GetFirstClient ns_ctx.go:552-559 */
static uint32_t first_client(const orc_t* o, uint32_t ns) {
    const orc_ns* n = &o->ns[ns];
    return n->norder ? n->order[0] : EMURX_ID_NONE;
}
static int is_bcast(const uint8_t* mac) { /* MACKey.IsBroadcast ns_ctx.go:77-82 */
    for (int i = 0; i < 6; i++) if (mac[i] != 0xff) return 0;
    return 1;
}
/* PluginDhcpNs.GetMacFromDhcp dhcp.go:863-891 + DHCPv4.DecodeFromBytes dhcpv4.go:125-172 */
static int dhcp_chaddr(const uint8_t* p, uint32_t packetSize, const emurx_rec* ps, uint8_t* mac) {
    uint16_t dlen = ps->l7_len;
    if (dlen < 240) return 0;
    if ((uint16_t)(ps->l7 + dlen) < ps->l7 || (uint32_t)ps->l7 + dlen > packetSize)
        return 0; /* the plugin's slice would panic / read stale bytes: no client */
    const uint8_t* d = p + ps->l7;
    if (be32(d + 236) != 0x63825363u) return 0; /* InvalidMagicCookie */
    if (dlen > 240) {
        const uint8_t* opt = d + 240;
        int stop = dlen - 240, start = 0;
        while (start < stop) { /* DHCPOption.decode dhcpv4.go:554-574 */
            uint8_t t = opt[start];
            if (t == 0 || t == 255) {
                if (t == 255) break;
                start++;
                continue;
            }
            if (stop - start < 2) return 0;       /* DecOptionNotEnoughData */
            uint8_t l = opt[start + 1];
            if ((int)l > stop - start - 2) return 0; /* DecOptionMalformed */
            start += l + 2;
        }
    }
    if (d[1] != 1) return 0; /* HardwareType != LinkTypeEthernet */
    if (d[2] != 6) return 0; /* HardwareLen != 6 */
    memcpy(mac, d + 28, 6);
    return 1;
}

static void set_lk(emurx_rec* r, int lk) {
    r->flags = (uint8_t)((r->flags & ~EMURX_FLAG_LK_MASK) | (lk << EMURX_FLAG_LK_SHIFT));
}
/* client found -> check client.PluginCtx.Get(plugin) where the handler does */
static void client_result(const orc_t* o, emurx_rec* r, uint32_t cid, int plug, int check) {
    if (cid == EMURX_ID_NONE) { set_lk(r, EMURX_LK_NO_CLIENT); return; }
    r->client_id = cid;
    if (check && !(o->cl[cid].plugins & (1u << plug))) { set_lk(r, EMURX_LK_CLIENT_NO_PLUGIN); return; }
    set_lk(r, EMURX_LK_CLIENT);
}

static void classify(const orc_t* o, const uint8_t* p, uint32_t packetSize, emurx_rec* r) {
    if (r->status != EMURX_ST_OK) return;
    /* CTunnelKey.Set thread_ctx.go:92-97 -> GetNs thread_ctx.go:777-784 */
    uint8_t key[12] = {0};
    key[0] = (uint8_t)r->vport; key[1] = (uint8_t)(r->vport >> 8);
    memcpy(key + 4, &r->vlan[0], 4);
    memcpy(key + 8, &r->vlan[1], 4);
    uint32_t ns;
    if (!bmap_find(&o->ns_map, key, &ns)) { set_lk(r, EMURX_LK_NO_NS); return; }
    r->ns_id = ns;
    int cb = r->proto, plug = cb_plugin[cb];
    if (!(o->ns[ns].plugins & (1u << plug))) { set_lk(r, EMURX_LK_NS_NO_PLUGIN); return; }
    const uint8_t* dmac = p; /* copy(mackey[:], p[0:6]) */
    switch (cb) {
    case EMURX_CB_ARP: { /* arp.go:904-949 */
        uint16_t op = be16(p + r->l3 + 6);
        if (op == 1) {
            uint32_t cid = lookup_ip4(o, ns, p + r->l3 + 24);
            client_result(o, r, cid, plug, 1);
        } else {
            set_lk(r, EMURX_LK_NS_LEVEL);
        }
        return;
    }
    case EMURX_CB_ICMP: { /* icmp.go:396-427: IPv4 dst, then IsUnicastToMe (client_ctx.go:389) */
        uint32_t cid = lookup_ip4(o, ns, p + r->l3 + 16);
        if (cid != EMURX_ID_NONE && !(packetSize > 6 && !memcmp(o->cl[cid].mac, p, 6)))
            cid = EMURX_ID_NONE;
        client_result(o, r, cid, plug, 0);
        return;
    }
    case EMURX_CB_IGMP: /* igmp.go:1581 namespace level */
    case EMURX_CB_MDNS: /* mdns.go:942 namespace level */
        set_lk(r, EMURX_LK_NS_LEVEL);
        return;
    case EMURX_CB_DHCP: { /* dhcp.go:893-917 */
        uint8_t mac[6];
        memcpy(mac, dmac, 6);
        if (is_bcast(mac) && !dhcp_chaddr(p, packetSize, r, mac)) { set_lk(r, EMURX_LK_NO_CLIENT); return; }
        client_result(o, r, lookup_mac(o, ns, mac), plug, 1);
        return;
    }
    case EMURX_CB_DHCPSRV: { /* dhcpsrv.go:1798-1826 */
        uint32_t cid = is_bcast(dmac) ? first_client(o, ns) : lookup_mac(o, ns, dmac);
        client_result(o, r, cid, plug, 1);
        return;
    }
    case EMURX_CB_EAPOL: { /* dot1x.go:624-650, dot1xDefaultDestMAC 01:80:c2:00:00:03 */
        static const uint8_t pae[6] = {0x01, 0x80, 0xc2, 0x00, 0x00, 0x03};
        uint32_t cid = !memcmp(dmac, pae, 6) ? first_client(o, ns) : lookup_mac(o, ns, dmac);
        client_result(o, r, cid, plug, 1);
        return;
    }
    case EMURX_CB_DHCPV6: /* dhcpv6.go:992-1012 */
    case EMURX_CB_PPP:    /* point2point.go:88-106 */
    case EMURX_CB_TCP:    /* plugin_transport.go:83-115 */
    case EMURX_CB_UDP:
        client_result(o, r, lookup_mac(o, ns, dmac), plug, 1);
        return;
    case EMURX_CB_ICMPV6: { /* ipv6.go:465-540: echo request -> LocalGlobal(dst) */
        if (be16(p + r->l4) == ((128 << 8) | 0)) {
            /* IPv6Header(p[L3:L3+40]) on a frame too short for it (ICMPv6 over IPv4) reads
               stale mbuf bytes in Go: undefined, reported as no client */
            if ((uint32_t)r->l3 + 40 > packetSize) { set_lk(r, EMURX_LK_NO_CLIENT); return; }
            uint32_t cid = lookup_ip6_local_global(o, ns, p + r->l3 + 24);
            if (cid != EMURX_ID_NONE && !(packetSize > 6 && !memcmp(o->cl[cid].mac, p, 6)))
                cid = EMURX_ID_NONE;                               /* IsUnicastToMe */
            if (cid != EMURX_ID_NONE && p[r->l3 + 8] == 0xff) cid = EMURX_ID_NONE; /* mcast src */
            client_result(o, r, cid, plug, 0);
        } else {
            set_lk(r, EMURX_LK_NS_LEVEL);
        }
        return;
    }
    }
}

void orc_parse_only(uint32_t cb_mask, const uint8_t* p, uint32_t len, uint16_t vport,
                    emurx_rec* r) {
    parse_packet(cb_mask, p, len, vport, r);
}

void orc_parse_frame(const orc_t* o, const uint8_t* p, uint32_t len, uint16_t vport,
                     emurx_rec* r) {
    parse_packet(o->cb_mask, p, len, vport, r);
    classify(o, p, len, r);
}

/* ===================================================================================== */
/* Counters: the increments ParsePacket / parsePacketL4 / HandleRxPacket make per frame   */
/* ===================================================================================== */
static void count_frame(const emurx_rec* r, uint32_t bytes, emurx_counters* c) {
    uint64_t* s = c->parser;
    if (r->status >= EMURX_ST_PANIC_L4LEN) { c->ref_panic++; return; }
    if (r->status == EMURX_ST_OK || r->status == EMURX_ST_NOT_SUPPORTED) {
        switch (r->proto) {
        case EMURX_CB_ARP: s[EMURX_PC_arpPkts]++; s[EMURX_PC_arpBytes] += bytes; break;
        case EMURX_CB_ICMP: s[EMURX_PC_icmpPkts]++; s[EMURX_PC_icmpBytes] += bytes; break;
        case EMURX_CB_IGMP: s[EMURX_PC_igmpPkts]++; s[EMURX_PC_igmpBytes] += bytes; break;
        case EMURX_CB_TCP: s[EMURX_PC_tcpPkts]++; s[EMURX_PC_tcpBytes] += bytes; break;
        case EMURX_CB_ICMPV6: s[EMURX_PC_Icmpv6Pkt]++; s[EMURX_PC_Icmpv6Bytes] += bytes; break;
        case EMURX_CB_EAPOL: s[EMURX_PC_eapolPkts]++; s[EMURX_PC_eapolBytes] += bytes; break;
        case EMURX_CB_PPP: break;
        default: /* UDP family: udpPkts first, then the demux counter (parser.go:649-680) */
            s[EMURX_PC_udpPkts]++; s[EMURX_PC_udpBytes] += bytes;
            if (r->proto == EMURX_CB_MDNS) { s[EMURX_PC_mDnsPkts]++; s[EMURX_PC_mDnsBytes] += bytes; }
            if (r->proto == EMURX_CB_DHCP || r->proto == EMURX_CB_DHCPV6) { s[EMURX_PC_dhcpPkts]++; s[EMURX_PC_dhcpBytes] += bytes; }
            if (r->proto == EMURX_CB_DHCPSRV) { s[EMURX_PC_dhcpSrvPkts]++; s[EMURX_PC_dhcpSrvBytes] += bytes; }
            break;
        }
        if (r->status == EMURX_ST_NOT_SUPPORTED) s[EMURX_PC_errParser]++; /* -1 -> errParser */
        return;
    }
    static const int err_counter[EMURX_NUM_STATUS] = {
        -1, -1, EMURX_PC_errPacketIsTooShort, EMURX_PC_errEAPolTooShort, EMURX_PC_errArpTooShort,
        EMURX_PC_errDot1qTooShort, EMURX_PC_errToManyDot1q, EMURX_PC_errIPv4TooShort,
        EMURX_PC_errIPv4HeaderTooShort, EMURX_PC_errIPv4Fragment, EMURX_PC_errIPv4cs,
        EMURX_PC_errIPv6TooShort, EMURX_PC_errIPv6HopLimitDrop, EMURX_PC_errIPv6Empty,
        EMURX_PC_errIPv6OptJumbo, EMURX_PC_errIPv6Fragment, EMURX_PC_errIcmpv4TooShort,
        EMURX_PC_errIcmpv4Cse, EMURX_PC_errTcpTooShort, EMURX_PC_tcpCsErr,
        EMURX_PC_errUdpTooShort, EMURX_PC_udpCsErr, EMURX_PC_errIcmpv6TooShort,
        EMURX_PC_errIcmpv6Cse, EMURX_PC_errIcmpv6Unsupported, EMURX_PC_errL4ProtoUnsupported,
        EMURX_PC_errL3ProtoUnsupported, -1, -1, -1, -1};
    s[err_counter[r->status]]++;
    s[EMURX_PC_errParser]++; /* HandleRxPacket thread_ctx.go:368-369 */
}

static void build_queues(const emurx_rec* rec, uint32_t n, uint32_t* qlist,
                         uint32_t qoff[EMURX_NUM_QUEUES + 1]) {
    uint32_t cnt[EMURX_NUM_QUEUES] = {0};
    for (uint32_t i = 0; i < n; i++)
        cnt[rec[i].status == EMURX_ST_OK ? rec[i].proto : EMURX_Q_DROP]++;
    qoff[0] = 0;
    for (int q = 0; q < EMURX_NUM_QUEUES; q++) qoff[q + 1] = qoff[q] + cnt[q];
    uint32_t pos[EMURX_NUM_QUEUES];
    for (int q = 0; q < EMURX_NUM_QUEUES; q++) pos[q] = qoff[q];
    if (qlist)
        for (uint32_t i = 0; i < n; i++)
            qlist[pos[rec[i].status == EMURX_ST_OK ? rec[i].proto : EMURX_Q_DROP]++] = i;
}

void orc_rx_batch(const orc_t* o, const uint8_t* frames, const emurx_desc* desc, uint32_t n,
                  emurx_rec* rec, uint32_t* qlist, uint32_t qoff[EMURX_NUM_QUEUES + 1],
                  emurx_counters* cnt) {
    if (cnt) memset(cnt, 0, sizeof(*cnt));
    for (uint32_t i = 0; i < n; i++) {
        orc_parse_frame(o, frames + desc[i].off, desc[i].len, desc[i].vport, &rec[i]);
        if (cnt) count_frame(&rec[i], desc[i].len, cnt);
    }
    if (qoff) build_queues(rec, n, qlist, qoff);
}

/* VethIFZmq.OnRxStream veth_zmq.go:277-320 — the offset walk, uint16 running offset */
int orc_zmq_descriptors(const uint8_t* stream, size_t len, emurx_desc* out, uint32_t cap,
                        uint32_t* n_out, int* parse_err) {
    uint32_t blen = (uint32_t)len;
    *n_out = 0;
    *parse_err = 0;
    if (blen < 4) { *parse_err = 1; return EMURX_OK; }
    uint32_t header = be32(stream);
    if (((header & 0xffff0000u) >> 16) != EMURX_ZMQ_MAGIC) { *parse_err = 1; return EMURX_OK; }
    int pkts = (int)(header & 0xffff);
    uint16_t of = 4;
    for (int i = 0; i < pkts; i++) {
        if (blen < (uint32_t)(uint16_t)(of + 4)) { *parse_err = 1; return EMURX_OK; }
        if ((uint16_t)(of + 4) < of) { *parse_err = 2; return EMURX_OK; } /* stream[of:of+4] panics */
        header = be32(stream + of);
        if ((header & 0xff000000u) != 0xAA000000u) { *parse_err = 1; return EMURX_OK; }
        uint8_t vport = (uint8_t)((header & 0x00ff0000u) >> 16);
        uint16_t pktLen = (uint16_t)(header & 0xffff);
        if (blen < (uint32_t)(uint16_t)(of + 4 + pktLen)) { *parse_err = 1; return EMURX_OK; }
        if (pktLen > EMURX_MAX_FRAME) { *parse_err = 2; return EMURX_OK; } /* MbufPoll.Alloc */
        if ((uint16_t)(of + 4 + pktLen) < (uint16_t)(of + 4)) { *parse_err = 2; return EMURX_OK; }
        if (*n_out >= cap) return EMURX_ENOSPC;
        out[*n_out].off = (uint16_t)(of + 4);
        out[*n_out].len = pktLen;
        out[*n_out].vport = vport;
        out[*n_out].pad = 0;
        (*n_out)++;
        of = (uint16_t)(of + 4 + pktLen);
    }
    return EMURX_OK;
}

int orc_rx_stream(const orc_t* o, const uint8_t* msg, size_t len, emurx_rec* rec,
                  uint32_t* qlist, uint32_t cap, uint32_t* n_out,
                  uint32_t qoff[EMURX_NUM_QUEUES + 1], emurx_counters* cnt) {
    emurx_desc* d = (emurx_desc*)malloc(sizeof(emurx_desc) * (cap ? cap : 1));
    int perr = 0;
    memset(cnt, 0, sizeof(*cnt));
    int rc = orc_zmq_descriptors(msg, len, d, cap, n_out, &perr);
    if (rc) { free(d); return rc; }
    cnt->rx_batch = 1;
    if (perr == 1) cnt->rx_parse_err = 1;
    if (perr == 2) cnt->ref_panic++;
    for (uint32_t i = 0; i < *n_out; i++) {
        cnt->rx_pkts++;              /* VethIFZmq.OnRx veth_zmq.go:233-234 */
        cnt->rx_bytes += d[i].len;
        orc_parse_frame(o, msg + d[i].off, d[i].len, d[i].vport, &rec[i]);
        count_frame(&rec[i], d[i].len, cnt);
    }
    build_queues(rec, *n_out, qlist, qoff);
    free(d);
    return EMURX_OK;
}

/* ===================================================================================== */
/* Tx-side checksum generation (the plugins' send paths)                                   */
/* ===================================================================================== */
static void put16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

/* One frame, in place.  IPv4Header.UpdateChecksum ip4.go:132-136; PktChecksumTcpUdp
   tcpip.go:38-40 with IPv4Header.GetPhCs ip4.go:49-58 as tcp_output.go:64-70 / udp.go:143-150
   call it; IPv6Header.FixL4ChecksumOffset ip6.go:40-44 (+ GetPhCs :127-134, nextH =
   o.NextHeader()); ICMPv4Header.UpdateChecksum icmp4.go:252-256. */
uint8_t orc_tx_frame(uint8_t* p, uint32_t len, uint16_t l3, uint16_t l4, uint16_t osize, uint8_t ops,
                     uint8_t nh) {
    const int kind = ops >> EMURX_TX_L4_SHIFT;
    static const int field[7] = {0, 16, 6, 16, 6, 2, 2};
    if (kind > EMURX_TX_L4_ICMP4) return EMURX_TX_RANGE;
    /* every slice the Go code takes must lie inside the frame */
    if ((ops & EMURX_TX_IPV4_HDR) && (uint32_t)l3 + 20 > len) return EMURX_TX_RANGE;
    /* the header slice: IHL * 4 bytes (20, or 24 with IGMP's router-alert option) */
    const uint32_t hlen = (ops & EMURX_TX_IPV4_HDR) && (p[l3] & 0xf) > 5 ? (uint32_t)(p[l3] & 0xf) << 2 : 20;
    if ((ops & EMURX_TX_IPV4_HDR) && (uint32_t)l3 + hlen > len) return EMURX_TX_RANGE;
    if ((kind == EMURX_TX_L4_TCP4 || kind == EMURX_TX_L4_UDP4) && (uint32_t)l3 + 20 > len) return EMURX_TX_RANGE;
    if (kind >= EMURX_TX_L4_TCP6 && kind <= EMURX_TX_L4_ICMP6 && (uint32_t)l3 + 40 > len) return EMURX_TX_RANGE;
    if (kind && (uint32_t)l4 + field[kind] + 2 > len) return EMURX_TX_RANGE;
    if (ops & EMURX_TX_IPV4_HDR) {
        put16(p + l3 + 10, 0);
        put16(p + l3 + 10, orc_checksum(p + l3, hlen, 0));
    }
    if (kind) {
        uint8_t* f = p + l4 + field[kind];
        uint32_t ph = 0;
        put16(f, 0);
        if (kind == EMURX_TX_L4_TCP4 || kind == EMURX_TX_L4_UDP4) ph = ipv4_phcs(p + l3);
        else if (kind != EMURX_TX_L4_ICMP4) ph = ipv6_phcs(p + l3, osize, (ops & EMURX_TX_V6_NH) ? nh : p[l3 + 6]);
        put16(f, orc_checksum(p + l4, len - l4, ph));
    }
    return EMURX_TX_OK;
}

void orc_tx_checksum(uint8_t* frames, const emurx_tx_desc* d, uint32_t n, uint8_t* status) {
    for (uint32_t i = 0; i < n; i++) {
        uint8_t st = orc_tx_frame(frames + d[i].off, d[i].len, d[i].l3, d[i].l4, d[i].osize, d[i].ops, d[i].nh);
        if (status) status[i] = st;
    }
}

/* ===================================================================================== */
/* Tx framing: VethIFZmq.Send / FlushTx src/emu/core/veth_zmq.go:149-200, statement by     */
/* statement (o.vec = the open message's frames, o.txVecSize = their bytes)               */
/* ===================================================================================== */
typedef struct {
    const uint8_t* frames;
    const emurx_desc* d;
    uint32_t first, count;  /* o.vec */
    uint32_t size;          /* o.txVecSize */
    uint8_t* out;
    uint64_t cap, at, nmsg;
    uint64_t* msg_off;
} orc_txz;

static void txz_put(orc_txz* z, const uint8_t* b, uint32_t len) {
    for (uint32_t k = 0; k < len; k++, z->at++)
        if (z->at < z->cap) z->out[z->at] = b[k];
}
static void txz_be32(orc_txz* z, uint32_t v) {
    const uint8_t b[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
    txz_put(z, b, 4);
}
/* FlushTx :149-178 */
static void txz_flush(orc_txz* z) {
    if (z->count == 0) return;
    z->msg_off[z->nmsg++] = z->at;
    txz_be32(z, ((uint32_t)EMURX_ZMQ_MAGIC << 16) + z->count);
    for (uint32_t k = 0; k < z->count; k++) {
        const emurx_desc* e = &z->d[z->first + k];
        txz_be32(z, ((uint32_t)EMURX_ZMQ_PKT_MAGIC << 24) + ((uint32_t)(e->vport & 0xff) << 16) + e->len);
        txz_put(z, z->frames + e->off, e->len);
    }
    z->first += z->count;
    z->count = 0;
    z->size = 0;
}
uint64_t orc_tx_zmq(const uint8_t* frames, const emurx_desc* d, uint32_t n, uint8_t* out, uint64_t cap,
                    uint64_t* msg_off, uint64_t* n_msgs) {
    orc_txz z = {frames, d, 0, 0, 0, out, cap, 0, 0, msg_off};
    for (uint32_t i = 0; i < n; i++) {  /* Send :180-200 */
        const uint32_t pktlen = d[i].len;
        if (z.size + pktlen >= EMURX_ZMQ_TX_MAX_BUFFER) txz_flush(&z);
        z.count++;  /* o.vec = append(o.vec, m) (frames i.. are contiguous in order) */
        z.size += pktlen;
        if (z.count == EMURX_ZMQ_TX_BURST) txz_flush(&z);
    }
    txz_flush(&z);
    msg_off[z.nmsg] = z.at;
    *n_msgs = z.nmsg;
    return z.at;
}

/* ===================================================================================== */
/* Transport flow tables and TransportCtx.handleRxPacket's decision                       */
/* ===================================================================================== */
static int orc_client_ok(const orc_t* o, uint32_t cid) { return cid < o->ncl && o->cl[cid].alive; }

/* TransportCtx.addFlowv4 / addFlowv6 client_ctx.go:629-651 (duplicate: ft_add_err_already_exits) */
int orc_flow_add(orc_t* o, uint32_t cid, const uint8_t* tuple, uint32_t tlen, uint32_t flow) {
    uint8_t k[41];
    if (!tuple || (tlen != 13 && tlen != 37)) return EMURX_EINVAL;
    if (!orc_client_ok(o, cid)) return EMURX_ENOENT;
    if (flow > EMURX_FLOW_ID_MAX) return EMURX_EINVAL;
    memcpy(k, &cid, 4);
    memcpy(k + 4, tuple, tlen);
    bmap* m = tlen == 13 ? &o->ft4_map : &o->ft6_map;
    if (bmap_find(m, k, NULL)) return EMURX_EEXIST;
    bmap_put(m, k, flow);
    o->cl[cid].has_ctx = 1; /* the socket's TransportCtx (socketApi.go:174-193) */
    return EMURX_OK;
}
/* TransportCtx.removeFlowv4 / removeFlowv6 client_ctx.go:597-627 */
int orc_flow_remove(orc_t* o, uint32_t cid, const uint8_t* tuple, uint32_t tlen) {
    uint8_t k[41];
    if (!tuple || (tlen != 13 && tlen != 37)) return EMURX_EINVAL;
    if (!orc_client_ok(o, cid)) return EMURX_ENOENT;
    memcpy(k, &cid, 4);
    memcpy(k + 4, tuple, tlen);
    bmap* m = tlen == 13 ? &o->ft4_map : &o->ft6_map;
    if (!bmap_find(m, k, NULL)) return EMURX_ENOENT;
    bmap_del(m, k);
    return EMURX_OK;
}
static void srv_key(uint8_t* k, uint32_t cid, uint16_t port, uint8_t proto) {
    memcpy(k, &cid, 4);
    k[4] = (uint8_t)(port >> 8); k[5] = (uint8_t)port; k[6] = proto;
}
/* serverCb[port][proto] (TransportCtx.serverCb, client_ctx.go:496; lookupServerPort :1142-1155) */
int orc_server_add(orc_t* o, uint32_t cid, uint16_t port, uint8_t proto) {
    uint8_t k[7];
    if (proto != 6 && proto != 17) return EMURX_EINVAL;
    if (!orc_client_ok(o, cid)) return EMURX_ENOENT;
    srv_key(k, cid, port, proto);
    if (bmap_find(&o->srv_map, k, NULL)) return EMURX_EEXIST;
    bmap_put(&o->srv_map, k, 1);
    o->cl[cid].has_ctx = 1;
    return EMURX_OK;
}
int orc_server_remove(orc_t* o, uint32_t cid, uint16_t port, uint8_t proto) {
    uint8_t k[7];
    if (proto != 6 && proto != 17) return EMURX_EINVAL;
    if (!orc_client_ok(o, cid)) return EMURX_ENOENT;
    srv_key(k, cid, port, proto);
    if (!bmap_find(&o->srv_map, k, NULL)) return EMURX_ENOENT;
    bmap_del(&o->srv_map, k);
    return EMURX_OK;
}
int orc_client_set_transport(orc_t* o, uint32_t cid, int has_ctx) {
    if (!orc_client_ok(o, cid)) return EMURX_ENOENT;
    o->cl[cid].has_ctx = has_ctx != 0;
    return EMURX_OK;
}

/* The flow decision for one classified frame: HandleRxTransPacket plugin_transport.go:117-128
   -> handleRxTransPacket :83-115 -> PluginTransClient.handleRxTransPacket :73-80 ->
   TransportCtx.handleRxPacket client_ctx.go:912-969 (fillv4tuple / fillv6tuple :720-765),
   handleRxTcpNewFlow :829-869, handleRxUdpNewFlow :871-904 up to OnAccept. */
static uint32_t flow_of(const orc_t* o, const uint8_t* p, uint32_t len, const emurx_rec* r) {
    if (r->status != EMURX_ST_OK || (r->proto != EMURX_CB_TCP && r->proto != EMURX_CB_UDP)) return EMURX_FLOW_NONE;
    if (((r->flags & EMURX_FLAG_LK_MASK) >> EMURX_FLAG_LK_SHIFT) != EMURX_LK_CLIENT) return EMURX_FLOW_NONE;
    const orc_client* c = &o->cl[r->client_id];
    if (!c->has_ctx) return EMURX_FLOW_NO_CTX;
    const uint8_t* ip = p + r->l3;
    const uint8_t* udp = p + r->l4; /* layers.UDPHeader(p[ps.L4 : ps.L4+4]) */
    uint8_t k[41];
    uint32_t v, proto;
    memcpy(k, &r->client_id, 4);
    if ((ip[0] >> 4) == 4) { /* buildTuplev4 :89-99 */
        memcpy(k + 4, ip + 12, 4);
        memcpy(k + 8, ip + 16, 4);
        memcpy(k + 12, udp, 4);
        proto = k[16] = ip[9];
        if (bmap_find(&o->ft4_map, k, &v)) return v;
    } else { /* buildTuplev6 :101-112 */
        memcpy(k + 4, ip + 8, 16);
        memcpy(k + 20, ip + 24, 16);
        memcpy(k + 36, udp, 4);
        proto = k[40] = r->next_hdr;
        if (bmap_find(&o->ft6_map, k, &v)) return v;
    }
    if (proto == 6) { /* TcpHeader(p[ps.L4:ps.L4+20]).GetFlags() & 0x3F != 0x2: ft_new_tcp_no_syn */
        uint8_t flags = (uint32_t)r->l4 + 13 < len ? udp[13] : 0; /* past the frame: stale mbuf bytes in Go */
        if ((flags & 0x3f) != 0x2) return EMURX_FLOW_NO_SYN;
    }
    uint8_t sk[7];
    srv_key(sk, r->client_id, (uint16_t)((udp[2] << 8) | udp[3]), proto == 6 ? 6 : 17);
    return bmap_find(&o->srv_map, sk, NULL) ? EMURX_FLOW_NEW : EMURX_FLOW_NO_SERVER;
}

void orc_flows(const orc_t* o, const uint8_t* frames, const emurx_desc* desc, const emurx_rec* rec,
               uint32_t n, uint32_t* flow) {
    for (uint32_t i = 0; i < n; i++) flow[i] = flow_of(o, frames + desc[i].off, desc[i].len, &rec[i]);
}
