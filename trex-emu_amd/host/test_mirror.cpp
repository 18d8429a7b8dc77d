// test_mirror.cpp — host-only checks of the table mirror (csrc/emurx_mirror.cpp), no GPU.
//
// Mirror::shrink (the allocation fallback of emurx_api.cpp ship_tables): a table
// that has filled to twice its target load (2 / spread: the IPv6 table sized for one address
// per client, then every client given a DHCPv6 address as well, CNSCtx.UpdateClientDIpv6
// ns_ctx.go:442-533) is shrunk step by step.  Each shrink must size the table from its live
// entries, keep one more insert under the 3/4 bound Hash::put relies on, keep every address
// findable, and refuse (ENOMEM upstream) once no denser table is smaller.
#include <cstdio>
#include <cstring>

#include "../csrc/emurx_mirror.h"

using namespace emurx_host;

static int fails = 0;
#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);  \
            ++fails;                                                  \
        }                                                             \
    } while (0)

static void addr(uint8_t a[16], uint32_t cid, uint8_t kind) {
    memset(a, 0, 16);
    a[0] = 0x20;
    a[1] = 0x01;
    a[2] = kind;
    a[12] = (uint8_t)(cid >> 24);
    a[13] = (uint8_t)(cid >> 16);
    a[14] = (uint8_t)(cid >> 8);
    a[15] = (uint8_t)cid;
}

static bool all_found(Mirror& m, uint32_t clients, uint32_t with_d) {
    for (uint32_t c = 0; c < clients; ++c)
        for (uint8_t kind = 6; kind <= (c < with_d ? 7 : 6); ++kind) {
            uint8_t a[16];
            addr(a, c, kind);
            uint32_t key[5] = {0}, v = 0;
            memcpy(key + 1, a, 16);
            if (m.image_lookup(kTabIp6, key, &v) != EMURX_OK || v != c) return false;
        }
    return true;
}

int main() {
    const uint32_t C = 4096;
    Mirror m;
    m.open(16, C);
    const uint8_t key[12] = {0};
    CHECK(m.ns_add(key, 0, EMURX_PLUG_ALL) == EMURX_OK);
    for (uint32_t c = 0; c < C; ++c) {
        uint8_t mac[6] = {0, 0x11, (uint8_t)(c >> 16), (uint8_t)(c >> 8), (uint8_t)c, 1}, ip4[4] = {10, 0, 0, 0};
        uint8_t ip6[16], d6[16] = {0};
        addr(ip6, c, 6);
        ip4[2] = (uint8_t)(c >> 8);
        ip4[3] = (uint8_t)c;
        CHECK(m.client_add(0, c, mac, ip4, ip6, d6, EMURX_PLUG_ALL) == EMURX_OK);
    }
    Hash& t = *m.hashes(kTabIp6);
    const uint32_t b0 = t.buckets, s0 = t.spread;
    // DHCPv6 addresses up to just below the rebuild: live + 1 more would pass 2 / spread
    uint32_t with_d = 0;
    while (!t.full(2) && with_d < C) {
        uint8_t d6[16];
        addr(d6, with_d, 7);
        CHECK(m.update_addr(with_d, 7, d6) == EMURX_OK);
        ++with_d;
    }
    CHECK(t.buckets == b0 && t.spread == s0);  // no growth yet: the table holds 2 / spread
    CHECK((uint64_t)t.live * s0 * 2 > (uint64_t)t.nslots() * 3);  // > 3/4 of 2 / spread
    std::printf("ip6 table: %u live in %u slots, spread %u\n", t.live, t.nslots(), t.spread);
    CHECK(all_found(m, C, with_d));
    int steps = 0;
    while (m.shrink(kTabIp6)) {
        ++steps;
        std::printf("shrunk: spread %u, %u slots, load %.3f\n", t.spread, t.nslots(), (double)t.live / t.nslots());
        CHECK((uint64_t)(t.live + 1) * 4 <= (uint64_t)t.nslots() * 3);  // Hash::put's bound, one more insert
        CHECK(!t.full(1));
        CHECK(all_found(m, C, with_d));
        CHECK(steps < 8);
    }
    CHECK(steps >= 1);
    CHECK(t.spread >= 2);
    // one more DHCPv6 address after the fallback: inserted, everything still found
    if (with_d < C) {
        uint8_t d6[16];
        addr(d6, with_d, 7);
        CHECK(m.update_addr(with_d, 7, d6) == EMURX_OK);
        ++with_d;
        CHECK(all_found(m, C, with_d));
    }
    std::printf(fails ? "FAILED %d\n" : "PASS TestShrinkFromLive\n", fails);
    return fails ? 1 : 0;
}
