"""Classification outcomes pinned by the reference's own plugin simulations.

Each capture in unit-test/exp (tests/golden/corpus_frames.npz) was recorded by a Go test that
builds one Namespace and its clients (createSimulationEnv in the plugin's *_test.go), injects
the rx frames and records what the plugins sent.  Rebuilding that environment from the test's
source and classifying the capture's rx frames gives an outcome the capture itself vouches
for: the plugin answered with frames that only a found client sends (an ARP or echo reply
from the client's MAC, the client's next DHCP / DHCPv6 / EAPOL message), or, for arp5, sent
no reply at all.  This pins the lookup rules -- MAC[dst], IPv4[dst] + IsUnicastToMe, IPv4 of
the ARP target, the IPv6 map behind CLookupByIPv6LocalGlobal, the DHCP chaddr of a broadcast
OFFER, the first client of an EAPOL PAE frame or of a broadcast to the DHCP server --
against the reference rather than against the oracle's reading of the Go code.
"""
import struct

# the one Namespace of every environment: vport 1, tags 0x8100/1 and 0x8100/2 (CTunnelKey bytes)
NS_KEY = struct.pack("<HHII", 1, 0, 0x81000001, 0x81000002)
PLUG = ["arp", "icmp", "igmp", "dhcp", "dhcpsrv", "dhcpv6", "mdns", "transport", "ipv6", "dot1x", "ppp"]

# createSimulationEnv of each plugin test: client 0's MAC / IPv4 / IPv6 and the one plugin the
# test creates on the Namespace and the client
ENVS = {
    # src/emu/plugins/icmp/icmp_test.go:76-100 (num = 1: a = b = 0)
    "icmp": dict(mac=bytes([0, 0, 1, 0, 0, 0]), ipv4=bytes([16, 0, 0, 0]), ipv6=None, plugin="icmp"),
    # src/emu/plugins/arp/arp_test.go:78-106
    "arp": dict(mac=bytes([0, 0, 1, 0, 0, 0]), ipv4=bytes([16, 0, 0, 0]), ipv6=None, plugin="arp"),
    # src/emu/plugins/ipv6/ipv6_test.go:81-113 (static Ipv6 2001:db8::2)
    "ipv6": dict(mac=bytes([0, 0, 1, 0, 0, 0]), ipv4=bytes([16, 0, 0, 0]),
                 ipv6=bytes([0x20, 0x01, 0x0D, 0xB8] + [0] * 11 + [2]), plugin="ipv6"),
    # src/emu/plugins/dhcpv4/dhcp_test.go:83-101 (no IPv4 yet)
    "dhcp": dict(mac=bytes([0, 0, 1, 0, 0, 1]), ipv4=None, ipv6=None, plugin="dhcp"),
    # src/emu/plugins/dhcpv6/dhcpv6_test.go:83-109
    "dhcpv6": dict(mac=bytes([0, 0, 1, 0, 0, 1]), ipv4=None, ipv6=None, plugin="dhcpv6"),
    # src/emu/plugins/dot1x/dot1x_test.go:82-102
    "dot1x": dict(mac=bytes([0, 0, 1, 0, 0, 1]), ipv4=None, ipv6=None, plugin="dot1x"),
    # src/emu/plugins/dhcpv4srv/dhcpsrv_test.go:413-455: vport 1 without tags, client 0 runs the
    # DHCP server (its plugins dhcpsrv + transport, the Namespace's dhcpsrv)
    "dhcpsrv": dict(mac=bytes([0, 0, 1, 0, 0, 0]), ipv4=bytes([16, 0, 0, 0]),
                    ipv6=bytes([0x20, 0x01, 0x0D, 0xB8] + [0] * 12), plugin="dhcpsrv",
                    client_plugins=("dhcpsrv", "transport"), key=struct.pack("<HHII", 1, 0, 0, 0)),
    # src/emu/plugins/igmp/igmp_test.go:114-132
    "igmp": dict(mac=bytes([0, 0, 1, 0, 0, 1]), ipv4=None, ipv6=None, plugin="igmp"),
    # src/emu/plugins/mdns/mdns_test.go:128-150 (vport 1 without tags)
    "mdns": dict(mac=bytes([0, 0, 1, 0, 0, 0]), ipv4=bytes([16, 0, 0, 0]), ipv6=None, plugin="mdns",
                 key=struct.pack("<HHII", 1, 0, 0, 0)),
    # src/emu/plugins/dns/dns_test.go:138-184: "dns:N" = clients 0..N-1 (N = the test's
    # clientsToSim), MAC 00:00:01:00:00:j, 16.0.0.j, 2001:db8::j, plugins dns + transport; the
    # DNS traffic rides transport UDP sockets, so the Namespace's transport plugin takes it
    "dns": dict(mac=None, ipv4=None, ipv6=None, plugin="transport", key=struct.pack("<HHII", 1, 0, 0, 0)),
}
# clientsToSim of each DNS capture (dns_test.go testname / clientsToSim pairs)
DNS_CLIENTS = {3: 1, 4: 1, 5: 2, 6: 2, 7: 2, 8: 2, 9: 2, 10: 2, 12: 2, 13: 3, 14: 4, 15: 4, 16: 4, 17: 4,
               18: 3, 19: 3, 20: 4, 21: 4}

# (capture, environment, lookup outcome of every rx frame, client id or None, the capture's evidence)
CASES = [
    ("icmp1.json", "icmp", "CLIENT", 0, "6 echo requests, 6 echo replies from 00:00:01:00:00:00"),
    ("arp4.json", "arp", "CLIENT", 0, "6 requests for 16.0.0.0, 6 ARP replies (op 2) from the client"),
    ("arp5.json", "arp", "NO_CLIENT", None, "6 requests for 16.0.0.5, no ARP reply in the capture"),
    ("icmpv6_1.json", "ipv6", "CLIENT", 0, "6 echo requests to 2001:db8::2, 6 echo replies from it"),
    ("icmpv6_2.json", "ipv6", "CLIENT", 0, "6 echo requests to 2001:db8::2, 6 echo replies from it"),
    ("dhcp1.json", "dhcp", "CLIENT", 0, "unicast OFFER / ACKs, the client's REQUESTs follow"),
    ("dhcp4.json", "dhcp", "CLIENT", 0, "unicast OFFERs, the client's REQUESTs follow"),
    ("dhcp5.json", "dhcp", "CLIENT", 0, "broadcast OFFERs (chaddr rule), the client's REQUESTs follow"),
    ("dhcp6.json", "dhcp", "CLIENT", 0, "broadcast OFFERs (chaddr rule), the client's REQUESTs follow"),
    ("dhcp7.json", "dhcp", "CLIENT", 0, "broadcast OFFERs (chaddr rule), the client's REQUESTs follow"),
    ("dhcpv6_1.json", "dhcpv6", "CLIENT", 0, "ADVERTISE / REPLY to the client's MAC, its next messages follow"),
    ("dhcpv6_3.json", "dhcpv6", "CLIENT", 0, "ADVERTISE / REPLY to the client's MAC, its next messages follow"),
    ("dhcpv6_4.json", "dhcpv6", "CLIENT", 0, "ADVERTISE / REPLY to the client's MAC, its next messages follow"),
    ("dhcpv6_5.json", "dhcpv6", "CLIENT", 0, "ADVERTISE / REPLY to the client's MAC, its next messages follow"),
    ("dot1x_1.json", "dot1x", "CLIENT", 0, "PAE group frames (first-client rule), EAPOL answers follow"),
    ("dot1x_4.json", "dot1x", "CLIENT", 0, "PAE group frames (first-client rule), EAPOL answers follow"),
    ("dot1x_7.json", "dot1x", "CLIENT", 0, "PAE group frames (first-client rule), EAPOL answers follow"),
] + [
    # broadcast DISCOVER / REQUEST -> GetFirstClient (the server), unicast ones -> MAC[dst]; the
    # server client answers from 00:00:01:00:00:00 in every capture but dhcpsrv7 (no answer)
    (f"dhcpsrv{i}.json", "dhcpsrv", "CLIENT", 0, "the server client (first client) answers")
    for i in (1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19)
] + [
    # Namespace-level callbacks: the Namespace found with the plugin, no client lookup; the
    # Namespace's plugin answered (IGMP / MLD reports, mDNS responses, ND advertisements)
    (f"igmp{i}.json", "igmp", "NS_LEVEL", None, "the Namespace's IGMP plugin reports")
    for i in (3, 4, 6, 10, 11)
] + [
    (f"mdns{i}.json", "mdns", "NS_LEVEL", None, "the Namespace's mDNS plugin answers every query")
    for i in range(3, 23)
] + [
    (f"{c}.json", "ipv6", "NS_LEVEL", None, "the Namespace's IPv6 plugin answers (NA, MLD reports)")
    for c in ("ipv6nd_1", "ipv6nd_2", "ipv6nd_3", "ipv6nd_4", "ipv6nd_rpc", "mld1_1", "mld2_1", "mld2_2", "mld2_10")
] + [
    # client "dst": the client whose MAC the frame is sent to (MAC[dst], the transport rule)
    (f"dns{i}.json", f"dns:{n}", "CLIENT", "dst", "the DNS plugins' queries and answers around them")
    for i, n in sorted(DNS_CLIENTS.items())
]


def rx_frames(z, capture):
    """The capture's rx frames, in order (z: the corpus npz)."""
    import numpy as np
    files = [str(x) for x in z["files"]]
    src, meta, off, ln, data = z["src"], z["meta"], z["off"], z["len"], z["data"]
    idx = np.nonzero((src == files.index(capture)) & (meta == 1))[0]
    return [data[off[i]:off[i] + ln[i]].tobytes() for i in idx]


def load_env(target, env):
    """One Namespace with the environment's plugin and its client(s): client 0 (ns id 0,
    client id 0), or for "dns:N" clients 0..N-1."""
    name, _, count = env.partition(":")
    e = ENVS[name]
    m = 1 << PLUG.index(e["plugin"])
    cm = 0
    for pl in e.get("client_plugins", (e["plugin"],)):
        cm |= 1 << PLUG.index(pl)
    assert target.ns_add(e.get("key", NS_KEY), 0, m) == 0
    if name == "dns":
        for j in range(int(count)):
            assert target.client_add(0, j, bytes([0, 0, 1, 0, 0, j]), bytes([16, 0, 0, j]),
                                     bytes([0x20, 0x01, 0x0D, 0xB8] + [0] * 11 + [j]), None, cm) == 0
        return
    assert target.client_add(0, 0, e["mac"], e["ipv4"], e["ipv6"], None, cm) == 0


def expected_clients(frames, cid):
    """The client id every frame must resolve to (None: no client)."""
    import numpy as np
    if cid == "dst":
        return np.array([f[5] for f in frames], np.uint32)
    return np.full(len(frames), 0xFFFFFFFF if cid is None else cid, np.uint32)
