"""Known-answer frames rebuilt byte-for-byte from the reference's own tests.

src/emu/core/parser_test.go builds each frame with gopacket.SerializeLayers; the
expectations are the test's own assertions (file:line cited per frame).
src/external/google/gopacket/layers/tcpip_test.go:15-19 pins two L4 checksums.
"""
from emurx import frames as F

SRC_MAC = "00:01:01:01:01:01"
DST_MAC = "00:02:02:02:02:02"


def arp_req():
    return F.arp(1, SRC_MAC, "0.0.0.0", "00:00:00:00:00:00", "0.0.0.0")


def test_parser_arp():
    """TestParserArp parser_test.go:114-171: three tags -> errToManyDot1q == 1."""
    l2 = (F.dot1q(7, F.ETH_DOT1Q) + F.dot1q(7, F.ETH_DOT1Q) + F.dot1q(0x1FF, F.ETH_ARP, pcp=3)
          + arp_req())
    return F.ethernet(DST_MAC, SRC_MAC, F.ETH_DOT1Q, l2), 7


def test_parser_arp1():
    """TestParserArp1 parser_test.go:173-234: arp cb once, Tun {7, 0x81000007, 0x81000fff}."""
    l2 = F.dot1q(7, F.ETH_DOT1Q) + F.dot1q(0xFFF, F.ETH_ARP, pcp=3) + arp_req()
    return F.ethernet(DST_MAC, SRC_MAC, F.ETH_DOT1Q, l2), 7


def test_parser_icmp():
    """TestParserIcmp parser_test.go:236-303: icmp cb, Tun as above, (L3,L4,L7)=(22,42,50).
    FixLengths + ComputeChecksums: IPv4 Length 44 is overwritten with 32."""
    icmp = F.icmp4(8, 0, 1, 0x11, bytes([1, 2, 3, 4]))
    ip = F.ipv4("16.0.0.1", "48.0.0.1", 1, icmp, ttl=128, ident=0xCC)
    l2 = F.dot1q(7, F.ETH_DOT1Q) + F.dot1q(0xFFF, F.ETH_IPV4, pcp=3) + ip
    return F.ethernet(DST_MAC, SRC_MAC, F.ETH_DOT1Q, l2), 7


def _dhcp1_payload():
    opts = [
        F.dhcp_option(53, bytes([1])),                 # DHCPOptMessageType Discover
        F.dhcp_option(12, b"example.com"),             # DHCPOptHostname
        F.dhcp_option(0),                              # DHCPOptPad
        F.dhcp_option(55, bytes([1, 28, 2, 3, 15, 6, 119, 12, 44, 26, 121, 42])),
    ]
    return F.dhcpv4(1, 0x12345678, "12:34:56:78:9a:bc", opts)


def test_parser_dhcp1(valid_ipcs=True):
    """TestParserDhcp1 parser_test.go:305-388 (UDP csum 0, IPv4 csum fixed afterwards):
    dhcp cb, Tun {7, 0x81000007, 0x81000001}, (22,42,50).
    TestParserDhcpInvalidCs :390-454 (valid_ipcs=False): errIPv4cs == 1."""
    u = F.udp(67, 68, _dhcp1_payload(), csum=0)
    ip = F.ipv4("16.0.0.1", "48.0.0.1", 17, u, ttl=128, ident=0xCC,
                csum="auto" if valid_ipcs else 0)
    l2 = F.dot1q(7, F.ETH_DOT1Q) + F.dot1q(0x1, F.ETH_IPV4, pcp=3) + ip
    return F.ethernet(DST_MAC, SRC_MAC, F.ETH_DOT1Q, l2), 7


def test_parser_dot1q_ppp():
    """TestParserDot1Q_PPP parser_test.go:35-75: tagged PPPoE discovery -> ppp cb."""
    return F.ethernet(DST_MAC, SRC_MAC, F.ETH_DOT1Q,
                      F.dot1q(100, F.ETH_PPPOE_DISC) + F.pppoe_padi()), 100


def test_parser_ppp():
    """TestParser_PPP parser_test.go:77-112: untagged PPPoE discovery -> ppp cb."""
    return F.ethernet(DST_MAC, SRC_MAC, F.ETH_PPPOE_DISC, F.pppoe_padi()), 0


IPV6_OPTION_PACKET = bytes([
    0x33, 0x33, 0x00, 0x00, 0x00, 0x01, 0x6c, 0x31, 0x0e, 0x28,
    0x4f, 0x57, 0x81, 0x00, 0x00, 0x67, 0x86, 0xdd, 0x60, 0x00,
    0x00, 0x00, 0x00, 0x24, 0x00, 0x01, 0xfe, 0x80, 0x00, 0x00,
    0x00, 0x00, 0x00, 0x00, 0x6e, 0x31, 0x0e, 0xff, 0xfe, 0x28,
    0x4f, 0x57, 0xff, 0x01, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
    0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x01, 0x3a, 0x00,
    0x01, 0x00, 0x05, 0x02, 0x00, 0x00, 0x82, 0x00, 0x8b, 0xe6,
    0x27, 0x10, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
    0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
    0x02, 0x7d, 0x00, 0x00])


def test_parser_ipv6_option():
    """TestParserIpv6Option parser_test.go:465-487 (literal frame, no assertion in Go):
    HBH with PadN then Router-Alert -> Flags=1, L3=18, L4=66; ICMPv6 csum fails."""
    return IPV6_OPTION_PACKET, 7


# tcpip_test.go:15-19 --------------------------------------------------------------------
IPV4_UDP_CSUM = 0xBC5F
IPV6_UDP_DSTOPTS_CSUM = 0x4D21


def tcpip_ipv4_udp(csum=IPV4_UDP_CSUM):
    """TestIPv4UDPChecksum tcpip_test.go:57-95: 192.0.2.1->198.51.100.1, 12345->9999."""
    u = F.udp(12345, 9999, b"", csum=csum)
    ip = F.ipv4("192.0.2.1", "198.51.100.1", 17, u, ttl=64)
    return F.ethernet(DST_MAC, SRC_MAC, F.ETH_IPV4, ip, pad=False), ip, u


def tcpip_ipv6_udp_dstopts(csum=IPV6_UDP_DSTOPTS_CSUM):
    """TestIPv6UDPChecksumWithIPv6DstOpts tcpip_test.go:97-135: PadN(4) dst-opts header."""
    u = F.udp(12345, 9999, b"", csum=csum)
    dst = bytes([17, 0, 0x01, 0x04, 0, 0, 0, 0])
    ip = F.ipv6("2001:db8::1", "2001:db8::2", 60, dst + u, hop=64)
    return F.ethernet(DST_MAC, SRC_MAC, F.ETH_IPV6, ip, pad=False), ip, u
