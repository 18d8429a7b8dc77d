"""Edge-case frames, one or more per return path of ParsePacket / parsePacketL4
(src/emu/core/parser.go:583-959), with the outcome read off the Go code by hand.

Each entry: (name, frame bytes, vport, expected status name, expected callback or None).
Used to pin the oracle (test_oracle_edge.py) and as GPU parity inputs (test_gpu_parity.py).
"""
import struct

from emurx import frames as F

D, S = "00:02:02:02:02:02", "00:01:01:01:01:01"
SIP4, DIP4 = "16.0.0.1", "48.0.0.1"
SIP6, DIP6 = "2001:db8::1", "2001:db8::2"


def eth(etype, payload, pad=False):
    return F.ethernet(D, S, etype, payload, pad=pad)


def v4(proto, l4, **kw):
    return eth(F.ETH_IPV4, F.ipv4(SIP4, DIP4, proto, l4, **kw))


def ph4(proto, n):
    return F.ipv4_pseudo(F.ip4(SIP4), F.ip4(DIP4), proto, n)


def ph6(n, nh, src=SIP6, dst=DIP6):
    return F.ipv6_pseudo(F.ip6(src), F.ip6(dst), n, nh)


def udp4(sp, dp, payload=b"abcd", csum="auto"):
    u = F.udp(sp, dp, payload, csum=csum, pseudo=ph4(17, 8 + len(payload)))
    return v4(17, u)


def udp6(sp, dp, payload=b"abcd", exts=b"", ext_nh=None, csum="auto"):
    u = F.udp(sp, dp, payload, csum=csum, pseudo=ph6(8 + len(payload), 17))
    return eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, ext_nh if exts else 17, exts + u))


def tcp4(payload=b"hello", doff=5, options=b"", csum="auto"):
    n = 20 + len(options) + len(payload)
    t = F.tcp(1000, 80, payload, doff=doff, options=options, csum=csum, pseudo=ph4(6, n))
    return v4(6, t)


def icmp6(typ, code=0, body=b"\x00\x01\x00\x01", csum="auto", src=SIP6, dst=DIP6, exts=b"",
          ext_nh=None):
    m = F.icmp6(typ, code, body, pseudo=ph6(4 + len(body), 58, src, dst), csum=csum)
    return eth(F.ETH_IPV6, F.ipv6(src, dst, ext_nh if exts else 58, exts + m))


def cases():
    c = []
    add = lambda *a: c.append(a)  # noqa: E731
    add("empty", b"", 0, "PACKET_TOO_SHORT", None)
    add("13B", bytes(13), 0, "PACKET_TOO_SHORT", None)
    add("eth_only_ipv4", eth(F.ETH_IPV4, b""), 0, "IPV4_TOO_SHORT", None)
    add("eapol_short", eth(F.ETH_EAPOL, b"\x01\x00\x00"), 0, "EAPOL_TOO_SHORT", None)
    add("eapol_ok", eth(F.ETH_EAPOL, b"\x01\x00\x00\x05"), 0, "OK", "eapol")
    add("arp_short", eth(F.ETH_ARP, bytes(27)), 0, "ARP_TOO_SHORT", None)
    add("arp_ok", eth(F.ETH_ARP, F.arp(1, S, "1.1.1.1", "00:00:00:00:00:00", "1.1.1.2")), 3, "OK", "arp")
    add("dot1q_short", eth(F.ETH_DOT1Q, b"\x00\x07\x08"), 0, "DOT1Q_TOO_SHORT", None)
    add("qinq_3tags", eth(F.ETH_QINQ, F.dot1q(5, F.ETH_DOT1Q) + F.dot1q(6, F.ETH_DOT1Q)
                          + F.dot1q(7, F.ETH_IPV4) + bytes(40)), 1, "TOO_MANY_DOT1Q", None)
    add("dot1q_pppoe_sess", eth(F.ETH_DOT1Q, F.dot1q(9, F.ETH_PPPOE_SESS) + bytes(10)), 2, "OK", "ppp")
    add("pppoe_disc", eth(F.ETH_PPPOE_DISC, F.pppoe_padi()), 0, "OK", "ppp")
    add("qinq_pcp_dei_masked", eth(F.ETH_QINQ, F.dot1q(0xABC, F.ETH_DOT1Q, pcp=7, dei=True)
                                   + F.dot1q(0x123, F.ETH_IPV4, pcp=5) + F.ipv4(SIP4, DIP4, 17, F.udp(1, 2, b"", csum=0))),
        9, "OK", "udp")
    # IPv4 header checks, in Go's order
    add("ipv4_ver5", v4(17, F.udp(1, 2, b"x", csum=0), version=5), 0, "IPV4_HDR_TOO_SHORT", None)
    add("ipv4_mf", v4(17, F.udp(1, 2, b"x", csum=0), flags=1), 0, "IPV4_FRAGMENT", None)
    add("ipv4_fragoff", v4(17, F.udp(1, 2, b"x", csum=0), frag=8), 0, "IPV4_FRAGMENT", None)
    add("ipv4_df_ok", v4(17, F.udp(1, 2, b"x", csum=0), flags=2), 0, "OK", "udp")
    add("ipv4_ihl4", v4(17, F.udp(1, 2, b"x", csum=0), ihl=4), 0, "IPV4_HDR_TOO_SHORT", None)
    add("ipv4_ihl15_short", v4(17, F.udp(1, 2, b"x", csum=0), ihl=15), 0, "IPV4_HDR_TOO_SHORT", None)
    add("ipv4_totlen_gt_frame", v4(17, F.udp(1, 2, b"x", csum=0), length=200), 0, "IPV4_TOO_SHORT", None)
    add("ipv4_bad_cs", v4(17, F.udp(1, 2, b"x", csum=0), csum=0x1234), 0, "IPV4_CS", None)
    opt = bytes([0x94, 0x04, 0x00, 0x00])  # router alert option, IHL 6
    u = F.udp(53, 5000, b"options", csum="auto", pseudo=ph4(17, 15))
    add("ipv4_options_udp", v4(17, u, options=opt), 0, "OK", "udp")
    add("ipv4_eth_padding", F.ethernet(D, S, F.ETH_IPV4, F.ipv4(SIP4, DIP4, 17, F.udp(7, 9, b"", csum="auto", pseudo=ph4(17, 8)))),
        0, "OK", "udp")
    # uint16 wraparound of l4len = totlen - IHL (parser.go:858)
    add("ipv4_totlen_lt_ihl_udp0", v4(17, F.udp(1, 2, b"abcd", csum=0), length=10), 0, "OK", "udp")
    add("ipv4_totlen_lt_ihl_udpcs", v4(17, F.udp(1, 2, b"abcd", csum=0x1111), length=10), 0, "PANIC_L4LEN", None)
    add("ipv4_totlen_lt_ihl_icmp", v4(1, F.icmp4(8, 0, 1, 1, b"abcd"), length=10), 0, "PANIC_L4LEN", None)
    add("ipv4_totlen_lt_ihl_tcp", v4(6, bytes(24), length=10), 0, "PANIC_L4LEN", None)
    add("ipv4_totlen_lt_ihl_igmp", v4(2, bytes(8), length=10), 0, "OK", "igmp")
    add("ipv4_totlen_wrap_udp0", v4(17, F.udp(1, 2, b"abcd", csum=0), length=0xFFF8), 0, "OK", "udp")
    add("ipv4_totlen_wrap_udpcs", v4(17, F.udp(1, 2, b"abcd", csum=5), length=0xFFF8), 0, "PANIC_L4LEN", None)
    # ICMPv4 / IGMP
    add("icmp_ok", v4(1, F.icmp4(8, 0, 7, 9, b"payload")), 0, "OK", "icmp")
    add("icmp_bad_cs", v4(1, F.icmp4(8, 0, 7, 9, b"payload", csum=1)), 0, "ICMPV4_CS", None)
    add("icmp_all_zero", v4(1, bytes(8)), 0, "ICMPV4_CS", None)
    add("icmp_too_short", v4(1, bytes(4)), 0, "ICMPV4_TOO_SHORT", None)
    # the checksum spans totlen - IHL = 4 bytes while the size check wants L4 + 8 bytes
    add("icmp_l4len_lt8_ok", eth(F.ETH_IPV4, F.ipv4(SIP4, DIP4, 1, bytes([0xFF, 0xFF, 0, 0]), length=24)
                                 + bytes(8)), 0, "OK", "icmp")
    add("igmp_ok", v4(2, bytes([0x11, 0x64, 0xEE, 0x9B, 0, 0, 0, 0])), 0, "OK", "igmp")
    add("igmp_short", v4(2, bytes(6)), 0, "ICMPV4_TOO_SHORT", None)
    # TCP
    add("tcp_ok", tcp4(), 0, "OK", "tcp")
    add("tcp_options_ok", tcp4(b"data", doff=7, options=bytes([2, 4, 5, 0xB4, 1, 1, 1, 0])), 0, "OK", "tcp")
    add("tcp_bad_cs", tcp4(csum=0xBEEF), 0, "TCP_CS", None)
    add("tcp_short", v4(6, bytes(19)), 0, "TCP_TOO_SHORT", None)
    add("tcp_doff_too_big", tcp4(b"", doff=15), 0, "TCP_TOO_SHORT", None)
    add("tcp_zero_cs_checked", tcp4(csum=0), 0, "TCP_CS", None)
    # UDP demux
    add("udp_ok", udp4(1234, 5000), 0, "OK", "udp")
    add("udp_cs0_skip", udp4(1234, 5000, csum=0), 0, "OK", "udp")
    add("udp_bad_cs", udp4(1234, 5000, csum=0xABCD), 0, "UDP_CS", None)
    add("udp_short", v4(17, bytes(7)), 0, "UDP_TOO_SHORT", None)
    add("udp_mdns", udp4(5353, 5353), 0, "OK", "mdns")
    add("udp_mdns_any_src", udp4(1, 5353), 0, "OK", "mdns")
    add("udp_dhcp", udp4(67, 68), 0, "OK", "dhcp")
    add("udp_dhcpsrv_68", udp4(68, 67), 0, "OK", "dhcpsrv")
    add("udp_dhcpsrv_67", udp4(67, 67), 0, "OK", "dhcpsrv")
    add("udp_dhcpsrv_other", udp4(69, 67), 0, "OK", "udp")
    add("udp_dhcpv6_over_v4", udp4(547, 546), 0, "OK", "udp")
    add("udp6_dhcpv6", udp6(547, 546), 0, "OK", "dhcpv6")
    add("udp6_dhcp_over_v6", udp6(67, 68), 0, "OK", "udp")
    add("udp6_mdns", udp6(5353, 5353), 0, "OK", "mdns")
    add("udp6_cs0", udp6(1, 2, csum=0), 0, "OK", "udp")
    add("udp6_bad_cs", udp6(1, 2, csum=0x7777), 0, "UDP_CS", None)
    # ICMPv6
    for t, exp in ((1, "OK"), (2, "OK"), (3, "OK"), (4, "OK"), (128, "OK"), (129, "OK"), (130, "OK"),
                   (131, "OK"), (132, "OK"), (133, "OK"), (134, "OK"), (135, "OK"), (136, "OK"),
                   (137, "ICMPV6_UNSUPPORTED"), (143, "ICMPV6_UNSUPPORTED"), (0, "ICMPV6_UNSUPPORTED")):
        add(f"icmp6_type{t}", icmp6(t), 0, exp, "icmpv6" if exp == "OK" else None)
    add("icmp6_bad_cs", icmp6(128, csum=0x1111), 0, "ICMPV6_CS", None)
    add("icmp6_short", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 58, bytes(3))), 0, "ICMPV6_TOO_SHORT", None)
    # L3/L4 unsupported
    add("l4_gre", v4(47, bytes(8)), 0, "L4_UNSUPPORTED", None)
    add("l3_lldp", eth(0x88CC, bytes(46)), 0, "L3_UNSUPPORTED", None)
    add("l3_after_tag", eth(F.ETH_DOT1Q, F.dot1q(3, 0x9000) + bytes(46)), 0, "L3_UNSUPPORTED", None)
    # IPv6 header checks
    add("ipv6_short", eth(F.ETH_IPV6, bytes(39)), 0, "IPV6_TOO_SHORT", None)
    add("ipv6_ver4", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 17, F.udp(1, 2, b"", csum=0), version=4)), 0,
        "IPV6_TOO_SHORT", None)
    add("ipv6_plen_gt", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 17, F.udp(1, 2, b"", csum=0), plen=100)), 0,
        "IPV6_TOO_SHORT", None)
    add("ipv6_hop0", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 17, F.udp(1, 2, b"", csum=0), hop=0)), 0,
        "IPV6_HOPLIMIT", None)
    hbh = F.ipv6_ext(17, bytes([1, 4, 0, 0, 0, 0]))
    add("ipv6_hbh_udp", udp6(9, 10, exts=hbh, ext_nh=0), 0, "OK", "udp")
    add("ipv6_frag", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 44, bytes(16))), 0, "IPV6_FRAGMENT", None)
    add("ipv6_jumbo_nh", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 194, bytes(16))), 0, "IPV6_JUMBO", None)
    add("ipv6_no_next", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 59, bytes(16))), 0, "IPV6_EMPTY", None)
    add("ipv6_hbh_then_frag", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 0, F.ipv6_ext(44, bytes(6)) + bytes(8))), 0,
        "IPV6_FRAGMENT", None)
    add("ipv6_ext_l4len_lt8", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 0, bytes([17, 0, 1, 4]))) + bytes(20), 0,
        "IPV6_TOO_SHORT", None)
    add("ipv6_ext_hl_gt_l4len", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 60, bytes([17, 3, 1, 4, 0, 0, 0, 0]))), 0,
        "IPV6_TOO_SHORT", None)
    chain = (F.ipv6_ext(60, bytes([1, 4, 0, 0, 0, 0])) + F.ipv6_ext(43, bytes([1, 4, 0, 0, 0, 0]))
             + F.ipv6_ext(17, bytes([5, 2, 0, 0, 1, 0])))
    add("ipv6_chain_ra_in_routing", udp6(11, 12, exts=chain, ext_nh=0), 0, "OK", "udp")
    add("ipv6_ra_mld", icmp6(130, body=bytes(20), exts=F.ipv6_ext(58, bytes([5, 2, 0, 0, 1, 0])), ext_nh=0,
                             dst="ff02::1"), 0, "OK", "icmpv6")
    # processIpv6Options reads p[i+1] past the body: PadN len 3 then a non-pad type at i = 5
    add("ipv6_opt_panic", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 0, bytes([17, 0, 1, 3, 0, 0, 0, 7])
                                                   + F.udp(1, 2, b"", csum=0))), 0, "PANIC_IPV6_OPT", None)
    add("ipv6_opt_pad1_run", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 0, bytes([17, 0, 0, 0, 0, 0, 0, 0])
                                                      + F.udp(1, 2, b"", csum=0))), 0, "OK", "udp")
    add("icmp_over_ipv6", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 1, F.icmp4(8, 0, 1, 1, b"xy"))), 0, "OK", "icmp")
    add("igmp_over_ipv6", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 2, bytes(8))), 0, "OK", "igmp")
    add("ipv6_plen_wrap_udp0", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 17, F.udp(1, 2, b"", csum=0), plen=0xFFFF)), 0,
        "OK", "udp")
    add("ipv6_plen_wrap_udpcs", eth(F.ETH_IPV6, F.ipv6(SIP6, DIP6, 17, F.udp(1, 2, b"", csum=9), plen=0xFFFF)), 0,
        "PANIC_L4LEN", None)
    # big frames
    big = bytes(range(256)) * 36
    add("udp_9216", udp4(1111, 2222, big[:9216 - 42]), 0, "OK", "udp")
    add("tcp_1518", tcp4(big[:1518 - 54]), 0, "OK", "tcp")
    add("udp6_odd_len", udp6(3, 4, payload=b"odd-length!"), 0, "OK", "udp")
    return c
