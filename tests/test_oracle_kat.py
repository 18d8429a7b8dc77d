"""Pin the CPU oracle to the reference's own known answers (no GPU).

Each case rebuilds a frame of src/emu/core/parser_test.go byte-for-byte and checks the
assertion that Go test makes; tcpip_test.go pins the checksum arithmetic.
"""
import numpy as np
import pytest

import kat_frames as K
from emurx import abi
from emurx import frames as F


def parse(o, frame, vport, mask=(1 << 12) - 1):
    import pyoracle
    return pyoracle.parse_only(frame, vport, mask)


def tun(r):
    return (int(r["vport"]), int(r["vlan0"]), int(r["vlan1"]))


def test_parser_arp_too_many_dot1q(oracle_built):
    f, vp = K.test_parser_arp()
    r = parse(None, f, vp)
    assert r["status"] == abi.ST["TOO_MANY_DOT1Q"]          # parser_test.go:166


def test_parser_arp1(oracle_built):
    f, vp = K.test_parser_arp1()
    r = parse(None, f, vp, 1 << abi.CB_ARP)
    assert r["status"] == abi.ST["OK"] and r["proto"] == abi.CB_ARP   # :222
    assert tun(r) == (7, 0x81000007, 0x81000FFF)             # :224-233


def test_parser_icmp(oracle_built):
    f, vp = K.test_parser_icmp()
    r = parse(None, f, vp, 1 << abi.CB_ICMP)
    assert r["status"] == abi.ST["OK"] and r["proto"] == abi.CB_ICMP
    assert tun(r) == (7, 0x81000007, 0x81000FFF)
    assert (r["l3"], r["l4"], r["l7"]) == (22, 42, 50)       # :297-302


def test_parser_dhcp1(oracle_built):
    f, vp = K.test_parser_dhcp1()
    r = parse(None, f, vp, 1 << abi.CB_DHCP)
    assert r["status"] == abi.ST["OK"] and r["proto"] == abi.CB_DHCP
    assert tun(r) == (7, 0x81000007, 0x81000001)             # :371-381
    assert (r["l3"], r["l4"], r["l7"]) == (22, 42, 50)       # :382-387


def test_parser_dhcp_invalid_cs(oracle_built):
    f, vp = K.test_parser_dhcp1(valid_ipcs=False)
    r = parse(None, f, vp, 1 << abi.CB_DHCP)
    assert r["status"] == abi.ST["IPV4_CS"]                  # :451


@pytest.mark.parametrize("case", ["test_parser_dot1q_ppp", "test_parser_ppp"])
def test_parser_ppp(oracle_built, case):
    f, vp = getattr(K, case)()
    r = parse(None, f, vp, (1 << 12) - 1)
    assert r["status"] == abi.ST["OK"] and r["proto"] == abi.CB_PPP
    assert r["l3"] == 0 and r["vport"] == vp
    if case == "test_parser_dot1q_ppp":
        assert r["vlan0"] == 0x81000064
    # default registration (Parser.Init): ppp -> parserNotSupported -> errParser
    r = parse(None, f, vp, 0)
    assert r["status"] == abi.ST["NOT_SUPPORTED"]


def test_parser_ipv6_option(oracle_built):
    f, vp = K.test_parser_ipv6_option()
    r = parse(None, f, vp)
    assert (r["l3"], r["l4"]) == (18, 66)
    assert r["flags"] & abi.FLAG_RTALERT
    assert r["status"] == abi.ST["ICMPV6_CS"]
    assert r["next_hdr"] == 58


def test_checksum_kat_ipv4_udp(oracle_built):
    import pyoracle
    frame, ip, u = K.tcpip_ipv4_udp(csum=0)
    ph = F.ipv4_pseudo(ip[12:16], ip[16:20], 17, 8)
    assert pyoracle.checksum(u, ph) == K.IPV4_UDP_CSUM        # tcpip_test.go:16
    frame, ip, u = K.tcpip_ipv4_udp()
    r = parse(None, frame, 0)
    assert r["status"] == abi.ST["OK"] and r["proto"] == abi.CB_UDP
    frame, ip, u = K.tcpip_ipv4_udp(csum=K.IPV4_UDP_CSUM ^ 1)
    assert parse(None, frame, 0)["status"] == abi.ST["UDP_CS"]


def test_checksum_kat_ipv6_dstopts(oracle_built):
    import pyoracle
    frame, ip, u = K.tcpip_ipv6_udp_dstopts(csum=0)
    ph = F.ipv6_pseudo(ip[8:24], ip[24:40], 8, 17)
    assert pyoracle.checksum(u, ph) == K.IPV6_UDP_DSTOPTS_CSUM  # tcpip_test.go:17
    frame, ip, u = K.tcpip_ipv6_udp_dstopts()
    r = parse(None, frame, 0)
    assert r["status"] == abi.ST["OK"] and r["proto"] == abi.CB_UDP
    assert r["l4"] == 14 + 40 + 8


def test_checksum_matches_python_restatement(oracle_built):
    import pyoracle
    rng = np.random.default_rng(1)
    for n in list(range(0, 40)) + [1499, 1500, 9000]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        init = int(rng.integers(0, 1 << 21))
        assert pyoracle.checksum(d, init) == F.csum_fold(d, init)
