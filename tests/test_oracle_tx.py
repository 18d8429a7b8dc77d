"""The oracle's tx checksum restatement (orc_tx_checksum) against the reference's own send
paths: every frame of the golden captures whose checksums the parser verified is rewritten
with those fields cleared, and must come back byte-identical to what the reference sent."""
import numpy as np

from emurx import abi
import tx_util


def test_tx_oracle_reproduces_captured_checksums(oracle_built):
    import pyoracle
    buf, d, want, zeroed = tx_util.corpus_tx_cases()
    kinds = np.bincount(d["ops"] >> abi.TX_L4_SHIFT, minlength=7)
    assert len(d) > 4000 and kinds[abi.TX_L4_TCP4] > 500 and kinds[abi.TX_L4_UDP4] > 1000
    assert kinds[abi.TX_L4_ICMP6] > 100 and kinds[abi.TX_L4_ICMP4] > 10
    got, st = pyoracle.tx_checksum(zeroed, d)
    assert (st == abi.TX_OK).all()
    bad = [int(i) for i, x in enumerate(d) if got[x["off"]:x["off"] + x["len"]].tobytes()
           != want[x["off"]:x["off"] + x["len"]].tobytes()]
    assert not bad, (len(bad), d[bad[:5]])


def test_tx_oracle_kat_and_range(oracle_built):
    """tcpip_test.go:15-19 KAT (0xbc5f) through the UDP4 op; out-of-range slices untouched."""
    import kat_frames as K
    import pyoracle
    f, _, _ = K.tcpip_ipv4_udp()
    from emurx import frames as F
    buf, desc = F.pack_frames([f, f[:30]])
    d = np.zeros(2, abi.TX_DESC_DTYPE)
    for k in range(2):
        d[k] = (desc[k]["off"], desc[k]["len"], 14, 34, 0,
                abi.TX_IPV4_HDR | (abi.TX_L4_UDP4 << abi.TX_L4_SHIFT), 0, (0, 0))
    z = buf.copy()
    p = int(d[0]["off"])
    z[p + 40:p + 42] = 0
    got, st = pyoracle.tx_checksum(z, d)
    assert list(st) == [abi.TX_OK, abi.TX_RANGE]
    assert (int(got[p + 40]) << 8 | int(got[p + 41])) == K.IPV4_UDP_CSUM
    q = int(d[1]["off"])
    assert got[q:q + 30].tobytes() == z[q:q + 30].tobytes()
