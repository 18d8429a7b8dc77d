"""Write the parser_test.go KAT frames (rebuilt byte-for-byte by tests/kat_frames.py) to a
binary fixture the C++ host tests read (trex-emu_amd/host/test_parser.cpp).

    python tests/golden/make_kat_frames.py      -> tests/golden/kat_frames.bin

Format (little endian): u32 count, then per frame: u16 name_len, name, u16 vport, u32 len,
bytes.  Data only: the frames and the vport each reference test sets.
"""
import struct
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path[:0] = [str(HERE.parent), str(HERE.parent.parent / "trex-emu_amd")]
import kat_frames as K  # noqa: E402

CASES = ["test_parser_dot1q_ppp", "test_parser_ppp", "test_parser_arp", "test_parser_arp1",
         "test_parser_icmp", "test_parser_dhcp1", "test_parser_ipv6_option"]


def frames():
    out = [(c, *getattr(K, c)()) for c in CASES]
    f, vp = K.test_parser_dhcp1(valid_ipcs=False)
    out.append(("test_parser_dhcp_invalid_cs", f, vp))
    return out


def main():
    b = bytearray(struct.pack("<I", len(frames())))
    for name, f, vp in frames():
        n = name.encode()
        b += struct.pack("<H", len(n)) + n + struct.pack("<HI", vp, len(f)) + bytes(f)
    (HERE / "kat_frames.bin").write_bytes(bytes(b))
    print(f"{len(frames())} frames -> {HERE / 'kat_frames.bin'}")


if __name__ == "__main__":
    main()
