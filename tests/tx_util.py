"""Tx checksum cases from the reference's golden captures: every frame the parser accepts
with a verified checksum gives a tx descriptor (the ops its producer ran) and the bytes the
reference's send path wrote.  Shared by the oracle test and the GPU parity test."""
import numpy as np

from emurx import abi

TX_DESC_DTYPE = np.dtype([("off", "<u4"), ("len", "<u2"), ("l3", "<u2"), ("l4", "<u2"), ("osize", "<u2"),
                          ("ops", "u1"), ("nh", "u1"), ("pad", "u1", 2)])
assert TX_DESC_DTYPE.itemsize == 16
KIND = {(4, 6): 1, (4, 17): 2, (6, 6): 3, (6, 17): 4, (6, 58): 5, (4, 1): 6}
FIELD = {1: 16, 2: 6, 3: 16, 4: 6, 5: 2, 6: 2}


def corpus_tx_cases():
    """-> (buf, desc, want, zeroed): frames of the golden corpus whose IPv4 header and/or
    L4 checksum the parser verified, in a batch buffer; `want` = the captured bytes,
    `zeroed` = the same with every field the ops rewrite cleared."""
    import pyoracle
    from emurx import frames as F
    from test_oracle_corpus import load_corpus
    data, off, ln, meta = load_corpus()
    frames = [data[o:o + l].tobytes() for o, l in zip(off, ln)]
    buf, desc = F.pack_frames(frames)
    o = pyoracle.Oracle()
    rec, _, _, _ = o.rx_batch(buf, desc)
    rows = []
    for i, r in enumerate(rec):
        if r["status"] != 0 or r["l3"] == 0:
            continue
        f = frames[i]
        l3, l4, nh = int(r["l3"]), int(r["l4"]), int(r["next_hdr"])
        ver = f[l3] >> 4
        ops = abi.TX_IPV4_HDR if ver == 4 else 0
        kind = KIND.get((ver, nh), 0)
        if kind in (2, 4) and f[l4 + 6:l4 + 8] == b"\0\0":
            kind = 0                      # UDP checksum 0: not computed, not verified
        if ver == 4 and nh == 1 and l4 == 0:
            kind = 0
        ops |= kind << abi.TX_L4_SHIFT
        if ops == 0:
            continue
        v6nh = 0
        if ver == 6 and l4 - l3 - 40 > 0:  # behind extension headers: the final next header
            ops |= abi.TX_V6_NH
            v6nh = nh
        rows.append((i, l3, l4, (l4 - l3 - 40) if ver == 6 else 0, ops, v6nh))
    d = np.zeros(len(rows), TX_DESC_DTYPE)
    for k, (i, l3, l4, osz, ops, v6nh) in enumerate(rows):
        d[k] = (desc[i]["off"], desc[i]["len"], l3, l4, osz, ops, v6nh, (0, 0))
    zeroed = buf.copy()
    for x in d:
        p = int(x["off"])
        if x["ops"] & abi.TX_IPV4_HDR:
            zeroed[p + int(x["l3"]) + 10:p + int(x["l3"]) + 12] = 0
        k = int(x["ops"]) >> abi.TX_L4_SHIFT
        if k:
            q = p + int(x["l4"]) + FIELD[k]
            zeroed[q:q + 2] = 0
    return buf, d, buf, zeroed
