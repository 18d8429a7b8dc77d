"""Host restatement of the Namespace-partition packing (test side of emurx_route_dev).

Given a batch's records (the oracle's, or the device's), the records whose Namespace was
found go to emurx_ns_owner(CTunnelKey), in frame order, tagged with their frame index and
the source rank (include/emu_rx.h emurx_route_rec)."""
import numpy as np

from emurx import abi
from emurx import frames as F
from emurx.rx import ns_owner


def owners(rec, n_parts):
    keys = {}
    out = np.full(len(rec), 0xFF, np.uint32)
    for i, r in enumerate(rec):
        if int(r["ns_id"]) == abi.ID_NONE:
            continue
        k = (int(r["vport"]), int(r["vlan0"]), int(r["vlan1"]))
        if k not in keys:
            keys[k] = ns_owner(F.tunnel_key(*k), n_parts)
        out[i] = keys[k]
    return out


def route(rec, n_parts, my_rank):
    """-> list over destinations of emurx_route_rec arrays (frame order)."""
    own = owners(rec, n_parts)
    out = []
    for d in range(n_parts):
        idx = np.nonzero(own == d)[0]
        rr = np.zeros(len(idx), abi.ROUTE_REC_DTYPE)
        rr["rec"] = rec[idx]
        rr["src_index"] = idx
        rr["src_rank"] = my_rank
        out.append(rr)
    return out
