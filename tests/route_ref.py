"""Host restatement of the Namespace-partition packing (test side of emurx_route_dev).

Given a batch's records (the oracle's, or the device's), the records whose Namespace was
found go to emurx_ns_owner(CTunnelKey), in frame order, tagged with their frame index and
the source rank (include/emu_rx.h emurx_route_rec)."""
import numpy as np

from emurx import abi
from emurx import frames as F
from emurx.rx import ns_owner


def owners(rec, n_parts):
    """emurx_ns_owner of every record's CTunnelKey (0xFF for records without a Namespace)."""
    out = np.full(len(rec), 0xFF, np.uint32)
    has = np.nonzero(rec["ns_id"] != abi.ID_NONE)[0]
    if not len(has):
        return out
    k = np.stack([rec["vport"][has].astype(np.uint64), rec["vlan0"][has].astype(np.uint64),
                  rec["vlan1"][has].astype(np.uint64)], 1)
    uk, inv = np.unique(k, axis=0, return_inverse=True)
    own = np.array([ns_owner(F.tunnel_key(int(a), int(b), int(c)), n_parts) for a, b, c in uk], np.uint32)
    out[has] = own[inv.reshape(-1)]
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
