"""Print INTEGRATION.md's entry-point index: every function include/emu_rx.h declares, by
group, with the header line that declares it.  Fails if a declared function has no group.

    python tools/entry_index.py            # print the table
    python tools/entry_index.py --write    # replace the table at the end of INTEGRATION.md
"""
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HDR = ROOT / "include" / "emu_rx.h"
DOC = ROOT / "INTEGRATION.md"

GROUPS = [
    ("Lifecycle and errors", ["emurx_abi_version", "emurx_build_id", "emurx_open", "emurx_close", "emurx_strerror"],
     "`NewThreadCtx` / `Parser.Init` (`thread_ctx.go`, `parser.go:567-581`)"),
    ("Parser registration", ["emurx_register", "emurx_set_callbacks_mask", "emurx_get_callbacks_mask"],
     "`Parser.Register` `parser.go:528-565`"),
    ("Namespace table", ["emurx_ns_add", "emurx_ns_remove", "emurx_ns_set_plugins", "emurx_ns_owner"],
     "`CThreadCtx.AddNs/RemoveNs` `thread_ctx.go:786-812`, ns `PluginCtx`"),
    ("Client tables", ["emurx_client_add", "emurx_clients_add", "emurx_client_remove", "emurx_client_set_plugins",
                       "emurx_client_update_ipv4", "emurx_client_update_ipv6", "emurx_client_update_dipv6",
                       "emurx_client_set_ra"],
     "`CNSCtx.AddClient/RemoveClient/UpdateClient*` `ns_ctx.go:332-533`, `client_ctx.go:60-66`, "
     "`rpc_base_cmds.go:350-406`"),
    ("Transport tables", ["emurx_flow_add", "emurx_flow_remove", "emurx_server_add", "emurx_server_remove",
                          "emurx_client_set_transport"],
     "`TransportCtx` maps `transport/client_ctx.go:490-497`"),
    ("Table shipment and diagnostics", ["emurx_sync", "emurx_table_stats", "emurx_image_lookup", "emurx_image_check"],
     "(device image of the maps above)"),
    ("Mid-batch mutations", ["emurx_table_gen", "emurx_recs_stale"], "DESIGN.md §2.2, `dhcp.go:718`"),
    ("Batched ingest (primary)", ["emurx_ingest_buffer", "emurx_ingest_submit", "emurx_ingest_wait",
                                  "emurx_ingest_stream", "emurx_zmq_walk_dev"],
     "`VethIFZmq.OnRxStream` over the rx `select` loop's messages, `thread_ctx.go:409-410`, `veth_zmq.go:277-320`"),
    ("Receive path (device-resident; per-message fallback)",
     ["emurx_classify_dev", "emurx_parse_dev", "emurx_rx_stream", "emurx_zmq_descriptors",
      "emurx_hist_to_counters", "emurx_hist_fold"],
     "`HandleRxPacket` `thread_ctx.go:365-375`, `ParsePacket` `parser.go:583-959`, `ParserStats`"),
    ("Several GPUs", ["emurx_set_partition", "emurx_route_dev", "emurx_classify_route_dev", "emurx_parse_route_dev",
                      "emurx_lookup_dev", "emurx_owner_key", "emurx_desc_keys_dev"],
     "`GetNs` `thread_ctx.go:772-784` on the Namespace owner (SURVEY §8e)"),
    ("Exchange (library-owned RCCL communicator)",
     ["emurx_comm_unique_id", "emurx_comm_init", "emurx_comm_init_all", "emurx_comm_destroy", "emurx_comm_info",
      "emurx_comm_library",
      "emurx_group_start", "emurx_group_end", "emurx_exchange_dev"],
     "no Go counterpart: the single goroutine's `MapNsT` (`thread_ctx.go:139,397-419,772-784`) split by owner "
     "(SURVEY §8e)"),
    ("Tx path", ["emurx_tx_checksum_dev", "emurx_tx_zmq_dev"],
     "gopacket checksum updates; `VethIFZmq.Send/FlushTx` `veth_zmq.go:149-200`"),
    ("Measurement", ["emurx_set_timing", "emurx_kernel_times", "emurx_copy_ceiling_dev", "emurx_last_stage",
                     "emurx_last_txz"],
     "(bench.py; `emurx_copy_ceiling_dev` is the measured HBM copy ceiling beside the roofline)"),
]


def declared():
    out = {}
    for i, line in enumerate(HDR.read_text().splitlines(), 1):
        # a declaration starts in column 0 with its return type (comments are indented)
        m = re.match(r"^(?:const\s+)?(?:int|void|u?int\d+_t|size_t|char|emurx_\w+)\b[\s\*]*(emurx_\w+)\s*\(", line)
        if m and m.group(1) not in out:
            out[m.group(1)] = i
    return out


def table():
    dec = declared()
    grouped = {n for _, ns, _ in GROUPS for n in ns}
    missing = sorted(set(dec) - grouped)
    extra = sorted(grouped - set(dec))
    if missing or extra:
        sys.exit(f"ungrouped: {missing}; not declared: {extra}")
    lines = [f"Every function `include/emu_rx.h` declares ({len(dec)}), by group, with the header line that "
             "declares it and the reference code it stands for (`tests/test_abi.py` checks that the library "
             "exports each one; `tools/entry_index.py` regenerates this table).", "",
             "| Group | Entry points (header line) | Reference |", "|---|---|---|"]
    for g, ns, ref in GROUPS:
        lines.append(f"| {g} | " + ", ".join(f"`{n}` ({dec[n]})" for n in ns) + f" | {ref} |")
    return "\n".join(lines) + "\n"


if __name__ == "__main__":
    t = table()
    if "--write" in sys.argv:
        s = DOC.read_text()
        head = s[:s.index("## Entry-point index")]
        DOC.write_text(head + "## Entry-point index\n\n" + t)
    else:
        print(t)
