"""One-line summaries of bench.py JSON lines (the last JSON line of each log given)."""
import json
import sys

for f in sys.argv[1:]:
    lines = [x for x in open(f).read().splitlines() if x.startswith("{")]
    if not lines:
        print(f, "no JSON line")
        continue
    d = json.loads(lines[-1])
    r = d.get("roofline", {})
    print(f"{f}: value {d['value']} ms/step {d['ms_per_step']} k_rx {r.get('kernel_ms_mean')} frac {r.get('frac')}")
    blocks = [("", d)] + [(k, d[k]) for k in ("namespace_exchange", "alternative") if isinstance(d.get(k), dict)]
    for name, b in blocks:
        e = b.get("exchange")
        if not e:
            continue
        ph = e.get("phases") or {}
        print(f"  {name or 'exchange'}: value {b.get('value')} step_dev {e.get('step_device_ms_mean')} "
              f"k_rx {ph.get('k_rx_ms')} oc {ph.get('owner_count_scan_ms')} look {ph.get('owner_lookup_ms')} "
              f"a2a {ph.get('all_to_all_ms')} B/frame {ph.get('bytes_per_frame_to_other_ranks')} "
              f"pipe {(e.get('pipelined') or {}).get('value')} one {(e.get('one_stream_steps') or {}).get('value')} "
              f"key {(e.get('key_derivation') or {}).get('key_ms')} nokey {(e.get('without_key_derivation') or {}).get('value')}")
    if "host_inclusive" in d:
        h = d["host_inclusive"]
        print(f"  host_inclusive: copy {h.get('with_host_copy')} prefilled {h.get('prefilled')}")
