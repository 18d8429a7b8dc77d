#!/bin/bash
# Kernel trace of tools/krx_kinds.py (config D, 2M frames): the start / end of every k_owner_count,
# k_route_scan and k_rx<2> of the parse_route calls, and the gaps between them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/gaps; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/p -o run -- python tools/krx_kinds.py > $out/kinds.log 2>&1 || exit $?
f=$(ls $out/p/*/run_kernel_trace.csv $out/p/run_kernel_trace.csv 2>/dev/null | head -n 1)
python - "$f" <<'PY' | tee $out/gaps.txt
import csv, sys, statistics as S
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r.get("Kernel_Name", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
rows.sort()
g1, g2, d_oc, d_sc, d_rx, span = [], [], [], [], [], []
for i in range(len(rows) - 2):
    a, b, c = rows[i], rows[i + 1], rows[i + 2]
    if "k_owner_count" in a[2] and "k_route_scan" in b[2] and "k_rx<2" in c[2]:
        g1.append((b[0] - a[1]) / 1e3); g2.append((c[0] - b[1]) / 1e3)
        d_oc.append((a[1] - a[0]) / 1e3); d_sc.append((b[1] - b[0]) / 1e3); d_rx.append((c[1] - c[0]) / 1e3)
        span.append((c[1] - a[0]) / 1e3)
m = lambda x: round(S.median(x), 2) if x else None
print({"calls": len(g1), "owner_count_us": m(d_oc), "gap1_us": m(g1), "scan_us": m(d_sc), "gap2_us": m(g2),
       "k_rx2_us": m(d_rx), "span_us": m(span)})
PY
rm -rf $out/p
