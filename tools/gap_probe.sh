#!/bin/bash
# kernel trace of tools/bin/gap_probe, then the median gaps per variant
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/gap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O -o gap -- $R/tools/bin/gap_probe > $O/out.txt 2>&1 || { tail -5 $O/out.txt; exit 1; }
python3 - "$O/gap_kernel_trace.csv" <<'PY'
import csv, sys, statistics as st
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "like" in r["Kernel_Name"]]
for v in range(4):
    seg = rows[v * 400:(v + 1) * 400]
    g1 = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(seg, seg[1:]) if "chainlike" in a["Kernel_Name"]]
    g2 = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(seg, seg[1:]) if "targetslike" in a["Kernel_Name"]]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in seg if "targetslike" in r["Kernel_Name"]]
    print("variant", v, "lds", "16K" if v & 1 else "150K", "spin", "0" if v & 2 else "100us",
          "gap chain->targets %.2f us" % st.median(g1), "gap targets->chain %.2f us" % st.median(g2), "targets dur %.2f us" % st.median(d))
PY
