#!/usr/bin/env python3
"""Per engine step, from a rocprofv3 --kernel-trace CSV: when the learner's streams start and
end relative to the step's rollout (the critical-path view of DESIGN §4).
    python tools/step_timeline.py gpurun_out/prof/c3_kernel_trace.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]) for r in rows)
roll = [k for k in ks if "k_rollout" in k[2]]
for i, r in enumerate(roll):
    t0 = r[0]
    t1 = roll[i + 1][0] if i + 1 < len(roll) else 1 << 62
    seg = [k for k in ks if t0 <= k[0] < t1]
    by = collections.defaultdict(list)
    for k in seg:
        by[k[3]].append(k)
    parts = []
    for sid in sorted(by):
        v = by[sid]
        names = collections.Counter(x[2].split("(")[0].split("::")[-1][:18] for x in v)
        busy = sum(x[1] - x[0] for x in v)
        parts.append(f"s{sid}[{(v[0][0] - t0) / 1e6:.1f}..{(v[-1][1] - t0) / 1e6:.1f} ms, n={len(v)}, "
                     f"busy {busy / 1e6:.1f}]")
    end = max(k[1] for k in seg)
    print(f"step {i}: end {(end - t0) / 1e6:.1f} ms  " + "  ".join(parts))
