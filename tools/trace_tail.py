#!/usr/bin/env python3
"""Average duration of a kernel's LAST n launches in a rocprofv3 kernel trace -- the launches
of bench.py's event-timed pass (its last K steps), which is what `kernel_ms` averages.  The
--stats summary averages every launch of the process, warmup steps included.

    python tools/trace_tail.py gpurun_out/prof/c3_kernel_trace.csv 80 'k_chain3<0, 0, 0>' \\
        1553 'k_chain3<1, 0, 0>' > profiles/r03_c3_trace_tail.json
"""
import csv
import json
import sys


def main():
    path = sys.argv[1]
    pairs = list(zip(sys.argv[2::2], sys.argv[3::2]))
    rows = {sub: [] for _, sub in pairs}
    with open(path) as f:
        for r in csv.DictReader(f):
            for sub in rows:
                if sub in r["Kernel_Name"]:
                    rows[sub].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = {"source": path, "kernels": {}}
    for n, sub in pairs:
        d = sorted(rows[sub])[-int(n):]
        ms = [(e - s) * 1e-6 for s, e in d]
        out["kernels"][sub] = {"last_launches": len(ms), "avg_ms": sum(ms) / max(len(ms), 1),
                               "all_launches": len(rows[sub]),
                               "all_avg_ms": sum((e - s) * 1e-6 for s, e in rows[sub]) / max(len(rows[sub]), 1)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
