#!/usr/bin/env python3
"""BR-stream accounting from a rocprofv3 kernel trace of bench.py (tools/trace_c3.sh): per
agent stream, over the un-instrumented timed pass (the middle of the trace), chain launches per
step, their excess over n x 8 SGD steps (n from the preceding k_br_targets' grid), and the
launches that overlapped a k_rollout on the ctx stream.

    python tools/br_stream_excess.py gpurun_out/trace/c3_kernel_trace.csv [us_per_step] [ms_per_step]
"""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    us = float(sys.argv[2]) if len(sys.argv) > 2 else 0.8315
    step_ms = float(sys.argv[3]) if len(sys.argv) > 3 else 168.0
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"] = int(r["Start_Timestamp"])
        r["e"] = int(r["End_Timestamp"])
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        r["k"] = m.group(1) if m else r["Kernel_Name"][:25]
    rows.sort(key=lambda r: r["s"])
    ctx = [r for r in rows if r["Stream_Id"] == "0"]
    roll = [(r["s"], r["e"]) for r in ctx if r["k"] == "k_rollout"]
    for sid in ("1", "2"):
        st = [r for r in rows if r["Stream_Id"] == sid]
        n = len(st)
        seg = st[int(n * 0.27):int(n * 0.60)]
        steps = (seg[-1]["e"] - seg[0]["s"]) / 1e6 / step_ms
        ex, ov = [], 0
        for a, b in zip(seg, seg[1:]):
            if a["k"] == "k_br_targets" and b["k"] == "k_chain3":
                nn = int(a["Grid_Size_X"]) // 256
                x = (b["e"] - b["s"]) / 1e3 - nn * 8 * us
                ex.append(x)
                if x > 30 and any(s < b["s"] + x * 1e3 and e > b["s"] for s, e in roll):
                    ov += 1
        big = [x for x in ex if x > 30]
        tg = sum((r["e"] - r["s"]) for r in seg if r["k"] == "k_br_targets") / 1e6
        print(f"stream {sid}: {len(ex) / steps:.1f} chain launches/step, excess {sum(ex) / steps / 1e3:.2f} ms/step "
              f"({len(big) / steps:.1f} launches/step > 30 us: {sum(big) / steps / 1e3:.2f} ms, {ov} of {len(big)} "
              f"beside a k_rollout); k_br_targets {tg / steps:.2f} ms/step")


if __name__ == "__main__":
    main()
