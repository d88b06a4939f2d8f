#!/usr/bin/env python3
"""Per-kernel HBM bytes per launch from two rocprofv3 --pmc passes -> profiles/pmc_<cfg>.json.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof -o pmc_fetch -- python3 bench.py --no-cpu
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof -o pmc_write -- python3 bench.py --no-cpu
    python tools/pmc_summary.py gpurun_out/prof c3 > profiles/pmc_c3.json

FETCH_SIZE / WRITE_SIZE are KB per dispatch.  MI355X_MICROARCH.md (HBM): on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read, so
hbm_bytes_per_launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024.
"""
import csv
import json
import sys
from collections import defaultdict

# bench.py kernel label -> substring of the rocprof kernel name
KERNELS = {
    "k_chain3_br": "k_chain3<1, 0, 0>",     # the one-engine instantiations (TABLE = 0)
    "k_chain3_ar": "k_chain3<0, 0, 0>",
    "k_rollout": "k_rollout(",
    "k_commit": "k_commit(",
    "k_br_targets": "k_br_targets(",
    "k_br_prep": "k_br_prep(",
    "k_ar_prep": "k_ar_prep(",
    "k_scan1": "k_scan1(",
    "k_scan2": "k_scan2(",
}


def per_kernel(path):
    vals = defaultdict(list)
    names = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            for label, sub in KERNELS.items():
                if sub in row["Kernel_Name"]:
                    vals[label].append(float(row["Counter_Value"]))
                    names[label] = row["Kernel_Name"]
    return vals, names


def main():
    d, cfg = sys.argv[1], sys.argv[2]
    fetch, names = per_kernel(f"{d}/pmc_fetch_counter_collection.csv")
    write, _ = per_kernel(f"{d}/pmc_write_counter_collection.csv")
    out = {"command": "rocprofv3 --pmc FETCH_SIZE (pass 1) / --pmc WRITE_SIZE (pass 2) -- "
                      "python3 bench.py --no-cpu --config " + cfg,
           "units": "FETCH_SIZE/WRITE_SIZE in KB per launch (rocprofv3); hbm_bytes_per_launch = "
                    "(2 x FETCH_SIZE + WRITE_SIZE) x 1024 (MI355X_MICROARCH.md: gfx950 FETCH_SIZE "
                    "counts half the bytes of wide coalesced reads)",
           "kernels": {}}
    for label in KERNELS:
        if not fetch.get(label) or not write.get(label):
            continue
        fk = sum(fetch[label]) / len(fetch[label])
        wk = sum(write[label]) / len(write[label])
        out["kernels"][label] = {"rocprof_name": names[label], "launches": len(fetch[label]),
                                 "fetch_kb": fk, "write_kb": wk,
                                 "hbm_bytes_per_launch": (2 * fk + wk) * 1024}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
