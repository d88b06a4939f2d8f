#!/usr/bin/env python3
"""C4's arithmetic on one GPU over more seeds than its gate runs (tests/test_gpu_slices.py::
test_c4_emulated_learns_within_the_cpu_seed_band: seeds 0..7): 8 replicas x 1,048,576 lanes in
128 pipelined slices, the AR nets exchanged after every slice (W0 + 2 x mean delta, bench
CONFIGS["c4"]), exact exploitability of replica 0's AR nets at 1 / 2 / 3 / 4 / 8 steps
(8.4 / 16.8 / 25.2 / 33.5 / 67M total hands), against the CPU reference's 24-seed band.

    python tests/studies/c4_gate_seeds.py --seeds 8 24 > profiles/r06/c4_gate_seeds8_23.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs=2, default=[8, 24], help="seed range [a, b)")
    args = ap.parse_args()
    import torch
    import bench
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    c4 = bench.CONFIGS["c4"]
    R, lanes, K = 8, c4["n_lanes"], c4["slices"]
    checkpoints = (1, 2, 3, 4, 8)
    curves = {}
    t0 = time.time()
    for s in range(*args.seeds):
        g = pkg.engine.EngineGroup(R, n_lanes=lanes, rl_capacity=c4["rl_capacity"], sl_capacity=c4["sl_capacity"],
                                   seed=1234 + 1000 * s, init_seed=1000 * s, slices=K, slice_lag=2)
        g.set_exchange(pkg.native.XCHG_AR, every=c4["xchg_every"], scale=c4["xchg_gain"] / R)
        g.average_ar()
        c = []
        for k in range(1, checkpoints[-1] + 1):
            g.step()
            if k in checkpoints:
                c.append((k * R * lanes, g.exploitability(0)["exploitability"]))
        curves[s] = c
        g.close()
        del g
        torch.cuda.empty_cache()
        print(f"seed {s} done at {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    with open(os.path.join(REPO, "tests", "golden", "cpu_band_c3mem_24.json")) as f:
        cpu = {int(h): np.array(v) for h, v in json.load(f)["curves_by_hands"].items()}
    last = max(cpu)
    report = []
    for i, k in enumerate(checkpoints):
        h = k * R * lanes
        xs = np.array([curves[s][i][1] for s in curves])
        near = min(cpu, key=lambda x: abs(x - min(h, last)))
        cm, cs = float(cpu[near].mean()), float(cpu[near].std())
        report.append({"hands": h, "cpu_checkpoint": near, "cpu_mean": cm, "cpu_std": cs,
                       "gpu_mean": float(xs.mean()), "gpu_std": float(xs.std()),
                       "margin_to_1sigma_bar": cm + cs - float(xs.mean())})
    print(json.dumps({"config": "c4 emulated (bench CONFIGS['c4'], 8 replicas)", "seeds": list(curves),
                      "curves": {str(s): c for s, c in curves.items()}, "report": report,
                      "wall_s": time.time() - t0}))


if __name__ == "__main__":
    main()
