#!/usr/bin/env python3
"""Cost of the per-launch HIP timing events on a C3 engine step (diagnostic).

Times K engine steps with nfsp_engine_set_timing off, then on, then off again, on one engine.
    python tools/timing_cost.py [--steps K] [--lanes N]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--lanes", type=int, default=1_048_576)
    args = ap.parse_args()
    import torch
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    eng = pkg.engine.SelfPlayEngine(n_lanes=args.lanes, rl_capacity=200_000, sl_capacity=2_000_000,
                                    seed=1234, init_seed=0)
    for _ in range(2):
        eng.step()
    torch.cuda.synchronize()
    out = {}
    for tag, on in (("off", False), ("on", True), ("off2", False)):
        eng.set_timing(on)
        eng.timings()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            eng.step()
        torch.cuda.synchronize()
        out[tag] = (time.perf_counter() - t0) / args.steps * 1e3
        print(tag, round(out[tag], 3), "ms/step", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
