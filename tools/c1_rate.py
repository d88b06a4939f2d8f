#!/usr/bin/env python3
"""C1 (BASELINE.json configs[0]: one Leduc env, two NFSP agents, main.train) on the GPU, two
ways, hands per second (diagnostic):
  dropin  the reference's own driver loop over the drop-in Env / Agent (selfplay.train:
          one hand at a time, every decision a libnfsp call from Python);
  engine  the batched engine at n_lanes = 1 (one hand per nfsp_engine_step).
    python tools/c1_rate.py [--seconds 20]
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
    ap.add_argument("--seconds", type=float, default=20.0)
    args = ap.parse_args()
    import random
    import torch
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    out = {}
    random.seed(0)
    env, p1, p2 = pkg.selfplay.make_main(init_seed=0)
    pkg.selfplay.train(env, p1, p2, episodes=200)          # warm-up: past the first updates
    hands, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.seconds:
        pkg.selfplay.train(env, p1, p2, episodes=200)
        hands += 200
    out["dropin_hands_per_s"] = hands / (time.perf_counter() - t0)
    print(json.dumps(out), flush=True)
    eng = pkg.engine.SelfPlayEngine(n_lanes=1, rl_capacity=40_000, sl_capacity=40_000, seed=1)
    for _ in range(300):
        eng.step()
    torch.cuda.synchronize()
    hands, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.seconds:
        for _ in range(500):
            eng.step()
        torch.cuda.synchronize()
        hands += 500
    out["engine_1lane_hands_per_s"] = hands / (time.perf_counter() - t0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
