#!/usr/bin/env python3
"""Predicted multi-GPU efficiency of the C4 shards from one GPU (diagnostic).

bench.py --gpus N runs one C3 engine per GPU with seeds 1234 + rank, and (with the AR
all-reduce on) synchronises the ranks once per engine step, so each step lasts as long as
its slowest rank.  This runs the ranks' engines one after another on one GPU, records every
step's duration, and reports for N = 1, 2, 4, 8:
  lockstep    = sum over steps of the max over ranks    (AR all-reduce on: bench default)
  independent = max over ranks of the sum over steps    (--ar-allreduce off)
  ideal       = mean over ranks of the sum over steps
as the efficiency ideal / lockstep (and ideal / independent).  The exchange itself (one
17.4 KB all-reduce per step) is not included.

    python tools/scale_predict.py [--ranks 8] [--steps 5] [--warmup 2]
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
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    import numpy as np
    import torch
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    t = np.zeros((args.ranks, args.steps))
    for r in range(args.ranks):
        eng = pkg.engine.SelfPlayEngine(n_lanes=1_048_576, rl_capacity=200_000, sl_capacity=2_000_000,
                                        seed=1234 + r, init_seed=r)
        for _ in range(args.warmup):
            eng.step()
        torch.cuda.synchronize()
        for s in range(args.steps):
            t0 = time.perf_counter()
            eng.step()
            torch.cuda.synchronize()
            t[r, s] = time.perf_counter() - t0
        del eng
        torch.cuda.empty_cache()
        print(f"rank {r}: {t[r].mean() * 1e3:.1f} ms/step", file=sys.stderr, flush=True)
    out = {"ms_per_step": (t * 1e3).round(2).tolist()}
    for n in (1, 2, 4, 8):
        if n > args.ranks:
            break
        x = t[:n]
        lock = x.max(axis=0).sum()
        indep = x.sum(axis=1).max()
        ideal = x.sum(axis=1).mean()
        out[f"n{n}"] = {"eff_lockstep": ideal / lock, "eff_independent": ideal / indep,
                        "hands_per_s_lockstep": n * args.steps * 1_048_576 / lock}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
