#!/usr/bin/env python3
"""The learner work of C4's 8 ranks, step by step, from the on-device emulation of the rank
path (an engine group of 8 replicas with bench.CONFIGS["c4"]'s slices, lag and per-slice AR
exchange, as tests/test_gpu_slices.py::test_c4_emulated_learns_within_the_cpu_seed_band runs it).

A rank's step is bound by its longest chain (the AR chain of its busier agent, or that agent's
BR stream), so its time follows the updates of its busier agent.  The ranks exchange the AR
nets after every slice, so the job runs at the pace of the slowest rank: lockstep efficiency
per step ~ mean over ranks / max over ranks of the busier agent's updates (a lower bound on
the loss: the per-slice maxima add the slices' own spread).

    python tools/c4_rank_spread.py [steps] [seed] > profiles/r04_c4_rank_spread.json
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    s = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    import bench
    import __graft_entry__ as ge
    pkg = ge.load_package()
    c4 = bench.CONFIGS["c4"]
    R = 8
    g = pkg.engine.EngineGroup(R, n_lanes=c4["n_lanes"], rl_capacity=c4["rl_capacity"],
                               sl_capacity=c4["sl_capacity"], seed=1234 + 1000 * s, init_seed=1000 * s,
                               slices=c4["slices"], slice_lag=2)
    g.set_exchange(pkg.native.XCHG_AR, every=c4["xchg_every"], scale=c4["xchg_gain"] / R)
    g.average_ar()
    prev = g.stats()["replicas"]
    rows = []
    for k in range(1, steps + 1):
        g.step()
        cur = g.stats()["replicas"]
        ar = np.array([[c["ar_updates"][a] - p["ar_updates"][a] for a in (0, 1)] for p, c in zip(prev, cur)])
        br = np.array([[c["br_updates"][a] - p["br_updates"][a] for a in (0, 1)] for p, c in zip(prev, cur)])
        busy = np.maximum(ar.max(axis=1), br.max(axis=1))          # the busier agent's updates
        rows.append({"step": k, "ar_updates": ar.tolist(), "br_updates": br.tolist(),
                     "busier_agent_updates": busy.tolist(),
                     "lockstep_efficiency_bound": float(busy.mean() / busy.max()),
                     "spread_max_over_min": float(busy.max() / busy.min())})
        prev = cur
        print(f"step {k}: busier-agent updates per rank {busy.tolist()}  mean/max {busy.mean() / busy.max():.4f}",
              file=sys.stderr, flush=True)
    g.close()
    print(json.dumps({"source": "tools/c4_rank_spread.py (engine group of 8, bench.CONFIGS['c4'], seed "
                      f"{s})", "steps": rows,
                      "lockstep_efficiency_bound_mean": float(np.mean([r["lockstep_efficiency_bound"] for r in rows]))},
                     indent=1))


if __name__ == "__main__":
    main()
