#!/usr/bin/env python3
"""Generates tests/golden/cpu_band_c3mem.json: the CPU reference's exploitability-vs-hands
seed band at C3's memories (M_RL 200k, M_SL 2M), the bar of tests/test_gpu_slices.py.

CPU side = the reference's main.train (main.py:21-75, one hand at a time, updates inside the
hand loop at agent/agent.py:153-154) restated in C++ (oracle/nfsp_cpu.cpp; pinned hand for hand
to oracle/nfsp_oracle.py by tests/test_cpu_port.py, which is pinned to the reference's own
event log by tests/golden/rollout_trace.npz).  Seed s: CPython/numpy streams seeded 1000 + s,
initial nets from init_seed s -- the GPU side of the test starts from the same nets
(SelfPlayEngine(init_seed=s)).  Every checkpoint is scored by oracle/exploit_oracle.py (exact
exploitability of the two AR nets as softmax mixed strategies, brute force on the CPU; the
GPU evaluator agrees within 1e-5, tests/test_exploit.py).

    python tests/golden/gen_cpu_band.py --seeds 8 --hands 32000000 --every 2000000
    python tests/golden/gen_cpu_band.py --seed0 8 --seeds 16 --out tests/golden/cpu_band_c3mem_s8.json
    python tests/golden/gen_cpu_band.py --merge tests/golden/cpu_band_c3mem.json \
        tests/golden/cpu_band_c3mem_s8.json --out tests/golden/cpu_band_c3mem_24.json

Seeds run on host threads (ctypes releases the GIL).  ~4 min on 8 cores.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "oracle"))

RL_CAP, SL_CAP = 200_000, 2_000_000


def run_seed(s, hands, every, out):
    import cpu_port
    cfg = cpu_port.make_cfg({"seed": 1000 + s}, init_seed=s, rl_capacity=RL_CAP, sl_capacity=SL_CAP)
    g = cpu_port.CpuGame(cfg)
    snaps = [(0, g.weights(0, 0), g.weights(1, 0))]
    done = 0
    while done < hands:
        g.train(every, stats_every=0)
        done += every
        snaps.append((done, g.weights(0, 0), g.weights(1, 0)))
    g.close()
    out[s] = snaps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=8)
    ap.add_argument("--seed0", type=int, default=0, help="first seed (a further sample of seeds)")
    ap.add_argument("--merge", nargs="+", default=None, help="merge band files (their seeds) into --out")
    ap.add_argument("--hands", type=int, default=32_000_000)
    ap.add_argument("--every", type=int, default=2_000_000)
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden", "cpu_band_c3mem.json"))
    args = ap.parse_args()
    if args.merge:
        return merge(args.merge, args.out)
    import exploit_oracle as E
    t0 = time.time()
    snaps = {}
    seeds = list(range(args.seed0, args.seed0 + args.seeds))
    th = [threading.Thread(target=run_seed, args=(s, args.hands, args.every, snaps)) for s in seeds]
    for t in th:
        t.start()
    for t in th:
        t.join()
    curves = {}
    for s in seeds:
        curves[s] = [(h, float(E.exploitability(w0, w1, 0)["exploitability"])) for h, w0, w1 in snaps[s]]
    by_h = {}
    for s in seeds:
        for h, v in curves[s]:
            by_h.setdefault(h, []).append(v)
    out = {"what": "exact exploitability (softmax mixed, chips) of main.train's AR nets vs hands, "
                   "C++ restatement of the reference (oracle/nfsp_cpu.cpp), C3 memories",
           "generator": "tests/golden/gen_cpu_band.py", "rl_capacity": RL_CAP, "sl_capacity": SL_CAP,
           "seeds": seeds, "cpu_seed": "1000 + s", "init_seed": "s",
           "curves_by_hands": {str(h): v for h, v in sorted(by_h.items())},
           "band": {str(h): [float(np.mean(v)), float(np.std(v))] for h, v in sorted(by_h.items())},
           "wall_s": round(time.time() - t0, 1)}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["band"]))


def merge(paths, out_path):
    """One band over the seeds of several band files (same memories, same checkpoints)."""
    ds = [json.load(open(p)) for p in paths]
    seeds, by_h = [], {}
    for d in ds:
        assert (d["rl_capacity"], d["sl_capacity"]) == (ds[0]["rl_capacity"], ds[0]["sl_capacity"])
        assert not set(seeds) & set(d["seeds"]), "overlapping seeds"
        seeds += d["seeds"]
        for h, v in d["curves_by_hands"].items():
            by_h.setdefault(h, []).extend(v)
    assert all(len(v) == len(seeds) for v in by_h.values())
    out = dict(ds[0], seeds=seeds, merged_from=[os.path.relpath(p, REPO) for p in paths],
               curves_by_hands=by_h, band={h: [float(np.mean(v)), float(np.std(v))] for h, v in by_h.items()},
               wall_s=sum(d["wall_s"] for d in ds))
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["band"]))


if __name__ == "__main__":
    main()
