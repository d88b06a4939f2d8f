#!/usr/bin/env python3
"""The cost of C4's per-slice lockstep, from the on-device emulation of the rank path (an engine
group of 8 replicas with bench.CONFIGS["c4"]'s slices, lag and per-slice AR exchange, as
tests/test_gpu_slices.py::test_c4_emulated_learns_within_the_cpu_seed_band runs it), with the
learner plans traced per slice (nfsp_group_set_trace).

A rank's AR chain launch of slice k runs both agents' AR chains at once, so it takes
~ 8 x max_a U_AR[r, a, k] SGD steps x the AR step; the exchange after it waits for every
rank's, so the AR stream of every rank runs sum_k max_r (that).  The BR streams never wait
for another rank.  Per step the model gives, in ms (AR / BR step times of the final chain,
plus the BR stream's per-step overhead of targets and launches measured in C3):
  independent[r] = max(AR_r, BR_r)            (each rank alone; C3's situation)
  lockstep_step  = max_r independent[r]       (ranks meeting once per step)
  lockstep_slice = max(sum_k max_r AR_rk, max_r BR_r)   (the exchange after every slice)
and the efficiency of the job against independent ranks, mean_r independent[r] / lockstep.

    python tools/c4_slice_spread.py [steps] [seed] [warmup] > profiles/r04_c4_slice_spread.json
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

AR_US, BR_US = 0.762, 0.726       # us per SGD step in the engine (profiles/r04_bench_final_pk.json)
BR_OVERHEAD_MS = 5.0              # per step and agent-0 stream: targets + chain launches


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    s = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 2
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
    for _ in range(warm):
        g.step()
    rows = []
    K = c4["slices"]
    for k in range(steps):
        g.set_trace(True)
        g.step()
        t = g.trace()                       # [K][R][agent][AR, BR] update counts
        g.set_trace(False)
        assert t.shape[0] == K, t.shape
        ar = 8 * t[:, :, :, 0].max(axis=2) * AR_US / 1e3          # [K][R] ms of the AR launch
        br = 8 * t[:, :, :, 1].sum(axis=0) * BR_US / 1e3          # [R][agent] ms of BR chains
        br_r = br.max(axis=1) + BR_OVERHEAD_MS                      # [R]
        ar_r = ar.sum(axis=0)                                       # [R]
        indep = np.maximum(ar_r, br_r)
        lock_step = indep.max()
        lock_slice = max(ar.max(axis=1).sum(), br_r.max())
        rows.append({"step": warm + k + 1,
                     "ar_ms_per_rank": [round(float(x), 2) for x in ar_r],
                     "br_ms_per_rank": [round(float(x), 2) for x in br_r],
                     "independent_ms_mean": round(float(indep.mean()), 2),
                     "lockstep_per_step_ms": round(float(lock_step), 2),
                     "lockstep_per_slice_ms": round(float(lock_slice), 2),
                     "eff_per_step": round(float(indep.mean() / lock_step), 4),
                     "eff_per_slice": round(float(indep.mean() / lock_slice), 4),
                     "slice_spread_ar_max_over_mean": round(float((ar.max(axis=1) / ar.mean(axis=1)).mean()), 4)})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    g.close()
    out = {"source": f"tools/c4_slice_spread.py {steps} {s} {warm} (engine group of 8, bench.CONFIGS['c4'], "
                     f"per-slice plans traced; AR {AR_US} / BR {BR_US} us per SGD step, BR overhead "
                     f"{BR_OVERHEAD_MS} ms per step)",
           "steps": rows,
           "eff_per_step_mean": round(float(np.mean([r["eff_per_step"] for r in rows])), 4),
           "eff_per_slice_mean": round(float(np.mean([r["eff_per_slice"] for r in rows])), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
