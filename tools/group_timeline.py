#!/usr/bin/env python3
"""Where a group step's time goes (HIP events per stream, nfsp_group_get_timings): one engine
group in a bench.py group configuration (default c4_emul_r8: C4's arithmetic on one GPU),
`steps` steps after `warmup`, ms per step of the rollout kernels, the prep, the targets, the
chain launches and the two learner streams' spans.

    python tools/group_timeline.py [config] [warmup] [steps]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import bench          # first: it sets GPU_MAX_HW_QUEUES (8) before anything initialises HIP
    import torch
    pkg = __import__("__graft_entry__").load_package()
    name = sys.argv[1] if len(sys.argv) > 1 else "c4_emul_r8"
    warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    cfg = bench.CONFIGS[name]
    R = cfg["replicas"]
    extra = {k: cfg[k] for k in ("slices", "slice_lag") if k in cfg}
    g = pkg.engine.EngineGroup(R, n_lanes=cfg["n_lanes"] // R, rl_capacity=cfg["rl_capacity"],
                               sl_capacity=cfg["sl_capacity"], seed=1234, init_seed=0,
                               avg_ar=not cfg.get("xchg_every"), **extra)
    if cfg.get("sched"):
        g.set_sched(**cfg["sched"])
    if cfg.get("xchg_every"):
        g.set_exchange(pkg.native.XCHG_AR, every=cfg["xchg_every"], scale=cfg["xchg_gain"] / R)
        g.average_ar()
    for _ in range(warmup):
        g.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.step()
    torch.cuda.synchronize()
    plain = (time.perf_counter() - t0) / steps * 1e3
    g.set_timing(True)
    g.timings()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.step()
    torch.cuda.synchronize()
    timed = (time.perf_counter() - t0) / steps * 1e3
    tm = g.timings()
    out = {"config": name, "replicas": R, "ms_per_step": plain, "ms_per_step_event_timed": timed,
           "per_step": {k: {"ms": v[0] / steps, "launches": v[1] / steps} for k, v in tm.items()},
           "note": "group timings sum the replicas' rollout / prep marks; chain and stream spans are the "
                   "group's shared launches (kept on replica 0); br_stream_a0 = the group's one BR stream"}
    print(json.dumps(out))
    g.close()


if __name__ == "__main__":
    main()
