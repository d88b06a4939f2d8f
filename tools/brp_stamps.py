#!/usr/bin/env python3
"""Where k_br_persist's time goes (diagnostic build): per chain workgroup the cycles waiting for
targets vs running pieces and the SGD steps; per helper the cycles waiting for queue slots vs
writing targets and the items.  Build and run:

    python tools/build_lib_variant.py brpst -DNFSP_BRP_STAMPS=1
    NFSP_LIB=tools/bin/libnfsp_brpst.so python tools/brp_stamps.py [config] [steps]
"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import bench
    import numpy as np
    import torch
    pkg = __import__("__graft_entry__").load_package()
    name = sys.argv[1] if len(sys.argv) > 1 else "c4_emul_r8_persist"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    cfg = bench.CONFIGS[name]
    R = cfg["replicas"]
    g = pkg.engine.EngineGroup(R, n_lanes=cfg["n_lanes"] // R, rl_capacity=cfg["rl_capacity"],
                               sl_capacity=cfg["sl_capacity"], seed=1234, init_seed=0,
                               slices=cfg.get("slices", 1), slice_lag=cfg.get("slice_lag", 1))
    g.set_sched(**cfg.get("sched", {"br_persist": 1}))
    if cfg.get("xchg_every"):
        g.set_exchange(pkg.native.XCHG_AR, every=cfg["xchg_every"], scale=cfg["xchg_gain"] / R)
        g.average_ar()
    lib = C.CDLL(pkg.native.LIB_PATH)
    buf = (C.c_ulonglong * (2 * 64 * 4))()
    g.step()
    g.check()
    lib.nfsp_debug_brp_stamps(buf, 1)
    for _ in range(steps):
        g.step()
    g.check()
    lib.nfsp_debug_brp_stamps(buf, 1)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(2, 64, 4).astype(np.float64)
    ch, he = a[0], a[1]
    used = ch[:, 2] > 0
    hu = he[:, 2] > 0
    out = {"config": name, "steps": steps, "chains": int(used.sum()), "helpers": int(hu.sum()),
           "chain_wait_cycles_per_step": (ch[used, 0] / steps).round().tolist(),
           "chain_run_cycles_per_step": (ch[used, 1] / steps).round().tolist(),
           "chain_sgd_steps_per_step": (ch[used, 2] / steps).round().tolist(),
           "chain_cycles_per_sgd_step": (ch[used, 1] / ch[used, 2]).round(1).tolist(),
           "chain_pieces_per_step": (ch[used, 3] / steps).round().tolist(),
           "helper_wait_cycles_per_step_mean": float(he[hu, 0].mean() / steps),
           "helper_work_cycles_per_step_mean": float(he[hu, 1].mean() / steps),
           "helper_items_per_step_mean": float(he[hu, 2].mean() / steps),
           "helper_cycles_per_item": float(he[hu, 1].sum() / max(he[hu, 2].sum(), 1))}
    print(json.dumps(out))
    g.close()


if __name__ == "__main__":
    main()
