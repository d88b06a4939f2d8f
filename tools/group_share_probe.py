#!/usr/bin/env python3
"""tests/test_gpu_group.py::test_group_sharing_cus_matches_standalone_engines as a probe: per
replica pick and net, the max |group - standalone| after each of 2 steps (NFSP_LIB selects an
A/B build of libnfsp).   python tools/group_share_probe.py [R] [repeats]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as ge  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    pkg = ge.load_package()
    import torch
    kw = dict(n_lanes=256, rl_capacity=1500, sl_capacity=1000, target_every=7)
    names = [f"a{a}{n}" for a in (0, 1) for n in ("AR", "BR", "TG")]
    for rep in range(reps):
        g = pkg.engine.EngineGroup(R, seed=4242, init_seed=3, **kw)
        picks = (0, R // 2, R - 1)
        solo = {r: pkg.engine.SelfPlayEngine(seed=4242 + r, init_seed=3 + r, **kw) for r in picks}
        for step in range(2):
            g.step()
            for e in solo.values():
                e.step()
            torch.cuda.synchronize()
            for r in picks:
                d = [float(np.abs(g.replicas[r].get_weights(a, n) - solo[r].get_weights(a, n)).max())
                     for a in (0, 1) for n in (0, 1, 2)]
                print(f"{os.path.basename(os.environ.get('NFSP_LIB', 'libnfsp.so'))} rep {rep} R {R} step {step} "
                      f"replica {r}: " + " ".join(f"{k}={v:.2g}" for k, v in zip(names, d)), flush=True)
        g.close()


if __name__ == "__main__":
    main()
