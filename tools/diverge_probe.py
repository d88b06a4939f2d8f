#!/usr/bin/env python3
"""Where does a long learner call leave the oracle?  Replays one C2 learner call with the
oracle, tracing every update, and runs the engine (deterministically re-created) with
nfsp_engine_set_update_limit(k) for several k: max |engine - oracle| per net vs k."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import learner_oracle as LO  # noqa: E402
from test_gpu_configs import C2, _oracle_cfg, _snapshot  # noqa: E402


def engine_at(pkg, k):
    eng = pkg.engine.SelfPlayEngine(seed=2024, init_seed=3, **C2)
    for _ in range(6):
        eng.step()
    eng.rollout()
    st, state = _snapshot(eng)
    if k is not None:
        eng.set_update_limit(k)
    eng.update()
    torch.cuda.synchronize()
    return eng, state


def main():
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    e0, state = engine_at(pkg, None)
    tr = {}
    LO.learner_step(_oracle_cfg(e0.cfg), state,
                    trace=lambda a, n, u, w: tr.__setitem__((a, n, u), w))
    out = []
    for k in (1, 2, 5, 10, 25, 50, 100, 200, 300, 400, 500):
        eng, _ = engine_at(pkg, k)
        row = {"k": k}
        for a in (0, 1):
            for n in (0, 1):
                key = (a, n, k - 1)
                if key in tr:
                    d = np.abs(eng.get_weights(a, n) - tr[key])
                    row[f"a{a}n{n}"] = [float(d.max()), float(np.median(d))]
        out.append(row)
        print(json.dumps(row), flush=True)




def detail():
    """The full call: which weights of each net are off, and the nets' outputs."""
    import nn_oracle as nn
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    eng, state = engine_at(pkg, None)
    want = LO.learner_step(_oracle_cfg(eng.cfg), state)
    obs = np.unique(np.concatenate([state[a]["rl_s2_bits"] for a in (0, 1)]))
    x = LO.bits_to_x(obs)
    for a in (0, 1):
        for n in (0, 1, 2):
            got, exp = eng.get_weights(a, n), want[a]["w"][n]
            d = np.abs(got - exp)
            w1 = d[:30 * 64].reshape(30, 64)
            act = nn.ACT_SOFTMAX if n == 0 else nn.ACT_RELU
            y0 = nn.MLP(act, 64, weights=nn.unpack_weights(got)).predict(x)
            y1 = nn.MLP(act, 64, weights=nn.unpack_weights(exp)).predict(x)
            print(json.dumps({"a": a, "net": n, "max": float(d.max()), "median": float(np.median(d)),
                              "frac_gt_1e-4": float((d > 1e-4).mean()),
                              "hidden_units_gt_1e-4": np.nonzero(w1.max(axis=0) > 1e-4)[0].tolist(),
                              "out_max": float(np.abs(y0 - y1).max()), "n_obs": int(len(obs))}), flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "detail":
    detail()
    sys.exit(0)


if __name__ == "__main__":
    main()
