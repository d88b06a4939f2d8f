"""The AR chain in the saturated-softmax regime.

The AR chain (csrc/chain3.h, k_chain3<0>) takes Keras' re-normalisation of the softmax,
p = y / sum(y), as p = y (sum(y) is 1 within a few ulps) and its exp / reciprocal from
v_exp_f32 / v_rcp_f32, so near Keras' clip bounds [1e-7, 1 - 1e-7] (keras categorical
cross-entropy, agent/agent.py:109-116 compiled with it, fitted at agent/agent.py:255-264) a
sample's clip decision can differ from the oracle's (oracle/nn_oracle.py: normalise, clip,
mask).  Round 3 measured the chain against the f32 reference chain with the layer-2 weights
scaled x60 (most outputs clipped): 4e-6 after one update, 0.2-3 after 5-200
(profiles/r03_chain_ar_saturated_compare.txt).  This test pins that regime on the engine
itself against the oracle:

* an engine whose AR nets' layer 2 is scaled x60 before a learner call (saturated softmax on
  most observations), stopped after k updates (nfsp_engine_set_update_limit) for every k;
* resynchronised replay: update k replayed by the oracle from the ENGINE's weights after k
  updates, compared with the engine after k + 1.  Bar: every single update agrees within 1e-5
  (relative to max(1, |w|)), although nearly every one has a p within 4e-7 (relative; ~3 ulps
  at 1 - 1e-7) of a clip bound -- the regime is the saturated one (measured: <= 2.1e-7);
* free replay (no resynchronisation): every onset of a > 1e-4 divergence lies in an update
  with a p within 4e-7 (relative) of a clip bound -- a clip-mask flip -- or a hidden
  pre-activation within 1e-7 of zero (the ReLU kink of test_gpu_learner_divergence.py).
The -s output of a run is kept as profiles/r04_learner_saturated.txt."""
import numpy as np
import pytest
import torch

import learner_oracle as LO
from test_gpu_configs import _oracle_cfg, _snapshot
from test_gpu_learner_divergence import _replay

pytestmark = pytest.mark.gpu

CFG = dict(n_lanes=16_384, rl_capacity=40_000, sl_capacity=40_000)
OW2 = 30 * 64 + 64             # packed W1 | b1 | W2 | b2: layer 2 starts here
SCALE = 60.0
NU = 40                        # updates replayed one by one, per agent
REL = 4e-7


def _engine_after(pkg, k):
    eng = pkg.engine.SelfPlayEngine(seed=3131, init_seed=8, **CFG)
    for _ in range(3):
        eng.step()
    for a in (0, 1):           # saturate the AR softmax: layer 2 x 60
        w = eng.get_weights(a, 0)
        w[OW2:] *= np.float32(SCALE)
        eng.set_weights(a, 0, w)
    eng.rollout()
    if k > 0:
        eng.set_update_limit(k)
        eng.update()
    torch.cuda.synchronize()
    return eng


def _rel(a, b):
    return float((np.abs(a - b) / np.maximum(1.0, np.abs(b))).max())


def test_saturated_ar_single_updates_agree_and_divergence_starts_at_clip_flips(pkg):
    eng0 = _engine_after(pkg, 0)
    st0, state = _snapshot(eng0)
    cfg = _oracle_cfg(eng0.cfg)
    quirks = eng0.cfg.quirks
    del eng0
    mbs = [list(LO.ar_minibatches(cfg, state, a, quirks)) for a in (0, 1)]
    n = min(NU, min(len(m) for m in mbs))
    assert n >= 20
    w_at = {0: [state[a]["w"][0] for a in (0, 1)]}
    for k in range(1, n + 1):
        e = _engine_after(pkg, k)
        w_at[k] = [e.get_weights(a, 0) for a in (0, 1)]
        del e
        torch.cuda.empty_cache()
    sat = []
    resync, flips = [], []
    for a in (0, 1):
        for k in range(n):
            closest = {}
            w_or, amb = _replay(cfg, mbs[a], k, k + 1, w_at[k][a], cfg["lr_ar"], rel=REL, closest=closest)
            d = _rel(w_or, w_at[k + 1][a])
            resync.append((a, k, d, closest.get(mbs[a][k][0], np.inf), bool(amb)))
            if d > 1e-5:
                flips.append((a, k, d))
        # the free replay from the start
        w = w_at[0][a]
        prev = 0.0
        for k in range(n):
            rc, closest = {}, {}
            w, amb = _replay(cfg, mbs[a], k, k + 1, w, cfg["lr_ar"], rel=REL, closest=closest, relu_closest=rc)
            d = _rel(w, w_at[k + 1][a])
            z = min(rc.values(), default=np.inf)
            if d > 1e-4 and prev <= 1e-4:               # an onset
                assert amb or z <= 1e-7, ("free replay left the engine with no clip flip or ReLU kink",
                                          a, k, d, min(closest.values(), default=np.inf), z)
                sat.append((a, k, d, "clip" if amb else "relu"))
            prev = d
    print("resynchronised single updates: agent, update, max rel |oracle - engine|, closest p to a clip "
          "bound (relative), ambiguous:", [(a, k, f"{d:.1e}", f"{c:.1e}", m) for a, k, d, c, m in resync])
    print("free-replay divergence onsets (agent, update, rel diff, cause):", sat)
    assert not flips, ("single updates past 1e-5", flips)
    # the regime is the saturated one: outputs at the clip bounds are common
    near = [c for _, _, _, c, _ in resync]
    assert min(near) < 1e-3
