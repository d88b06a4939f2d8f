"""Pins the cause of the whole-C2-call divergence (test_gpu_configs.py).

A whole C2 learner call (~700 AR updates per agent, M_SL full) leaves one AR net ~4e-3 away
from the oracle's replay, while every prefix the parity tests replay agrees within 1e-4.
Round 2 attributed it to Keras' cross-entropy clip mask on a saturated softmax.  This test
measures it instead, and the clip mask is NOT the cause: no normalised output comes closer
than 1.2e-3 (relative) to a clip bound anywhere in the call.  The cause is the ReLU's kink:
hidden pre-activations within ~5e-8 of zero, whose sign (and so the ReLU derivative) follows
the summation order -- exact-f32 products summed in the matrix cores' order on the GPU, in
numpy's order in the oracle.

* Resynchronised replay, per agent's AR net, in chunks of CH updates: the oracle replays
  updates [u0, u1) from the ENGINE's weights after u0 updates (the engine re-created
  deterministically and stopped by nfsp_engine_set_update_limit) and is compared with the
  engine after u1 updates.  Bar: every chunk within 1e-5 (measured <= 3.6e-7): update for
  update, the arithmetic agrees.
* Free replay of the whole call (no resynchronisation, as test_gpu_configs compares it),
  with probes on the oracle's fit: per chunk, the smallest |pre-activation| and the closest
  normalised output to a clip bound.  Bar: wherever the free replay first leaves the engine
  by more than 1e-4, the chunk it left in holds a pre-activation within 1e-7 of zero.
"""
import numpy as np
import pytest
import torch

import learner_oracle as LO
import nn_oracle as nn
from test_gpu_configs import C2, _oracle_cfg, _snapshot

pytestmark = pytest.mark.gpu

CH = 64
REL = 4e-7


def _engine_after(pkg, k):
    """The C2 engine of test_gpu_configs._c2_engine (6 steps, then the 7th rollout), then the
    learner call stopped after k updates per chain (k = 0: not run)."""
    eng = pkg.engine.SelfPlayEngine(seed=2024, init_seed=3, **C2)
    for _ in range(6):
        eng.step()
    eng.rollout()
    if k == 0:
        return eng
    eng.set_update_limit(k)
    eng.update()
    torch.cuda.synchronize()
    return eng


def _replay(cfg, mbs, u0, u1, w, lr, rel=REL, closest=None, relu_closest=None):
    """Oracle AR updates [u0, u1) from weights w; returns (weights, set of updates with an
    ambiguous clip decision: some p within a relative `rel` of a clip bound).  `closest`
    (dict): per update, the smallest relative distance of any p to a clip bound."""
    net = nn.MLP(nn.ACT_SOFTMAX, 64, weights=nn.unpack_weights(w))
    amb = set()
    cur = [None]
    lo, hi = float(nn.CE_EPS), 1.0 - float(nn.CE_EPS)

    def probe(p):
        p = np.asarray(p, np.float64)
        r = np.minimum(np.abs(p - hi) / hi, np.abs(p - lo) / lo)
        if closest is not None:
            closest[cur[0]] = min(closest.get(cur[0], np.inf), float(r.min()))
        if (r <= rel).any():
            amb.add(cur[0])
    net.clip_probe = probe

    def rprobe(z):
        if relu_closest is not None:
            relu_closest[cur[0]] = min(relu_closest.get(cur[0], np.inf), float(np.abs(z).min()))
    net.relu_probe = rprobe
    for u, xb, ya, perms in mbs[u0:u1]:
        if xb is None:
            continue
        cur[0] = u
        net.fit(LO.bits_to_x(xb), ya, np.float32(lr), epochs=cfg["epochs"], perms=perms)
    return net.flat(), amb


def test_whole_c2_call_divergence_is_a_relu_kink(pkg):
    eng0 = _engine_after(pkg, 0)
    st0, state = _snapshot(eng0)
    cfg = _oracle_cfg(eng0.cfg)
    quirks = eng0.cfg.quirks
    del eng0
    mbs = [list(LO.ar_minibatches(cfg, state, a, quirks)) for a in (0, 1)]
    U = max(len(m) for m in mbs)
    assert U > 500
    bounds = list(range(0, U, CH)) + [U]
    weights_at = {0: [state[a]["w"][0] for a in (0, 1)]}
    report = []
    ambiguous_total = 0
    for i in range(len(bounds) - 1):
        u0, u1 = bounds[i], bounds[i + 1]
        eng = _engine_after(pkg, u1)
        weights_at[u1] = [eng.get_weights(a, 0) for a in (0, 1)]
        del eng
        torch.cuda.empty_cache()
        for a in (0, 1):
            if u0 >= len(mbs[a]):
                continue
            w_or, amb = _replay(cfg, mbs[a], u0, min(u1, len(mbs[a])), weights_at[u0][a], cfg["lr_ar"])
            d = float(np.abs(w_or - weights_at[u1][a]).max())
            report.append((a, u0, u1, d, sorted(amb)))
            ambiguous_total += len(amb)
            assert d <= 1e-5, report[-1]
    print("resynchronised: agent, u0, u1, max|oracle - engine|, updates with a p near a clip bound:",
          [(a, u0, u1, f"{d:.2e}", amb[:4]) for a, u0, u1, d, amb in report])
    # The same call replayed WITHOUT resynchronising (what test_gpu_configs compares): where
    # does it leave the engine, and did an ambiguous clip decision come first?
    free = []
    for a in (0, 1):
        w = state[a]["w"][0]
        closest = {}
        prev_d = 0.0
        for i in range(len(bounds) - 1):
            u0, u1 = bounds[i], min(bounds[i + 1], len(mbs[a]))
            if u0 >= len(mbs[a]):
                continue
            rc = {}
            w, _ = _replay(cfg, mbs[a], u0, u1, w, cfg["lr_ar"], closest=closest, relu_closest=rc)
            d = float(np.abs(w - weights_at[bounds[i + 1]][a]).max())
            near = min(((v, u) for u, v in closest.items() if u < u1), default=(np.inf, None))
            rnear = min(((v, u) for u, v in rc.items()), default=(np.inf, None))
            free.append((a, u1, d, near[0], near[1], rnear[0], rnear[1]))
            if d > 1e-4 and prev_d <= 1e-4:             # the onset of a divergence
                assert rnear[0] <= 1e-7, ("left the engine without a ReLU at its kink", free[-1])
            prev_d = d
    print("free replay: agent, after u updates, max|oracle - engine|, closest p to a clip bound "
          "(relative), at update, smallest |pre-activation| in the chunk, at update:",
          [(a, u1, f"{d:.2e}", f"{c:.1e}", cu, f"{z:.1e}", zu) for a, u1, d, c, cu, z, zu in free])
    # the clip mask is not what diverges: no output came near a clip bound
    assert min(c for _, _, _, c, _, _, _ in free) > 1e-4
