"""Parity at BASELINE.json's C2 and C3 sizes (configs[1], configs[2]).

C2: 65,536 lanes, M_RL = M_SL = 40,000, eta 0.1.
* sampled lanes of a rollout (wave / workgroup edges, the last lane, random ones) are
  replayed one by one by oracle/rollout_oracle.py._one_lane and found in the memories
  through the per-lane record counts (test_gpu_fullsize._check_lanes);
* one whole learner call (nfsp_engine_update, ~1,000 updates per agent and net, with the
  memories full: M_RL wraps, the reservoir replaces) is replayed update by update by
  oracle/learner_oracle.py.

C3: 1,048,576 lanes, M_RL 200k, M_SL 2M.  A whole C3 learner call is ~20k updates per agent
and net.  The updates of a chain are sequential, so a prefix of them is exact.  The test
hook nfsp_engine_set_update_limit runs the first 200 updates of every chain.  The oracle
replays the same 200, on the engine's memories after two C3 steps and a rollout.

Bars: update counts, iteration and epsilon schedules, and the reservoir after the call are
exact.  Weights, on a prefix of the updates (C3: the first 200, C2: the first 100): max 1e-4,
median 1e-7, as in test_gpu_learner.py.

On a whole C2 call (~500-700 updates per net) the max bar does not hold, and the test says
by how much.  The cause is measured and pinned by tests/test_gpu_learner_divergence.py:
replayed from the engine's own weights every 64 updates, the oracle agrees within 3.6e-7
throughout; the free replay leaves (agent 1's AR net, ~3e-3 after update ~330) where a
hidden pre-activation sits within ~6e-8 of zero, so its ReLU derivative follows the
summation order.  (Not, as round 2 guessed, Keras' clip mask: no output comes within 1e-3 of
a clip bound.)  The whole-call bars here are therefore a bound on that divergence: median
1e-7, max 1e-2, at most 10% of the weights off by more than 1e-4, and the nets' outputs on
every distinct observation in M_RL within 5e-3 (measured: 1.1e-3).
"""
import numpy as np
import pytest
import torch

import learner_oracle as LO
import nn_oracle as nn
from test_gpu_fullsize import _bits_dev, _check_lanes, _sample_lanes

pytestmark = pytest.mark.gpu

C2 = dict(n_lanes=65_536, rl_capacity=40_000, sl_capacity=40_000, eta=0.1)
C3 = dict(n_lanes=1_048_576, rl_capacity=200_000, sl_capacity=2_000_000)


def _snapshot(eng):
    """The engine after a rollout, in learner_oracle's state layout (bits computed on device)."""
    st = eng.stats()
    out = []
    for a in (0, 1):
        m = eng.memories(a)
        n_sl = int(st["last_sl"][a])
        out.append(dict(
            w={n: eng.get_weights(a, n) for n in (0, 1, 2)},
            rl_total=int(st["rl_total"][a]), last_rl=int(st["last_rl"][a]),
            sl_total=int(st["sl_total"][a]), last_sl=n_sl,
            iteration=int(st["iteration"][a]), br_updates=int(st["br_updates"][a]),
            epsilon=float(st["epsilon"][a]),
            rl_s_bits=_bits_dev(m["rl_s"]), rl_s2_bits=_bits_dev(m["rl_s2"]),
            rl_a=m["rl_a"].cpu().numpy(), rl_r=m["rl_r"].cpu().numpy(), rl_t=m["rl_t"].cpu().numpy(),
            sl_s_bits=_bits_dev(m["sl_s"]), sl_a=m["sl_a"].cpu().numpy(),
            pend_x=m["pend_x"][:n_sl].cpu().numpy().astype(np.int64) & 0xFFFFFFFF,
            pend_a=m["pend_a"][:n_sl].cpu().numpy(), pend_pos=m["pend_pos"][:n_sl].cpu().numpy()))
    return st, out


def _oracle_cfg(c):
    return dict(c=c.inserts_per_update, batch=c.batch, epochs=c.epochs, rl_capacity=c.rl_capacity,
                sl_capacity=c.sl_capacity, target_every=c.target_every, lr_br=c.lr_br, lr_ar=c.lr_ar,
                gamma=c.gamma, seed=c.seed, epsilon=c.epsilon)


def _check_learner(eng, st0, st1, want, state, prefix=None, strict=True):
    obs = np.unique(np.concatenate([state[a]["rl_s2_bits"] for a in (0, 1)]))
    x = LO.bits_to_x(obs)
    for a in (0, 1):
        W = want[a]
        assert st1["br_updates"][a] == W["br_updates"]
        assert st1["ar_updates"][a] - st0["ar_updates"][a] == W["ar_updates"]
        assert st1["iteration"][a] == W["iteration"]
        assert st1["epsilon"][a] == pytest.approx(W["epsilon"], rel=1e-12)
        if prefix is None:
            assert st1["exploitability"][a] == pytest.approx(W["exploitability"], abs=1e-4)
        else:
            assert W["U_br"] > prefix and W["U"] > prefix        # the prefix is a strict one
        for n in (0, 1, 2):
            got = eng.get_weights(a, n)
            d = np.abs(got - W["w"][n])
            assert np.median(d) <= 1e-7, (a, n, np.median(d))
            if strict:
                assert d.max() <= 1e-4, (a, n, d.max())
            else:
                assert (d > 1e-4).mean() <= 0.10 and d.max() <= 1e-2, (a, n, d.max(), (d > 1e-4).mean())
            act = nn.ACT_SOFTMAX if n == 0 else nn.ACT_RELU
            y0 = nn.MLP(act, 64, weights=nn.unpack_weights(got)).predict(x)
            y1 = nn.MLP(act, 64, weights=nn.unpack_weights(W["w"][n])).predict(x)
            assert np.abs(y0 - y1).max() <= (1e-5 if strict else 5e-3), (a, n, np.abs(y0 - y1).max())
        m = eng.memories(a)
        size = int(st1["sl_size"][a])
        assert np.array_equal(_bits_dev(m["sl_s"][:size]), W["res_x"][:size])
        assert np.array_equal(m["sl_a"][:size].cpu().numpy(), W["res_a"][:size])


def _c2_engine(pkg, check_lanes=False):
    """C2 after six steps (M_RL wraps, the reservoir replaces) and the 7th rollout."""
    seed = 2024
    eng = pkg.engine.SelfPlayEngine(seed=seed, init_seed=3, **C2)
    eng.rollout()
    if check_lanes:
        _check_lanes(eng, seed, 0, _sample_lanes(C2["n_lanes"], 64, 11))
    eng.update()
    for _ in range(5):
        eng.step()
    before = tuple(int(v) for v in eng.stats()["rl_total"])
    eng.rollout()                                   # g = 6
    if check_lanes:
        _check_lanes(eng, seed, 6, _sample_lanes(C2["n_lanes"], 64, 12), rl_before=before)
    st0, state = _snapshot(eng)
    assert min(st0["rl_total"]) > C2["rl_capacity"] and max(st0["sl_total"]) > C2["sl_capacity"]
    return eng, st0, state


@pytest.mark.parametrize("prefix", [100, None])
def test_c2_rollout_sampled_lanes_and_learner_call(pkg, prefix):
    eng, st0, state = _c2_engine(pkg, check_lanes=prefix is not None)
    if prefix is not None:
        eng.set_update_limit(prefix)
    eng.update()
    st1 = eng.stats()
    want = LO.learner_step(_oracle_cfg(eng.cfg), state, quirks=eng.cfg.quirks, max_updates=prefix)
    assert min(w["U_br"] for w in want) > 500
    _check_learner(eng, st0, st1, want, state, prefix=prefix, strict=prefix is not None)


def test_c3_learner_prefix(pkg):
    eng = pkg.engine.SelfPlayEngine(seed=4321, init_seed=7, **C3)
    for _ in range(2):
        eng.step()
    eng.rollout()
    st0, state = _snapshot(eng)
    assert min(st0["rl_total"]) > C3["rl_capacity"]          # M_RL is the capacity window
    prefix = 200
    eng.set_update_limit(prefix)
    eng.update()
    st1 = eng.stats()
    want = LO.learner_step(_oracle_cfg(eng.cfg), state, quirks=eng.cfg.quirks, max_updates=prefix)
    _check_learner(eng, st0, st1, want, state, prefix=prefix)
