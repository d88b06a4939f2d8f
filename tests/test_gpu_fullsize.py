"""Parity and invariants at BASELINE.json's full single-GPU size (C3: 1,048,576 lanes,
M_RL 200k, M_SL 2M; C5: the Kuhn swap-in at the same size).

The oracle cannot replay a million hands in a test's time, so the full-size rollout is
checked through properties that do not depend on its size:
* sampled lanes (the first and last of each 64-lane wave and 256-lane workgroup
  boundary, the last lane, and random ones) replayed one by one by
  oracle/rollout_oracle.py._one_lane.  The engine's Philox counters are per lane and per
  hand, so a lane's hand does not depend on the others.  Its records are located in M_RL
  and the pending M_SL list through the exclusive prefix of the per-lane counts
  (nfsp_engine_lane_counts).  Bars as in test_gpu_engine.py: bit-exact observations, r, t,
  RL positions; action vectors within 1e-6;
* every record of the rollout: s / s2 are valid observations (one private card in the
  round-0 card row; the round-1 row empty or holding that card and the public card),
  r a multiple of 0.5 within the stakes, t in {0, 1}; rewards zero-sum over the hands;
* after whole engine steps: update counts, schedules and target syncs follow the
  reference cadence (agent/agent.py:153,209-273); memory sizes; determinism of a
  C3 step (two engines, same seed, identical weights bit for bit).
"""
import numpy as np
import pytest
import torch

import rollout_oracle as R

pytestmark = pytest.mark.gpu

C3 = dict(n_lanes=1_048_576, rl_capacity=200_000, sl_capacity=2_000_000)


def _weights_flat(eng):
    return np.concatenate([eng.get_weights(a, n) for a in (0, 1) for n in (0, 1, 2)])


def _bits_dev(x):
    """[n, 30] 0/1 float rows (device) -> int64 bit masks (host)."""
    w = (torch.ones(30, dtype=torch.int64, device=x.device) << torch.arange(30, device=x.device))
    return ((x != 0).to(torch.int64) * w).sum(dim=1).cpu().numpy()


def _sample_lanes(n, k, seed):
    edges = [0, 1, 63, 64, 255, 256, 4095, 4096, n // 2, n - 2, n - 1]
    rng = np.random.RandomState(seed)
    return sorted(set(edges) | set(rng.randint(0, n, size=k).tolist()))


def _check_lanes(eng, seed, g, lanes, game="leduc", rl_before=(0, 0)):
    st = eng.stats()
    cnt = eng.lane_counts()
    assert cnt[:, 0].sum() == st["last_rl"][0] and cnt[:, 1].sum() == st["last_rl"][1]
    assert cnt[:, 2].sum() == st["last_sl"][0] and cnt[:, 3].sum() == st["last_sl"][1]
    pre = np.zeros_like(cnt)
    pre[1:] = np.cumsum(cnt, axis=0)[:-1]
    w = _weights_flat(eng)
    alias = bool(eng.cfg.quirks & 4)
    eps = (float(st["epsilon"][0]), float(st["epsilon"][1]))
    mems = [eng.memories(p) for p in (0, 1)]
    for L in lanes:
        ref = R._one_lane(L, g, seed, w, eps, eng.cfg.eta, alias, game)
        for p in (0, 1):
            m = mems[p]
            n = len(ref["rl"][p])
            assert cnt[L, p] == n, (L, p)
            rows = torch.tensor((rl_before[p] + pre[L, p] + np.arange(n)) % m["log_cap"],
                                dtype=torch.int64, device=m["rl_s"].device)
            if n:
                exp = ref["rl"][p]
                assert np.array_equal(_bits_dev(m["rl_s"][rows]), [e[0] for e in exp]), (L, p)
                assert np.array_equal(_bits_dev(m["rl_s2"][rows]), [e[3] for e in exp]), (L, p)
                a = m["rl_a"][rows].cpu().numpy()
                assert np.abs(a - np.array([e[1] for e in exp])).max() <= 1e-6, (L, p)
                assert np.array_equal(m["rl_r"][rows].cpu().numpy(), np.array([e[2] for e in exp], np.float32))
                assert np.array_equal(m["rl_t"][rows].cpu().numpy(), np.array([e[4] for e in exp], np.uint8))
            k = len(ref["sl"][p])
            assert cnt[L, 2 + p] == k, (L, p)
            if k:
                q = slice(int(pre[L, 2 + p]), int(pre[L, 2 + p]) + k)
                px = m["pend_x"][q].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
                assert np.array_equal(px, [e[0] for e in ref["sl"][p]]), (L, p)
                pa = m["pend_a"][q].cpu().numpy()
                assert np.abs(pa - np.array([e[1] for e in ref["sl"][p]])).max() <= 1e-6
                pos = m["pend_pos"][q].cpu().numpy()
                assert np.array_equal(pos, [rl_before[p] + pre[L, p] + e[2] for e in ref["sl"][p]])
    return cnt


def _valid_obs(bits, game):
    """Observation bit masks: one private card in the round-0 card row (bits 24..26); the
    round-1 row (27..29) empty or holding the private and the public card (Leduc)."""
    r0 = (bits >> 24) & 7
    r1 = (bits >> 27) & 7
    one = (r0 != 0) & ((r0 & (r0 - 1)) == 0)
    if game == "kuhn":           # one betting round: no round-1 history or card bits
        return one & (r1 == 0) & (((bits >> 6) & 63) == 0) & (((bits >> 18) & 63) == 0)
    n1 = np.array([bin(int(v)).count("1") for v in range(8)])[r1]
    return one & ((r1 == 0) | (((r1 & r0) != 0) & (n1 <= 2)))


@pytest.mark.parametrize("game", ["leduc", "kuhn"])
def test_fullsize_rollout_sampled_lanes_and_records(pkg, game):
    g_id = pkg.native.GAME_KUHN if game == "kuhn" else pkg.native.GAME_LEDUC
    seed = 1234
    eng = pkg.engine.SelfPlayEngine(seed=seed, init_seed=0, game=g_id, inserts_per_update=1 << 30, **C3)
    eng.rollout()
    st = eng.stats()
    assert st["hands"] == C3["n_lanes"]
    _check_lanes(eng, seed, 0, _sample_lanes(C3["n_lanes"], 96, 5), game)
    # every record of the rollout
    assert st["reward"][0] + st["reward"][1] == 0.0          # zero-sum hands
    for p in (0, 1):
        m = eng.memories(p)
        n = int(st["last_rl"][p])
        for key in ("rl_s", "rl_s2"):
            b = _bits_dev(m[key][:n])
            assert _valid_obs(b, game).all(), key
        r = m["rl_r"][:n].cpu().numpy()
        assert np.all(2 * r == np.round(2 * r)) and np.abs(r).max() <= 13
        t = m["rl_t"][:n].cpu().numpy()
        assert set(np.unique(t).tolist()) <= {0, 1}
        assert (r[t == 0] == 0).all()                       # rewards only on terminal tuples
        k = int(st["last_sl"][p])
        assert _valid_obs(m["pend_x"][:k].cpu().numpy().astype(np.int64) & 0xFFFFFFFF, game).all()
    # the second rollout of the same engine (g = 1: dealers flip, fresh Philox counters)
    eng.update()
    before = tuple(int(v) for v in eng.stats()["rl_total"])
    eng.rollout()
    _check_lanes(eng, seed, 1, _sample_lanes(C3["n_lanes"], 32, 6), game, rl_before=before)


def _eps_after(eps0, updates):
    e = eps0
    for u in range(1, updates + 1):
        e = e ** 1 / (2 * u)                     # agent/agent.py:253 (iteration = 2u)
    return e


def test_fullsize_engine_steps_follow_the_reference_cadence(pkg):
    eng = pkg.engine.SelfPlayEngine(seed=77, init_seed=1, **C3)
    for _ in range(2):
        eng.step()
    st = eng.stats()
    B, ipu, every = eng.cfg.batch, eng.cfg.inserts_per_update, eng.cfg.target_every
    for a in (0, 1):
        trig = st["rl_total"][a] // ipu
        U = trig - 1 if trig >= 1 else 0           # BR update iff M_RL size at the trigger > batch
        assert ipu == 128 and B == 128
        assert st["br_updates"][a] == U
        assert st["iteration"][a] == 2 * U
        assert st["target_syncs"][a] == (U + every - 1) // every
        assert 0 < st["ar_updates"][a] <= trig
        assert st["lr_br"][a] == pytest.approx(0.05 / (1 + 0.003 * np.sqrt(2 * U)), rel=1e-6)   # f32
        assert st["temp"][a] == pytest.approx(1 / (1 + 0.02 * np.sqrt(2 * U)), rel=1e-12)
        assert st["epsilon"][a] == pytest.approx(_eps_after(0.06, U), rel=1e-12, abs=0)
        assert st["rl_size"][a] == min(st["rl_total"][a], C3["rl_capacity"])
        assert st["sl_size"][a] == min(st["sl_total"][a], C3["sl_capacity"])
        for n in (0, 1, 2):
            assert np.isfinite(eng.get_weights(a, n)).all()


def test_fullsize_step_is_deterministic(pkg):
    def run():
        e = pkg.engine.SelfPlayEngine(seed=4321, init_seed=2, **C3)
        e.step()
        return e.stats(), _weights_flat(e)
    s1, w1 = run()
    torch.cuda.empty_cache()
    s2, w2 = run()
    assert s1 == s2
    assert np.array_equal(w1, w2)
    assert min(s1["br_updates"]) > 1000
