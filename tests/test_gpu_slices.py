"""Lane slices (nfsp_engine_cfg.slices): C3's 1,048,576 envs advanced in 16 slices of 65,536,
the learner consuming each slice's inserts before the next slice acts.  That bounds the
engine's declared policy lag (include/nfsp.h) by one slice instead of one million hands, so
C3 learns at the rate of the reference's one-hand-at-a-time main.train (main.py:27-67,
update trigger agent/agent.py:153-154).

* a lane's hand does not depend on the slicing (Philox counters and the dealer use the
  global lane id and the lane's hand count): with the learner off, a sliced engine fills
  M_RL and M_SL exactly like an unsliced one, record for record;
* at C3 size with the learner on, sampled lanes of the sliced rollouts replay bit-exact
  through oracle/rollout_oracle.py (global lane ids, hand index = rollouts // slices); with
  pipelined slices (slice_lag 2) against the snapshot they acted with, for Leduc and for
  bench.py's C5-textbook form (Kuhn, NFSP_TEXTBOOK_MSE);
* the C3 learning gate: exact exploitability after 8M / 16M / 25M / 33M hands at C3 (1M
  lanes, 16 slices, M_RL 200k, M_SL 2M) against the CPU seed band of the reference's
  main.train restated in C++ with the same memories and initial nets, 24 seeds
  (tests/golden/cpu_band_c3mem_24.json);
* the same gate for C4's arithmetic (8 x 1M lanes in 128 pipelined slices, the average-policy
  nets exchanged after every slice), emulated on one GPU by an engine group.
"""
import json
import os

import numpy as np
import pytest
import torch

import rollout_oracle as R
from test_gpu_fullsize import _bits_dev, _sample_lanes, _weights_flat

pytestmark = pytest.mark.gpu

C3 = dict(n_lanes=1_048_576, rl_capacity=200_000, sl_capacity=2_000_000)
HERE = os.path.dirname(os.path.abspath(__file__))


def _logical_rl(eng, p):
    """M_RL as the reference's deque: the last min(total, capacity) records, oldest first."""
    st = eng.stats()
    m = eng.memories(p)
    tot = int(st["rl_total"][p])
    n = min(tot, int(eng.cfg.rl_capacity))
    rows = torch.arange(tot - n, tot, device=m["rl_s"].device) % m["log_cap"]
    return {k: m[k][rows].cpu().numpy() for k in ("rl_s", "rl_a", "rl_r", "rl_s2", "rl_t")}


def test_slicing_leaves_every_hand_unchanged(pkg):
    """Learner off: 4 slices of 2,048 lanes fill the memories exactly like 8,192 lanes at once."""
    kw = dict(n_lanes=8192, rl_capacity=20_000, sl_capacity=3_000, seed=99, init_seed=3,
              inserts_per_update=1 << 30)
    a = pkg.engine.SelfPlayEngine(**kw)
    b = pkg.engine.SelfPlayEngine(slices=4, **kw)
    for _ in range(3):                 # M_RL wraps, the reservoir replaces
        a.step()
        b.step()
    sa, sb = a.stats(), b.stats()
    assert sb["rollouts"] == 4 * sa["rollouts"] == 12
    for k in ("hands", "rl_total", "sl_total", "rl_size", "sl_size", "actions", "reward"):
        assert sa[k] == sb[k], k
    assert sa["sl_total"][0] > kw["sl_capacity"] and sa["rl_total"][0] > kw["rl_capacity"]
    for p in (0, 1):
        ma, mb = _logical_rl(a, p), _logical_rl(b, p)
        for k in ma:
            assert np.array_equal(ma[k], mb[k]), (p, k)
        n = int(sa["sl_size"][p])
        xa, xb = a.memories(p), b.memories(p)
        assert np.array_equal(xa["sl_s"][:n].cpu().numpy(), xb["sl_s"][:n].cpu().numpy())
        assert np.array_equal(xa["sl_a"][:n].cpu().numpy(), xb["sl_a"][:n].cpu().numpy())


def _check_slice_lanes(eng, seed, lanes, rl_before, w=None, eps=None, game="leduc"):
    """Sampled local lanes of the last rollout vs the oracle's replay of their global lanes
    (acting nets / epsilon: the engine's current ones unless given)."""
    lane0, g = eng.last_slice()
    st = eng.stats()
    cnt = eng.lane_counts()
    assert len(cnt) == eng.slice_lanes
    assert cnt[:, 0].sum() == st["last_rl"][0] and cnt[:, 1].sum() == st["last_rl"][1]
    pre = np.zeros_like(cnt)
    pre[1:] = np.cumsum(cnt, axis=0)[:-1]
    w = _weights_flat(eng) if w is None else w
    eps = (float(st["epsilon"][0]), float(st["epsilon"][1])) if eps is None else eps
    mems = [eng.memories(p) for p in (0, 1)]
    for L in lanes:
        q = int(eng.cfg.quirks)
        ref = R._one_lane(lane0 + L, g, seed, w, eps, eng.cfg.eta, bool(q & 4), game, ext=q)
        for p in (0, 1):
            m = mems[p]
            n = len(ref["rl"][p])
            assert cnt[L, p] == n, (L, p)
            if n:
                rows = torch.tensor((rl_before[p] + pre[L, p] + np.arange(n)) % m["log_cap"],
                                    dtype=torch.int64, device=m["rl_s"].device)
                exp = ref["rl"][p]
                assert np.array_equal(_bits_dev(m["rl_s"][rows]), [e[0] for e in exp]), (L, p)
                assert np.array_equal(_bits_dev(m["rl_s2"][rows]), [e[3] for e in exp]), (L, p)
                assert np.abs(m["rl_a"][rows].cpu().numpy() - np.array([e[1] for e in exp])).max() <= 1e-6
                assert np.array_equal(m["rl_r"][rows].cpu().numpy(), np.array([e[2] for e in exp], np.float32))
            k = len(ref["sl"][p])
            assert cnt[L, 2 + p] == k, (L, p)
            if k:
                q = slice(int(pre[L, 2 + p]), int(pre[L, 2 + p]) + k)
                px = m["pend_x"][q].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
                assert np.array_equal(px, [e[0] for e in ref["sl"][p]]), (L, p)
                pos = m["pend_pos"][q].cpu().numpy()
                assert np.array_equal(pos, [rl_before[p] + pre[L, p] + e[2] for e in ref["sl"][p]])


def test_c3_sliced_rollouts_replay_on_the_oracle(pkg):
    """C3 at 16 slices, learner on: after one whole step (16 learner calls), the next two
    slices' sampled lanes replay bit-exact with their global lane ids and hand index 1."""
    seed = 2468
    eng = pkg.engine.SelfPlayEngine(seed=seed, init_seed=4, slices=16, **C3)
    eng.step()
    st = eng.stats()
    assert st["hands"] == C3["n_lanes"] and st["rollouts"] == 16
    assert min(st["br_updates"]) > 1000            # the learner ran between the slices
    S = eng.slice_lanes
    for k in range(2):
        before = tuple(int(v) for v in eng.stats()["rl_total"])
        eng.rollout()
        assert eng.last_slice() == (k * S, 1)
        _check_slice_lanes(eng, seed, _sample_lanes(S, 48, 10 + k), before)
        eng.update()


@pytest.mark.parametrize("K", [2, 8])
def test_pipelined_slices_act_with_the_nets_two_slices_back(pkg, K):
    """cfg.slice_lag 2: slice j acts with the nets and epsilon left by slice j - 2's learner
    (the step's start for j < 2), while slice j - 1's chains run.  The last slice of a step is
    replayed on the oracle with exactly those nets: for K = 2 the nets from before the step,
    for K = 8 the snapshot the engine kept (nfsp_engine_snapshot)."""
    seed = 1357
    eng = pkg.engine.SelfPlayEngine(seed=seed, init_seed=5, slices=K, slice_lag=2,
                                    n_lanes=262_144, rl_capacity=200_000, sl_capacity=2_000_000)
    eng.step()                                     # the learner has trained
    w_start = _weights_flat(eng)
    eps_start = tuple(float(v) for v in eng.stats()["epsilon"])
    eng.step()
    st = eng.stats()
    assert st["rollouts"] == 2 * K and st["hands"] == 2 * 262_144
    assert min(st["br_updates"]) > 100
    if K == 2:
        w, eps = w_start, eps_start
    else:
        w, eps = eng.snapshot((K - 1) & 1)
        assert not np.array_equal(w, w_start)      # trained past the step's start
    # the acting nets are not the final ones: the last slices' learners ran after they acted
    assert not np.array_equal(w.reshape(2, 3, -1)[:, :2], _weights_flat(eng).reshape(2, 3, -1)[:, :2])
    assert eng.last_slice() == ((K - 1) * eng.slice_lanes, 1)
    before = tuple(int(st["rl_total"][p] - st["last_rl"][p]) for p in (0, 1))
    _check_slice_lanes(eng, seed, _sample_lanes(eng.slice_lanes, 48, 20 + K), before, w, eps)


def test_pipelined_snapshot_keeps_the_epsilon_its_slice_acted_with(pkg):
    """The epsilon half of the snapshot: a setting where epsilon has NOT
    decayed to ~0 between the slices (eps 0.9, eta 1 so every decision is an eps-greedy BR one,
    an update per ~1,500 RL inserts so eps / iteration falls slowly).  The last slice of the
    first step is replayed with snapshot (K - 1) & 1's nets and epsilon; the epsilon after the
    step, which a snapshot overwritten by the last slice's own learner call would report, differs
    and would change ~2% of the draws."""
    seed, K = 6060, 8
    eng = pkg.engine.SelfPlayEngine(seed=seed, init_seed=3, slices=K, slice_lag=2, n_lanes=4096,
                                    rl_capacity=20_000, sl_capacity=20_000, inserts_per_update=2048,
                                    epsilon=0.9, eta=1.0)
    eng.step()
    st = eng.stats()
    w, eps = eng.snapshot((K - 1) & 1)
    assert 1e-3 < min(eps) and max(eps) < 0.9                   # decayed, but far from 0
    assert st["epsilon"][0] < 0.5 * eps[0]                     # the step's last learner moved it
    assert eng.last_slice() == ((K - 1) * eng.slice_lanes, 0)
    before = tuple(int(st["rl_total"][p] - st["last_rl"][p]) for p in (0, 1))
    _check_slice_lanes(eng, seed, range(eng.slice_lanes), before, w, eps)


def test_kuhn_textbook_pipelined_slices_replay_on_the_oracle(pkg):
    """bench.py's C5-textbook form (Kuhn, NFSP_TEXTBOOK_MSE, 16 pipelined slices) at 262,144
    lanes: the last slice of the second step replays bit-exact with the snapshot it acted with
    (sampled AR actions, reservoir M_SL, constant epsilon included)."""
    seed, K = 4242, 16
    eng = pkg.engine.SelfPlayEngine(seed=seed, init_seed=2, slices=K, slice_lag=2, n_lanes=262_144,
                                    rl_capacity=200_000, sl_capacity=2_000_000,
                                    game=pkg.native.GAME_KUHN, quirks=pkg.native.TEXTBOOK_MSE)
    eng.step()
    eng.step()
    st = eng.stats()
    assert st["rollouts"] == 2 * K and min(st["br_updates"]) > 100
    w, eps = eng.snapshot((K - 1) & 1)
    assert eng.last_slice() == ((K - 1) * eng.slice_lanes, 1)
    before = tuple(int(st["rl_total"][p] - st["last_rl"][p]) for p in (0, 1))
    _check_slice_lanes(eng, seed, _sample_lanes(eng.slice_lanes, 48, 77), before, w, eps, game="kuhn")


def test_pipelined_step_is_deterministic(pkg):
    def run():
        e = pkg.engine.SelfPlayEngine(seed=808, init_seed=6, slices=16, slice_lag=2, **C3)
        e.step()
        e.step()
        return e.stats(), _weights_flat(e)
    s1, w1 = run()
    torch.cuda.empty_cache()
    s2, w2 = run()
    assert s1 == s2
    assert np.array_equal(w1, w2)


def _band():
    """The CPU reference's band: tests/golden/cpu_band_c3mem_24.json, 24 seeds (the 8 of
    cpu_band_c3mem.json merged with 16 more, tests/golden/gen_cpu_band.py)."""
    with open(os.path.join(HERE, "golden", "cpu_band_c3mem_24.json")) as f:
        return json.load(f)


def _band_report(band, gpu, hands_of):
    cpu = {int(h): np.array(v) for h, v in band["curves_by_hands"].items()}
    last = max(cpu)
    report = []
    for k, xs in gpu.items():
        h = hands_of(k)
        near = min(cpu, key=lambda x: abs(x - min(h, last)))   # the CPU checkpoint (every 2M hands) nearest
        cm, cs = float(cpu[near].mean()), float(cpu[near].std())
        gm, gs = float(np.mean(xs)), float(np.std(xs))
        report.append((h, near, round(cm, 3), round(cs, 3), round(gm, 3), round(gs, 3), round(cm + cs - gm, 3)))
    return report


def test_c3_sliced_learns_within_the_cpu_seed_band(pkg):
    """BASELINE.json's second metric at C3, as bench.py measures C3 (1M lanes, 16 pipelined
    slices): the exploitability-vs-hands curve lies within the CPU reference's seed band.
    Bars at every checkpoint: |GPU mean - CPU mean| <= 2 sigma, and the GPU mean >= 0.1 chips
    inside CPU mean + 1 sigma (sigma: the CPU seeds' std).  GPU: 16 seeds (1234 + s, initial
    nets s); CPU: 24 seeds.
    Round 6 (profiles/r06/c3_slices_seeds*.json, 24 GPU seeds): 1.639 / 1.564 / 1.522 / 1.475 at
    8.4 / 16.8 / 25.2 / 33.5M hands against the CPU's 1.440 / 1.399 / 1.386 / 1.381 (sigma
    ~0.46): +0.2 to +0.43 sigma, 0.27-0.37 chips inside the bar.  Round 5's gate compared 8 GPU
    seeds with the first 8 CPU seeds alone, whose mean happened to be 0.15-0.2 chips below the 24
    seeds' (sigma 0.25 vs 0.46), and passed 8.4M by 0.036."""
    import bench
    c3 = bench.CONFIGS["c3"]
    K, lag = c3["slices"], c3["slice_lag"]
    assert (K, lag) == (16, 2) and c3["n_lanes"] == C3["n_lanes"]
    band = _band()
    assert len(band["seeds"]) == 24
    checkpoints = (8, 16, 24, 32)                  # engine steps of 1,048,576 hands
    gpu = {c: [] for c in checkpoints}
    for s in range(16):
        eng = pkg.engine.SelfPlayEngine(seed=1234 + s, init_seed=s, slices=K, slice_lag=lag, **C3)
        for k in range(1, checkpoints[-1] + 1):
            eng.step()
            if k in gpu:
                gpu[k].append(eng.exploitability(0)["exploitability"])
        eng.close()
        del eng
        torch.cuda.empty_cache()
    report = _band_report(band, gpu, lambda k: k * C3["n_lanes"])
    print("hands, cpu checkpoint, cpu mean, cpu std, gpu mean, gpu std, margin:", report)
    for (h, near, cm, cs, gm, gs, margin) in report:
        assert abs(gm - cm) <= 2 * cs, report
        assert gm <= cm + cs - 0.1, report          # >= 0.1 chips inside the bar


def test_c4_emulated_learns_within_the_cpu_seed_band(pkg):
    """C4's arithmetic on one GPU, as bench.py --gpus 8 runs it (bench.CONFIGS["c4"]): 8 shards of
    1,048,576 lanes (C3's memories each) in 128 pipelined slices (slice_lag 2), the average-policy
    nets exchanged after EVERY slice -- W0 + 2 x the mean of the shards' deltas, the rank path's
    arithmetic (tests/test_gpu_exchange.py shows the ranks equal to a group bit for bit) -- done on
    device by an engine group.  Exploitability at equal TOTAL hands against the CPU band, from the
    first checkpoint (one step = 8.4M hands) to 8 steps (67M), with the C3 bar:
    |GPU mean - CPU mean| <= 2 sigma and GPU mean <= CPU mean + 1 sigma (16 GPU seeds, the 24 CPU
    seeds).  Besides the bar, a margin: the GPU mean sits >= 0.1 chips below CPU mean + 1 sigma at
    every checkpoint.  Seeds 0-7 measured 1.421 / 1.234 / 1.216 / 1.165 / 1.103 (round 5), seeds
    8-15 1.707 / 1.415 / 1.372 / 1.339 / 1.309 (profiles/r06/c4_gate_seeds8_23.json): ~0.34 chips
    inside the 24-seed bar at 8.4M, more later.  Measured at 128 slices (profiles/r04_c4x_k128_ar_g2.json): 1.421 at 8.4M (bar
    1.539), 1.234 / 1.216 / 1.165 at 16.8 / 25.2 / 33.5M; 64 slices (round 4's C4) passed 8.4M by
    0.012 chips, round 3's once-per-step exchange reached the band only from 33.5M."""
    import bench
    c4 = bench.CONFIGS["c4"]
    band = _band()
    R, lanes, K = 8, c4["n_lanes"], c4["slices"]
    assert (K, c4["slice_lag"], c4["xchg_every"], c4["xchg_gain"]) == (128, 2, 1, 2.0)
    checkpoints = (1, 2, 3, 4, 8)                  # steps of 8 x 1,048,576 hands
    gpu = {c: [] for c in checkpoints}
    for s in range(16):
        g = pkg.engine.EngineGroup(R, n_lanes=lanes, rl_capacity=c4["rl_capacity"], sl_capacity=c4["sl_capacity"],
                                   seed=1234 + 1000 * s, init_seed=1000 * s, slices=K, slice_lag=2)
        g.set_exchange(pkg.native.XCHG_AR, every=c4["xchg_every"], scale=c4["xchg_gain"] / R)
        g.average_ar()                             # the common start: replica 0's nets
        for k in range(1, checkpoints[-1] + 1):
            g.step()
            if k in gpu:
                gpu[k].append(g.exploitability(0)["exploitability"])
        assert g.stats()["hands"] == checkpoints[-1] * R * lanes
        # one AR net: every replica holds the exchanged nets
        w0 = g.replicas[0].get_weights(0, 0)
        assert all(np.array_equal(w0, e.get_weights(0, 0)) for e in g.replicas[1:])
        g.close()
        del g
        torch.cuda.empty_cache()
    report = _band_report(band, gpu, lambda k: k * R * lanes)
    print("hands, cpu checkpoint, cpu mean, cpu std, gpu mean, gpu std, margin:", report)
    for (h, near, cm, cs, gm, gs, margin) in report:
        assert abs(gm - cm) <= 2 * cs, report
        assert gm <= cm + cs - 0.1, report          # >= 0.1 chips inside the bar


def test_pipelined_step_equals_its_declared_schedule(pkg):
    """cfg.slice_lag 2 is exactly its declared semantics: a lag-1 engine driven slice by slice
    -- slice j's rollout acting with the nets and epsilon left by slice j - 2's learner (the
    step's start for j < 2, nfsp_rollout_with), then its learner -- ends every step with the
    same nets, counters and memories, bit for bit, as the pipelined engine."""
    K = 4
    kw = dict(n_lanes=32_768, slices=K, rl_capacity=20_000, sl_capacity=30_000, seed=4711, init_seed=9,
              target_every=13)
    a = pkg.engine.SelfPlayEngine(slice_lag=2, **kw)
    b = pkg.engine.SelfPlayEngine(slice_lag=1, **kw)
    for step in range(3):
        a.step()
        snap = [_weights_flat(b)] * 2
        eps = [tuple(float(v) for v in b.stats()["epsilon"])] * 2
        for j in range(K):
            b.rollout_with(snap[j & 1], eps[j & 1])
            b.update()
            if j + 2 < K:
                snap[j & 1] = _weights_flat(b)
                eps[j & 1] = tuple(float(v) for v in b.stats()["epsilon"])
        sa, sb = a.stats(), b.stats()
        assert sa == sb, (step, {k: (sa[k], sb[k]) for k in sa if sa[k] != sb[k]})
        assert np.array_equal(_weights_flat(a), _weights_flat(b)), step
    assert min(sa["br_updates"]) > 50 and sa["target_syncs"][0] > 3
    for p in (0, 1):
        ma, mb = _logical_rl(a, p), _logical_rl(b, p)
        for k in ma:
            assert np.array_equal(ma[k], mb[k]), (p, k)
        n = int(sa["sl_size"][p])
        assert np.array_equal(a.memories(p)["sl_a"][:n].cpu().numpy(), b.memories(p)["sl_a"][:n].cpu().numpy())
