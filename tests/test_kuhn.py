"""Kuhn swap-in (BASELINE config C5).

The reference has no Kuhn game; the swap-in reuses the Leduc machinery (include/nfsp.h
NFSP_GAME_KUHN).  Its parity is therefore anchored analytically: the oracle evaluator
scores Kuhn's known Nash equilibrium family (Kuhn 1950; first actor bets the best card with
3 alpha, bluffs the worst with alpha, calls with the middle card at alpha + 1/3) at
exploitability 0 and the first actor's value at -1/18, for every alpha in [0, 1/3].  The GPU
env, evaluator and engine rollout are then checked against the oracle restatement.
"""
import itertools

import numpy as np
import pytest

import exploit_oracle as eo
import nfsp_oracle as orc
import nn_oracle as nn

K, Q, J = 0, 1, 2            # rank 0 is the best card


def nash(seat, alpha):
    """Kuhn's equilibrium for `seat`, as a function of its observation bits (history bits
    12p + 2 slot + act of round 0, card bit 24 + rank)."""
    o = 1 - seat

    def fn(obs):
        card = next(r for r in range(3) if (obs >> (24 + r)) & 1)
        h = obs & 0xFFFFFF
        if h == 0:                                        # first to act
            b = {K: 3 * alpha, Q: 0.0, J: alpha}[card]
            return (0.0, 1.0 - b, b)
        if h == 1 << (12 * o):                            # second, facing a check
            b = {K: 1.0, Q: 0.0, J: 1.0 / 3.0}[card]
            return (0.0, 1.0 - b, b)
        if h == 1 << (12 * o + 1):                        # second, facing a bet
            c = {K: 1.0, Q: 1.0 / 3.0, J: 0.0}[card]
            return (1.0 - c, c, 0.0)
        if h == (1 << (12 * seat)) | (1 << (12 * o + 3)):  # first, checked, facing a bet
            c = {K: 1.0, Q: alpha + 1.0 / 3.0, J: 0.0}[card]
            return (1.0 - c, c, 0.0)
        raise AssertionError(f"unreachable Kuhn observation {h:#x}")
    return eo.TabularPolicy(fn)


@pytest.mark.parametrize("alpha", [0.0, 0.1, 1.0 / 3.0])
def test_oracle_kuhn_nash_is_unexploitable(alpha):
    p0, p1 = nash(0, alpha), nash(1, alpha)
    r = eo.exploitability_of(p0, p1, "kuhn")
    assert abs(r["exploitability"]) < 1e-12
    assert abs(r["value0"]) < 1e-12                       # dealer alternation: seats equal
    # seat 0 always first to act: the game value -1/18
    v = eo.on_policy_value0(p0, p1, "kuhn", dealers=(0,))
    assert v == pytest.approx(-1.0 / 18.0, abs=1e-12)


def test_oracle_kuhn_deviation_is_exploitable():
    p0, p1 = nash(0, 0.1), nash(1, 0.1)
    always_bet = eo.TabularPolicy(lambda obs: (0.0, 0.0, 1.0))
    assert eo.exploitability_of(always_bet, p1, "kuhn")["exploitability"] > 0.05
    assert eo.exploitability_of(p0, always_bet, "kuhn")["exploitability"] > 0.05


def test_oracle_kuhn_env_rules():
    env = orc.Env(deal_source=lambda: (K, J, 0), game="kuhn")
    env.reset(0)
    assert env.contrib == [2, 2]                         # antes 1 / 1
    env.step(np.array([0, 0, 1.0]), 0)                   # bet
    env.step(np.array([0, 0, 1.0]), 1)                   # a re-raise is remapped to a call
    assert env.terminated and env.reward[0] == 2.0 and env.reward[1] == -2.0
    env.reset(1)
    env.step(np.array([0, 1.0, 0]), 1)                   # check
    env.step(np.array([0, 1.0, 0]), 0)                   # check: showdown, K beats J
    assert env.terminated and env.reward[0] == 1.0
    env.reset(0)
    env.step(np.array([1.0, 0, 0]), 0)                   # fold: loses the ante
    assert env.terminated and env.reward[0] == -1.0 and env.reward[1] == 1.0


# ---- GPU ----------------------------------------------------------------------
@pytest.mark.gpu
def test_gpu_kuhn_env_exhaustive(pkg):
    """Every deal x dealer x raw action sequence (fold/call/raise, 4 deep; the actor
    alternates from the dealer, steps after the end included) through the batched env
    (nfsp_env_*, one env per case) vs the oracle Env: both players' get_state after every
    step, bit for bit."""
    import torch
    nat = pkg.native
    cases = [(r0, r1, d, seq) for r0, r1 in itertools.permutations(range(3), 2) for d in (0, 1)
             for seq in itertools.product(range(3), repeat=4)]
    n = len(cases)
    ctx = nat.Context(n, seed=3, game=nat.GAME_KUHN)
    dev = "cuda"
    ranks = torch.tensor([[c[0], c[1], 0] for c in cases], dtype=torch.uint8, device=dev)
    dealer = torch.tensor([c[2] for c in cases], dtype=torch.uint8, device=dev)
    ctx.call("nfsp_env_set_deal", nat.ptr(ranks))
    ctx.call("nfsp_env_reset", nat.ptr(dealer))
    envs = []
    for (r0, r1, d, _) in cases:
        e = orc.Env(deal_source=lambda r0=r0, r1=r1: (r0, r1, 0), game="kuhn")
        e.reset(d)
        envs.append(e)
    s = torch.empty((n, 30), device=dev)
    a = torch.empty((n, 3), device=dev)
    r = torch.empty(n, device=dev)
    s2 = torch.empty((n, 30), device=dev)
    t = torch.empty(n, dtype=torch.uint8, device=dev)
    w = (1 << np.arange(30, dtype=np.int64))
    for k in range(5):
        if k > 0:
            pl = np.array([(c[2] + k - 1) % 2 for c in cases], np.uint8)
            act = np.zeros((n, 3), np.float32)
            act[np.arange(n), [c[3][k - 1] for c in cases]] = 1.0
            # keep the device buffers referenced until the stream has consumed them
            act_d = torch.as_tensor(act, device=dev)
            pl_d = torch.as_tensor(pl, device=dev)
            mask_d = torch.ones(n, dtype=torch.uint8, device=dev)
            ctx.call("nfsp_env_step", nat.ptr(act_d), 0, nat.ptr(pl_d), nat.ptr(mask_d))
            torch.cuda.synchronize()
            for i, e in enumerate(envs):
                e.step(act[i].astype(np.float64), int(pl[i]))
        for p in (0, 1):
            ctx.call("nfsp_env_get_state", p, None, nat.ptr(s), nat.ptr(a), nat.ptr(r), nat.ptr(s2), nat.ptr(t))
            sb = (s.cpu().numpy().astype(np.int64) * w).sum(axis=1)
            s2b = (s2.cpu().numpy().astype(np.int64) * w).sum(axis=1)
            for i, e in enumerate(envs):
                es, ea, er, es2, et = e.get_state(p)
                assert sb[i] == orc_bits(es) and s2b[i] == orc_bits(es2), (k, p, cases[i])
                assert np.array_equal(a[i].cpu().numpy().astype(np.float64), ea.reshape(3)), (k, p, cases[i])
                assert float(r[i]) == float(er) and bool(t[i]) == bool(et), (k, p, cases[i])


def orc_bits(x):
    v = np.asarray(x).reshape(-1)
    return int(sum(int(v[i] != 0) << i for i in range(30)))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_gpu_kuhn_exploitability_matches_oracle(pkg, mode):
    import torch
    rng = np.random.RandomState(5)
    w0 = nn.MLP(nn.ACT_SOFTMAX, 64, rng=rng).flat()
    w1 = nn.MLP(nn.ACT_SOFTMAX, 64, rng=rng).flat()
    ctx = pkg.native.Context(1, game=pkg.native.GAME_KUHN)
    d0, d1 = torch.as_tensor(w0, device="cuda"), torch.as_tensor(w1, device="cuda")
    got = pkg.engine.exploitability(ctx, d0.data_ptr(), d1.data_ptr(), mode)
    want = eo.exploitability(w0, w1, mode, "kuhn")
    for k in ("br0", "br1", "exploitability", "value0"):
        assert got[k] == pytest.approx(want[k], abs=1e-5), k


@pytest.mark.gpu
def test_gpu_kuhn_engine_rollout_matches_oracle(pkg):
    """The fused rollout with game = Kuhn against rollout_oracle's Kuhn lanes."""
    import rollout_oracle as R
    from test_gpu_engine import check_rollout, weights_flat
    N, seed = 2000, 99
    eng = pkg.engine.SelfPlayEngine(n_lanes=N, seed=seed, init_seed=4, eta=0.3, inserts_per_update=1 << 30,
                                    game=pkg.native.GAME_KUHN)
    w = weights_flat(eng)
    eng.rollout()
    ref = R.rollout_with_positions(N, 0, seed, w, (0.06, 0.06), eta=0.3, alias=True, game="kuhn")
    check_rollout(eng, ref)
    st = eng.stats()
    assert np.array_equal(np.array(st["actions"]), ref["actions"])
    assert np.allclose(st["reward"], ref["reward"])


@pytest.mark.gpu
def test_gpu_kuhn_training_lowers_exploitability(pkg):
    """C5's correctness direction: self-play on Kuhn moves the AR nets toward equilibrium."""
    eng = pkg.engine.SelfPlayEngine(n_lanes=8192, rl_capacity=40_000, sl_capacity=40_000, seed=21,
                                    game=pkg.native.GAME_KUHN)
    e0 = eng.exploitability(0)["exploitability"]
    for _ in range(60):
        eng.step()
    e1 = eng.exploitability(0)["exploitability"]
    assert e1 < e0


@pytest.mark.gpu
def test_gpu_kuhn_textbook_beats_the_reference_plateau(pkg):
    """C5 (exploitability -> 0): the reference algorithm plateaus on Kuhn (0.75 chips at 256
    lanes after 40M hands, profiles/r02_kuhn_sweep/ref256.jsonl) because its SL targets are
    the raw BR output and its epsilon is divided by the iteration (agent/agent.py:147-151,253).
    The textbook-NFSP extensions (NFSP_TEXTBOOK) fix both and reach ~0.44 by 5M hands
    (tb256.jsonl).  Bar at a small budget (2M hands, 256 lanes, 3 seeds, same start): the
    textbook mean is at least 0.2 chips below the reference mean."""
    def run(quirks, s):
        eng = pkg.engine.SelfPlayEngine(n_lanes=256, rl_capacity=200_000, sl_capacity=2_000_000,
                                        seed=100 + s, init_seed=s, game=pkg.native.GAME_KUHN,
                                        quirks=quirks)
        for _ in range(2_000_000 // 256):
            eng.step()
        return eng.exploitability(0)["exploitability"]
    ref = [run(pkg.native.QUIRKS_REFERENCE, s) for s in range(3)]
    tb = [run(pkg.native.TEXTBOOK, s) for s in range(3)]
    assert np.mean(tb) <= np.mean(ref) - 0.2, (ref, tb)


@pytest.mark.gpu
def test_gpu_kuhn_c5_exploitability_toward_zero(pkg):
    """C5 at its full size (1,048,576 Kuhn lanes, C3 memories): NFSP with the expected-return
    Q loss (NFSP_TEXTBOOK_MSE) drives the exact exploitability from 1.02 to below 0.15 chips
    in 40 engine steps (42M hands; profiles/r02_textbook_mse/kuhn_c5.jsonl: 0.084 at 42M).
    The Huber-loss variants stay at 0.3-0.44 and the reference algorithm at 0.75
    (Huber's clipped gradient biases Q by up to ~1 chip on bimodal returns)."""
    eng = pkg.engine.SelfPlayEngine(n_lanes=1_048_576, rl_capacity=200_000, sl_capacity=2_000_000,
                                    seed=1234, init_seed=0, game=pkg.native.GAME_KUHN,
                                    quirks=pkg.native.TEXTBOOK_MSE)
    e0 = eng.exploitability(0)["exploitability"]
    for _ in range(40):
        eng.step()
    e1 = eng.exploitability(0)["exploitability"]
    assert e0 > 1.0 and e1 < 0.15, (e0, e1)


@pytest.mark.gpu
def test_gpu_kuhn_c5_sliced_reaches_the_plateau_in_a_third_of_the_hands(pkg):
    """bench.py's C5-textbook form: the same 1,048,576 lanes advanced in 16 pipelined slices
    (cfg.slices 16, slice_lag 2: policy lag 128k hands instead of 1M).  Measured over 4 seeds
    (profiles/r03_kuhn_tb_slices.json): 0.091 +- 0.009 chips after 12 steps (12.6M hands),
    where the one-rollout form is at 0.280 +- 0.076 and needs ~40 steps to reach 0.11.  Bar:
    below 0.13 after 12 steps (one seed; > 4 sigma above the measured mean)."""
    eng = pkg.engine.SelfPlayEngine(n_lanes=1_048_576, rl_capacity=200_000, sl_capacity=2_000_000,
                                    seed=1234, init_seed=0, game=pkg.native.GAME_KUHN,
                                    quirks=pkg.native.TEXTBOOK_MSE, slices=16, slice_lag=2)
    for _ in range(12):
        eng.step()
    e1 = eng.exploitability(0)["exploitability"]
    assert e1 < 0.13, e1


@pytest.mark.gpu
def test_gpu_kuhn_c5_exploitability_below_0_05(pkg):
    """C5's "exploitability -> 0" (BASELINE configs[4]) at full size: 1,048,576 Kuhn lanes in 16
    pipelined slices, textbook NFSP with the MSE Q loss and the reference's decaying epsilon
    (NFSP_TEXTBOOK_MSE_DECAY), lr_ar 0.02.  Measured over 440M hands (profiles/r06/
    kuhn_tb_epsdecay_lrar02.jsonl): 0.022 at 21M hands, 0.012 at 42M, 0.009-0.016 to 440M.  With
    a constant epsilon (NFSP_TEXTBOOK_MSE) the curve stops at 0.06-0.09 at every learning rate
    tried (kuhn_tb_*.jsonl): the epsilon-random BR actions enter M_SL as uniform actions.  The
    reference algorithm is at 0.68 after 440M (kuhn_ref_slices16.jsonl).  Bar: < 0.05 after 24
    steps (25M hands)."""
    nat = pkg.native
    assert nat.TEXTBOOK_MSE_DECAY == 440
    eng = pkg.engine.SelfPlayEngine(n_lanes=1_048_576, rl_capacity=200_000, sl_capacity=2_000_000,
                                    seed=1234, init_seed=0, game=nat.GAME_KUHN, quirks=nat.TEXTBOOK_MSE_DECAY,
                                    slices=16, slice_lag=2, lr_ar=0.02)
    e0 = eng.exploitability(0)["exploitability"]
    for _ in range(24):
        eng.step()
    e1 = eng.exploitability(0)["exploitability"]
    assert e0 > 1.0 and e1 < 0.05, (e0, e1)


@pytest.mark.parametrize("p", [0.55, 0.7])
def test_huber_q_fixed_point_is_not_the_mean(p):
    """Reason of record for the reference algorithm's Kuhn plateau.  Its BR loss
    is Huber (agent/agent.py:91-99): the gradient clamp(e, -1, 1) drives a Q value whose target
    is a +-2-chip showdown won with probability p to the point where E clamp(t - q) = 0, i.e.
    q = 2 - (1 - p) / p for p > 1/2 -- not the mean 4p - 2.  At p = 0.55 that is 1.18 against
    0.2: Q jumps by ~2 chips around p = 1/2, where fictitious play keeps the opponent's mixing.
    The MSE form (NFSP_EXT_MSE_Q) converges to the mean.  The oracle's Keras restatement
    (nn_oracle.MLP, linear head so no unit dies), one observation, the reference's fit."""
    obs = np.zeros((1, nn.N_IN), np.float32)
    obs[0, [0, 13, 24]] = 1.0                     # a history bit, another, a card
    out = {}
    for act in (nn.ACT_LINEAR, nn.ACT_LINEAR_MSE):
        net = nn.MLP(act, rng=np.random.RandomState(3))
        rng = np.random.RandomState(11)
        tail = []
        for u in range(600):
            t = np.where(rng.random_sample((128, 1)) < p, 2.0, -2.0).astype(np.float32) * np.ones((1, 3), np.float32)
            net.fit(np.repeat(obs, 128, axis=0), t, 0.02, shuffle_rng=rng)
            if u >= 400:
                tail.append(float(net.predict(obs)[0].mean()))
        out[act] = float(np.mean(tail))
    assert abs(out[nn.ACT_LINEAR] - (2 - (1 - p) / p)) < 0.1, out
    assert abs(out[nn.ACT_LINEAR_MSE] - (4 * p - 2)) < 0.1, out
