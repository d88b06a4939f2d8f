"""GPU parity of the fused engine (nfsp_rollout / nfsp_engine_update) against the CPU
oracle (oracle/rollout_oracle.py + nfsp_oracle + nn_oracle).

Bars: observations, rewards, terminal flags, record order, RL stream positions and
reservoir slots bit-exact; action vectors within 1e-6 (softmax expf vs numpy exp);
weights after the learner within 1e-5."""
import numpy as np
import pytest
import torch

import nn_oracle as nn
import rollout_oracle as R
from rollout_oracle import philox4x32

pytestmark = pytest.mark.gpu

U32 = np.uint32


def bits(rows):
    rows = np.asarray(rows)
    assert np.all((rows == 0) | (rows == 1))
    return (rows.astype(np.uint64) << np.arange(30, dtype=np.uint64)).sum(axis=1)


def engine(pkg, **kw):
    return pkg.engine.SelfPlayEngine(**kw)


def weights_flat(eng):
    return np.concatenate([eng.get_weights(a, n) for a in (0, 1) for n in (0, 1, 2)])


def check_rollout(eng, ref, rl_before=(0, 0)):
    for p in (0, 1):
        m = eng.memories(p)
        st = eng.stats()
        n = st["last_rl"][p]
        assert n == len(ref["rl"][p]), (p, n, len(ref["rl"][p]))
        lo = rl_before[p]
        rows = (np.arange(lo, lo + n) % m["log_cap"])
        s = m["rl_s"].cpu().numpy()[rows]
        s2 = m["rl_s2"].cpu().numpy()[rows]
        a = m["rl_a"].cpu().numpy()[rows]
        r = m["rl_r"].cpu().numpy()[rows]
        t = m["rl_t"].cpu().numpy()[rows]
        exp = ref["rl"][p]
        assert np.array_equal(bits(s), np.array([e[0] for e in exp], np.uint64))
        assert np.array_equal(bits(s2), np.array([e[3] for e in exp], np.uint64))
        assert np.abs(a - np.array([e[1] for e in exp])).max() <= 1e-6
        assert np.array_equal(r, np.array([e[2] for e in exp], np.float32))
        assert np.array_equal(t, np.array([e[4] for e in exp], np.uint8))
        k = st["last_sl"][p]
        assert k == len(ref["sl"][p])
        px = m["pend_x"][:k].cpu().numpy().astype(np.uint32)
        pa = m["pend_a"][:k].cpu().numpy()
        pp = m["pend_pos"][:k].cpu().numpy()
        assert np.array_equal(px, np.array([e[0] for e in ref["sl"][p]], np.uint32))
        assert np.abs(pa - np.array([e[1] for e in ref["sl"][p]])).max() <= 1e-6
        assert np.array_equal(pp, np.array([e[2] for e in ref["sl"][p]]))


@pytest.mark.parametrize("quirks", [7, 3, 120, 248])  # 120: one-hot SL, reservoir, linear Q, const eps;
                                                       # 248 = NFSP_TEXTBOOK (+ sampled AR actions)
def test_rollout_matches_oracle(pkg, quirks):
    N, seed = 3000, 1234
    eng = engine(pkg, n_lanes=N, seed=seed, quirks=quirks, init_seed=11, eta=0.3,
                 inserts_per_update=1 << 30)
    w = weights_flat(eng)
    eng.rollout()
    ref = R.rollout_with_positions(N, 0, seed, w, (0.06, 0.06), eta=0.3, alias=bool(quirks & 4), ext=quirks)
    check_rollout(eng, ref)
    st = eng.stats()
    assert np.array_equal(np.array(st["actions"]), ref["actions"])
    assert np.allclose(st["reward"], ref["reward"])
    assert st["hands"] == N
    # second rollout: the RL stream continues where the first ended; g = 1 flips dealers
    eng.update()            # no trigger (inserts_per_update huge): just consumes the inserts
    before = tuple(eng.stats()["rl_total"])
    eng.rollout()
    ref2 = R.rollout_with_positions(N, 1, seed, w, (0.06, 0.06), eta=0.3, alias=bool(quirks & 4),
                                    rl_before=before, ext=quirks)
    check_rollout(eng, ref2, rl_before=before)


def test_learner_first_updates_match_oracle(pkg):
    N, seed = 2048, 77
    probe = engine(pkg, n_lanes=N, seed=seed, init_seed=3, eta=0.5, inserts_per_update=1 << 30)
    probe.rollout()
    n_rl = probe.stats()["last_rl"]
    c = int(min(n_rl))
    assert max(n_rl) < 2 * c          # exactly one trigger per agent
    del probe
    eng = engine(pkg, n_lanes=N, seed=seed, init_seed=3, eta=0.5, inserts_per_update=c)
    w0 = {(a, n): eng.get_weights(a, n) for a in (0, 1) for n in (0, 1, 2)}
    eng.rollout()
    mem = [eng.memories(a) for a in (0, 1)]
    logs = [{k: v.cpu().numpy().copy() for k, v in m.items() if torch.is_tensor(v)} for m in mem]
    eng.set_loss_log(True)
    eng.update()
    st = eng.stats()
    losses = eng.losses()
    for a in (0, 1):
        L = logs[a]
        # ---- BR: targets from the (initial) target net, Huber fit, schedules
        rows, perms = eng.last_update(a, 1)
        assert len(set(rows.tolist())) == 128 and rows.min() >= 0 and rows.max() < c
        br = nn.MLP(nn.ACT_RELU, 64, weights=nn.unpack_weights(w0[(a, 1)]))
        tgt_net = nn.MLP(nn.ACT_RELU, 64, weights=nn.unpack_weights(w0[(a, 2)]))
        s = L["rl_s"][rows]
        s2 = L["rl_s2"][rows]
        act = L["rl_a"][rows]
        r = L["rl_r"][rows].astype(np.float64)
        target = tgt_net.predict(s)
        qn = tgt_net.predict(s2).max(axis=1)
        vals = r + 0.95 * qn.astype(np.float64)          # terminal bootstrap quirk
        expl = float(np.mean(target.max(axis=1).astype(np.float64)))
        for k in range(128):
            target[0][int(np.argmax(act[k]))] = vals[k]    # row-0 quirk
        ep_br = []
        br.fit(s, target, np.float32(0.05), perms=perms, epoch_losses=ep_br)
        got = eng.get_weights(a, 1)
        assert np.abs(got - br.flat()).max() <= 1e-5
        # loss log (the TensorBoard scalars of agent/agent.py:243): Keras epoch losses
        assert losses[f"Player{a}rl/loss_last"] == pytest.approx(ep_br[-1], abs=1e-5)
        assert losses[f"Player{a}rl/loss_mean"] == pytest.approx(np.mean(ep_br), abs=1e-5)
        assert np.abs(eng.get_weights(a, 2) - got).max() == 0     # first update syncs
        assert st["iteration"][a] == 2 and st["br_updates"][a] == 1
        assert st["epsilon"][a] == pytest.approx(0.06 / 2)
        assert st["lr_br"][a] == pytest.approx(0.05 / (1 + 0.003 * np.sqrt(2)), rel=1e-6)
        assert st["temp"][a] == pytest.approx(1 / (1 + 0.02 * np.sqrt(2)))
        assert st["exploitability"][a] == pytest.approx(expl, abs=1e-6)
        # ---- AR: reservoir holds the SL records made before the trigger, CE fit
        k_sl = st["sl_total"][a]
        pos = L["pend_pos"][:k_sl]
        n_before = int((pos <= c).sum())
        rows_ar, perms_ar = eng.last_update(a, 0)
        if n_before > 128:
            assert st["ar_updates"][a] == 1
            assert rows_ar.max() < n_before
            x = np.array([[(int(v) >> f) & 1 for f in range(30)]
                          for v in L["pend_x"][:k_sl].astype(np.uint32)[rows_ar]], np.float32)
            y = L["pend_a"][:k_sl][rows_ar]
            ar = nn.MLP(nn.ACT_SOFTMAX, 64, weights=nn.unpack_weights(w0[(a, 0)]))
            ep_ar = []
            ar.fit(x, y, np.float32(0.1), perms=perms_ar, epoch_losses=ep_ar)
            assert np.abs(eng.get_weights(a, 0) - ar.flat()).max() <= 1e-5
            assert losses[f"Player{a}sl/loss_last"] == pytest.approx(ep_ar[-1], abs=1e-5)
            assert losses[f"Player{a}sl/loss_mean"] == pytest.approx(np.mean(ep_ar), abs=1e-5)
        else:
            assert st["ar_updates"][a] == 0
        assert st["sl_size"][a] == min(k_sl, 40000)


def test_reservoir_replacement_rule(pkg):
    """utils/ReservoirBuffer.py:18-28 with the engine's Philox draws: j = 1 + r % N,
    replace slot j iff j < N (slot 0 is never replaced)."""
    N, seed, cap = 2048, 5, 150
    eng = engine(pkg, n_lanes=N, seed=seed, init_seed=1, eta=0.6, sl_capacity=cap,
                 inserts_per_update=1 << 30)
    eng.rollout()
    pend = [{k: eng.memories(a)[k].cpu().numpy().copy() for k in ("pend_x", "pend_a")}
            for a in (0, 1)]
    n_sl = eng.stats()["last_sl"]
    eng.update()
    for a in (0, 1):
        assert n_sl[a] > cap
        res_x = np.zeros(cap, np.uint64)
        res_a = np.zeros((cap, 3), np.float32)
        for q in range(n_sl[a]):
            if q < cap:
                slot = q
            else:
                c = philox4x32(np.array([0x83000000 | a], U32), np.array([q & 0xFFFFFFFF], U32),
                               np.array([q >> 32], U32), np.array([0], U32),
                               U32(seed), U32(0))
                r64 = (int(c[0][0]) << 32) | int(c[1][0])
                j = 1 + r64 % cap
                slot = j if j < cap else -1
            if slot >= 0:
                res_x[slot] = int(pend[a]["pend_x"][q]) & 0xFFFFFFFF
                res_a[slot] = pend[a]["pend_a"][q]
        m = eng.memories(a)
        assert np.array_equal(bits(m["sl_s"].cpu().numpy()[:cap]), res_x)
        assert np.array_equal(m["sl_a"].cpu().numpy()[:cap], res_a)
        assert eng.stats()["sl_size"][a] == cap


def test_engine_steps_are_deterministic(pkg):
    def run():
        e = engine(pkg, n_lanes=4096, seed=9, init_seed=2, inserts_per_update=64)
        for _ in range(3):
            e.step()
        st = e.stats()
        return st, np.concatenate([e.get_weights(a, n) for a in (0, 1) for n in (0, 1, 2)])
    s1, w1 = run()
    s2, w2 = run()
    assert s1 == s2
    assert np.array_equal(w1, w2)
    assert s1["br_updates"][0] > 10 and s1["ar_updates"][0] > 0


@pytest.mark.gpu
def test_device_views_keep_the_engine_alive(pkg):
    """Zero-copy views (weights, memories) reference the engine: its device memory outlives them."""
    import gc
    import weakref
    eng = pkg.engine.SelfPlayEngine(n_lanes=256, rl_capacity=1000, sl_capacity=1000)
    eng.step()
    w = eng.weights_tensor(0, 0)
    m = eng.memories(0)["rl_s"]
    ref = weakref.ref(eng)
    del eng
    gc.collect()
    assert ref() is not None
    assert torch.isfinite(w).all() and m.shape[1] == 30
    del w, m
    gc.collect()
    assert ref() is None


def test_engine_rejects_unknown_quirk_bits(pkg):
    with pytest.raises(pkg.native.NativeError, match="unknown bits"):
        pkg.engine.SelfPlayEngine(n_lanes=64, quirks=512)
    with pytest.raises(pkg.native.NativeError, match="requires NFSP_EXT_LINEAR_Q"):
        pkg.engine.SelfPlayEngine(n_lanes=64, quirks=pkg.native.EXT_MSE_Q)
    eng = pkg.engine.SelfPlayEngine(n_lanes=64, quirks=pkg.native.QUIRKS_REFERENCE | pkg.native.TEXTBOOK_MSE)
    eng.step()
    assert eng.stats()["hands"] == 64


def test_engine_rejects_step_records_past_the_chains_32_bit_offsets(pkg):
    """k_chain3 reads an agent's step records through a buffer descriptor with 32-bit offsets:
    a slice whose records would pass 2 GiB is refused at creation, before any allocation."""
    with pytest.raises(pkg.native.NativeError, match="exceed 2 GiB"):
        pkg.engine.SelfPlayEngine(n_lanes=1 << 23, inserts_per_update=32)
    eng = pkg.engine.SelfPlayEngine(n_lanes=1 << 23, slices=16, inserts_per_update=32, rl_capacity=1000,
                                    sl_capacity=1000)
    eng.close()
