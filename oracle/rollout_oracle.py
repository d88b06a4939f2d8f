"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the batched engine's rollout
(``nfsp_rollout``) built from the pinned oracle pieces.

Only tests / smoke / bench's cpu_baseline may import this.  Each lane plays ONE hand of
main.train with ``nfsp_oracle.Env`` and the reference's ``Agent.play`` semantics
(agent/agent.py:130-156, main.py:27-67); the only differences from the sequential
reference are the ones the engine declares (include/nfsp.h, nfsp_engine section):

* randomness comes from Philox4x32-10 (restated here in numpy and checked against the
  Random123 known-answer vectors in tests/test_rollout_oracle.py) instead of CPython's
  ``random`` / ``np.random``, with the engine's counter layout:
    deal      counter (lane, g_lo, g_hi, 0): j5 = below(x,6), j4 = below(y,5), j3 = below(z,4)
              -> the first three swaps of random.shuffle (leduc/deck.py:42-44)
    eta       counter (lane, g_lo, g_hi, 1): x -> dealer, y -> other; BR iff u01 <= eta
    decision  counter (lane, g_lo, g_hi, 2 + k) for the k-th BR decision of the hand:
              x -> eps draw (BR net iff u01 > eps), (y, z, w) -> np.random.rand(1,1,3)
  with below(u, n) = (u * n) >> 32 and u01(u) = (u >> 8) * 2^-24;
* dealer of lane L in rollout g = (L + g) & 1 (the reference alternates per hand);
* lane slices (nfsp_engine_cfg.slices): a rollout plays lanes [lane0, lane0 + n_lanes) of
  the engine's global lane ids, and g is the lanes' hand count (rollouts // slices);
* no updates inside the rollout (the engine's learner runs after it).

Records come out per agent in the engine's canonical order: lane ascending, then play
order within the hand.  RL tuples follow the reference's view aliasing when
``alias`` is set: every tuple of a hand carries the player's LAST pre-action ``s`` and
``a`` of that hand.
"""
from __future__ import annotations

import numpy as np

try:
    from . import nfsp_oracle as orc
    from . import nn_oracle as nn
except ImportError:  # pragma: no cover
    import nfsp_oracle as orc
    import nn_oracle as nn

U32 = np.uint32
M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10, vectorised over numpy uint32 arrays (Salmon et al., SC'11)."""
    c0, c1, c2, c3 = (np.asarray(v, dtype=U32).copy() for v in (c0, c1, c2, c3))
    k0 = np.asarray(k0, dtype=U32).copy()
    k1 = np.asarray(k1, dtype=U32).copy()
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(U32), (p0 & MASK).astype(U32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(U32), (p1 & MASK).astype(U32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = (k0 + W0).astype(U32)
            k1 = (k1 + W1).astype(U32)
    return c0, c1, c2, c3


def below(u, n):
    return int((int(u) * int(n)) >> 32)


def u01(u):
    return float(np.float32((int(u) >> 8) * 5.9604644775390625e-08))


def deal_from_draws(j5, j4, j3):
    d = list(range(6))
    d[5], d[j5] = d[j5], d[5]
    d[4], d[j4] = d[j4], d[4]
    d[3], d[j3] = d[j3], d[3]
    return d[5] >> 1, d[4] >> 1, d[3] >> 1


EXT_SL_ONEHOT, EXT_RESERVOIR, EXT_LINEAR_Q, EXT_EPS_CONST, EXT_SAMPLE_AR = 8, 16, 32, 64, 128   # nfsp.h


class Nets:
    """The four acting heads of a rollout from the engine's packed [2][3][NP] weights."""

    def __init__(self, w_flat, br_act=nn.ACT_RELU):
        w = np.asarray(w_flat, np.float32).reshape(2, 3, -1)
        self.ar = [nn.MLP(nn.ACT_SOFTMAX, 64, weights=nn.unpack_weights(w[a, 0])) for a in (0, 1)]
        self.br = [nn.MLP(br_act, 64, weights=nn.unpack_weights(w[a, 1])) for a in (0, 1)]


def orc_bits(x) -> int:
    v = np.asarray(x).reshape(-1)
    return int(sum(int(v[i] != 0) << i for i in range(30)))


def rollout_with_positions(n_lanes, g, seed, w_flat, eps, eta=0.1, alias=True, rl_before=(0, 0),
                           game="leduc", ext=0, lane0=0):
    """rollout() plus, for each SL record, its global RL stream position (what the engine
    stores in its pending list).  ``ext``: the engine's NFSP_EXT_* bits (include/nfsp.h).
    ``lane0``: global id of the first lane (a slice of a sliced engine)."""
    out = rollout_lanes(n_lanes, g, seed, w_flat, eps, eta, alias, game, ext, lane0)
    rl = ([], [])
    sl = ([], [])
    base = list(rl_before)
    for lane in out["lanes"]:
        for p in (0, 1):
            for (xb, y, local) in lane["sl"][p]:
                sl[p].append((xb, y, base[p] + local))
            rl[p].extend(lane["rl"][p])
            base[p] += len(lane["rl"][p])
    return dict(rl=rl, sl=sl, actions=out["actions"], reward=out["reward"])


def rollout_lanes(n_lanes, g, seed, w_flat, eps, eta=0.1, alias=True, game="leduc", ext=0, lane0=0):
    """Like rollout() but keeps the records per lane (global lanes lane0 .. lane0 + n_lanes)."""
    lanes = []
    actions = np.zeros((2, 3), np.int64)
    reward = np.zeros(2)
    for L in range(lane0, lane0 + n_lanes):
        res = _one_lane(L, g, seed, w_flat, eps, eta, alias, game, ext)
        lanes.append(res)
        actions += res["actions"]
        reward += res["reward"]
    return dict(lanes=lanes, actions=actions, reward=reward)


_NETS_CACHE = {}


def deal_kuhn(j3, j2):
    """nfsp_device.h deal_kuhn: P0 = below(3), P1 = one of the two ranks left."""
    return int(j3), int((j3 + 1 + j2) % 3), 0


def _one_lane(L, g, seed, w_flat, eps, eta, alias, game="leduc", ext=0):
    # the cache holds the weights object itself: an id() alone can be reused by a later
    # array once the first is freed, which would replay lanes with stale nets
    br_act = nn.ACT_LINEAR if ext & EXT_LINEAR_Q else nn.ACT_RELU
    if _NETS_CACHE.get("w") is not w_flat or _NETS_CACHE.get("br_act") != br_act:
        _NETS_CACHE.clear()
        _NETS_CACHE["w"] = w_flat
        _NETS_CACHE["br_act"] = br_act
        _NETS_CACHE["nets"] = Nets(w_flat, br_act)
    nets = _NETS_CACHE["nets"]
    k0, k1 = U32(seed & 0xFFFFFFFF), U32((seed >> 32) & 0xFFFFFFFF)
    glo, ghi = U32(g & 0xFFFFFFFF), U32((g >> 32) & 0xFFFFFFFF)
    one = lambda v: np.array([v], U32)  # noqa: E731
    dx, dy, dz, _ = (v[0] for v in philox4x32(one(L), one(glo), one(ghi), one(0), k0, k1))
    ex, ey, _, _ = (v[0] for v in philox4x32(one(L), one(glo), one(ghi), one(1), k0, k1))
    dealer = (L + g) & 1
    lhand = 1 - dealer
    if game == "kuhn":
        ranks = deal_kuhn(below(dx, 3), below(dy, 2))
    else:
        ranks = deal_from_draws(below(dx, 6), below(dy, 5), below(dz, 4))
    pol_br = [False, False]
    pol_br[dealer] = not (u01(ex) > eta)
    pol_br[lhand] = not (u01(ey) > eta)
    env = orc.Env(deal_source=lambda: ranks, game=game)
    env.reset(dealer)
    hand_rl = []
    n_rl_p = [0, 0]
    sl = ([], [])
    actions = np.zeros((2, 3), np.int64)
    reward = np.zeros(2)
    dec = [0]
    dec_ar = [0]

    def play(p, initial):
        if not initial:
            s, a, r, s2, t = env.get_state(p)
            if np.average(a) != 0:
                hand_rl.append((p, s, a, np.array(s), np.array(a), float(r), np.array(s2), t))
                n_rl_p[p] += 1
            if t:
                reward[p] += float(r)
                return True
        x = env.obs(p).reshape(1, 1, 30)
        if not pol_br[p]:
            y = nets.ar[p].predict(x).reshape(3)
            if ext & EXT_SAMPLE_AR:          # sample the average policy (textbook NFSP)
                c = [v[0] for v in philox4x32(one(L), one(glo), one(ghi), one(0x80000000 + dec_ar[0]), k0, k1)]
                dec_ar[0] += 1
                r = np.float32(u01(c[0]))
                v = 0 if r < y[0] else (1 if r < np.float32(y[0] + y[1]) else 2)
                y = np.eye(3, dtype=np.float32)[v]
        else:
            c = [v[0] for v in philox4x32(one(L), one(glo), one(ghi), one(2 + dec[0]), k0, k1)]
            dec[0] += 1
            if u01(c[0]) > eps[p]:
                y = nets.br[p].predict(x).reshape(3)
            else:
                y = np.array([u01(c[1]), u01(c[2]), u01(c[3])], np.float32)
        env.step(np.asarray(y, np.float64).reshape(1, 1, 3), p)
        if pol_br[p]:
            ysl = np.asarray(y, np.float32).copy()
            if ext & EXT_SL_ONEHOT:          # the action taken (textbook NFSP)
                ysl = np.eye(3, dtype=np.float32)[int(np.argmax(ysl))]
            sl[p].append((orc_bits(x), ysl, n_rl_p[p]))
        actions[p][int(np.argmax(y))] += 1
        return False

    d_t = l_t = False
    first = True
    while not (d_t and l_t):
        rnd = env.round_index
        if not d_t:
            d_t = play(dealer, first)
            first = False
        if not l_t:
            l_t = play(lhand, False)
        if rnd == env.round_index and not d_t:
            d_t = play(dealer, False)
    rl = ([], [])
    for (p, s_v, a_v, s_c, a_c, r, s2, t) in hand_rl:
        s_use, a_use = (s_v, a_v) if alias else (s_c, a_c)
        rl[p].append((orc_bits(s_use), np.asarray(a_use, np.float64).reshape(3).astype(np.float32),
                      r, orc_bits(s2), bool(t)))
    return dict(rl=rl, sl=sl, actions=actions, reward=reward, ranks=ranks, dealer=dealer,
                pol_br=pol_br)
