"""TEST INFRASTRUCTURE ONLY -- the engine's learner step (csrc/learner.hip, nfsp_engine_update)
restated in numpy, so one whole engine step can be replayed update by update.

Only ``tests/`` imports this module; it is a checker, never the thing measured or shipped.

What it restates (the reference semantics each piece follows):

* the trigger plan: update_strategy once per ``c`` RL inserts of an agent (the
  ``game_step % 128`` trigger, agent/agent.py:153-154).  Trigger m fires at RL stream
  position p_m = m c.  A BR update needs min(p_m, capacity) > batch (agent/agent.py:211);
* BR (agent/agent.py:209-253):
  * rows: 128 distinct M_RL rows from the window [p_m - min(p_m, cap), p_m), i.e. the FIFO
    as it was at the trigger.  They are drawn by Philox(TAG_SAMPLE | dbg, m, (attempt << 8)
    | b); a duplicate of an earlier pick redraws with the next attempt;
  * targets: from the target net.  The TD value r + gamma q_next is evaluated in double:
    py2 / numpy 1.x promote ``gamma * np.float32`` to float64.  (nfsp_oracle, run under
    numpy 2, gets a float32 product, NEP 50; the two differ in the last bit of a target.)
    The quirks (TERMINAL_BOOTSTRAP, ROW0_TARGET) are flag-gated;
  * proxy: the mean of the row maxima, in double;
  * fit: Keras fit with 2 epochs of 32-row minibatches.  The epoch permutation ranks the
    Philox(TAG_PERM | dbg, m, (e << 8) | b) keys;
  * lr = lr0 / (1 + 0.003 sqrt(iteration)), as float32, with iteration = it0 + 2u;
  * target sync after the fit when target_count % every == 0;
  * eps = eps / iteration, temp = 1 / (1 + 0.02 sqrt(iteration));
* AR (agent/agent.py:255-264): M_SL as it was at the trigger.  That is its size then, and
  each slot's content then: the latest SL insert of this rollout made at or before the
  trigger, else the pre-rollout reservoir row.  The not-quite reservoir
  (utils/ReservoirBuffer.py:18-28) draws j = 1 + r % N from Philox(TAG_RES | a, total, 0)
  and replaces iff j < N.  128 distinct slots, then the same fit as BR (lr_ar, CE).

Network arithmetic is nn_oracle's (parity with the GPU chain within a tolerance: the chain
sums exact products on bf16 matrix cores, numpy uses BLAS).
"""
from __future__ import annotations

import math

import numpy as np

import nn_oracle as nn
from rollout_oracle import philox4x32

TAG_SAMPLE, TAG_PERM, TAG_RES = 0x81000000, 0x82000000, 0x83000000
QUIRK_TERMINAL_BOOTSTRAP, QUIRK_ROW0_TARGET = 1, 2
M32 = 0xFFFFFFFF


def _ph(stream, m, low, k0, k1):
    """Philox4x32-10 at counters (stream, m_lo, m_hi, low[i]) -> (x, y) arrays."""
    low = np.asarray(low, np.uint32)
    n = low.shape[0]
    x, y, _, _ = philox4x32(np.full(n, stream, np.uint32), np.full(n, m & M32, np.uint32),
                            np.full(n, (m >> 32) & M32, np.uint32), low, k0, k1)
    return x.astype(np.uint64), y.astype(np.uint64)


def sample_distinct(batch, lo, win, stream, m, k0, k1):
    """learner sample_distinct: batch distinct positions in [lo, lo + win)."""
    cand = np.zeros(batch, np.int64)
    attempt = np.zeros(batch, np.uint32)
    redraw = np.ones(batch, bool)
    while True:
        idx = np.nonzero(redraw)[0]
        if len(idx):
            x, y = _ph(stream, m, (attempt[idx] << 8) | idx.astype(np.uint32), k0, k1)
            r64 = (x << np.uint64(32)) | y
            cand[idx] = lo + (r64 % np.uint64(win)).astype(np.int64)
            attempt[idx] += 1
        dup = np.array([bool(np.any(cand[:b] == cand[b])) for b in range(batch)])
        if not dup.any():
            return cand
        redraw = dup


def draw_perm(batch, e, stream, m, k0, k1):
    """Keras fit's per-epoch shuffle: perm[rank] = b, rank = order of the key of b."""
    b = np.arange(batch, dtype=np.uint32)
    x, _ = _ph(stream, m, (np.uint32(e) << 8) | b, k0, k1)
    key = (x.astype(np.uint32) & np.uint32(0xFFFFFF00)) | b
    perm = np.empty(batch, np.int64)
    perm[np.argsort(key, kind="stable")] = np.arange(batch)      # rank of each b
    out = np.empty(batch, np.int64)
    out[perm] = np.arange(batch)
    return out


EXT_RESERVOIR, EXT_LINEAR_Q, EXT_EPS_CONST = 16, 32, 64      # include/nfsp.h NFSP_EXT_*
EXT_MSE_Q = 256


def reservoir_slots(a, sl_total0, n_sl, cap, k0, k1, ext=0):
    """Slot of each SL insert of the rollout (-1: not stored).  ext & EXT_RESERVOIR: a true
    reservoir (Algorithm R, j = U{0..tot}) instead of the reference's randrange(1, N + 1)."""
    slots = np.empty(n_sl, np.int64)
    for q in range(n_sl):
        tot = sl_total0 + q
        if tot < cap:
            slots[q] = tot
        else:
            x, y, _, _ = philox4x32(np.uint32(TAG_RES | a), np.uint32(tot & M32), np.uint32((tot >> 32) & M32),
                                    np.uint32(0), k0, k1)
            r64 = (int(x) << 32) | int(y)
            j = r64 % (tot + 1) if ext & EXT_RESERVOIR else 1 + r64 % cap
            slots[q] = j if j < cap else -1
    return slots


def bits_to_x(bits):
    bits = np.asarray(bits, np.int64).reshape(-1)
    return ((bits[:, None] >> np.arange(30)) & 1).astype(np.float32)


def ar_minibatches(cfg, state, a, quirks=7, slots=None, build_below=None):
    """The AR updates of agent a's learner call, in order: yields (u, bits [B], targets [B, 3],
    perms [E, B]) -- M_SL as of the trigger (k_ar_prep) -- or (u, None, None, None) for an
    update skipped because M_SL holds <= batch records.  The inputs of an AR update do not
    depend on the weights, so any stretch of the chain can be replayed from given weights.
    build_below: only updates u < build_below get their minibatch drawn; later active ones
    yield (u, True, None, None) (a replayed prefix only needs their count)."""
    c, B, E = cfg["c"], cfg["batch"], cfg["epochs"]
    k0, k1 = cfg["seed"] & M32, (cfg["seed"] >> 32) & M32
    st = state[a]
    P0 = st["rl_total"] - st["last_rl"]
    m_first = P0 // c + 1
    m_last = (P0 + st["last_rl"]) // c
    U = max(0, m_last - m_first + 1)
    n_sl = st["last_sl"]
    sl0 = st["sl_total"] - n_sl
    cap = cfg["sl_capacity"]
    if slots is None:
        slots = reservoir_slots(a, sl0, n_sl, cap, k0, k1, quirks)
    pos = np.asarray(st["pend_pos"][:n_sl], np.int64)
    # each slot's inserts of this rollout in insert order: the latest one before a
    # trigger is a bisection (slot contents as of the trigger)
    order = np.argsort(slots, kind="stable")
    ss = slots[order]
    for u in range(U):
        m = m_first + u
        pm = m * c
        nb = int(np.searchsorted(pos, pm, side="right"))
        count = min(sl0 + nb, cap)
        if count <= B:
            yield u, None, None, None
            continue
        if build_below is not None and u >= build_below:
            yield u, True, None, None
            continue
        picks = sample_distinct(B, 0, count, TAG_SAMPLE | (a * 2), m, k0, k1)
        xb = np.empty(B, np.int64)
        ya = np.empty((B, 3), np.float32)
        for b, j in enumerate(picks):
            lo, hi = np.searchsorted(ss, j, side="left"), np.searchsorted(ss, j, side="right")
            qs = order[lo:hi]                           # this slot's inserts, ascending
            k = int(np.searchsorted(qs, nb, side="left"))
            if k:
                q = qs[k - 1]
                xb[b], ya[b] = st["pend_x"][q], st["pend_a"][q]
            else:
                xb[b], ya[b] = st["sl_s_bits"][j], st["sl_a"][j]
        perms = np.stack([draw_perm(B, e, TAG_PERM | (a * 2), m, k0, k1) for e in range(E)])
        yield u, xb, ya, perms


def learner_step(cfg, state, quirks=7, max_updates=None, trace=None):
    """Replay nfsp_engine_update.

    cfg: dict(c, batch, epochs, rl_capacity, sl_capacity, target_every, lr_br, lr_ar, gamma,
         seed).
    state[a]: the engine after the rollout, before the update:
      * w: {0: AR, 1: BR, 2: target} flat weights;
      * rl_total, last_rl, sl_total, last_sl, iteration, br_updates, epsilon;
      * rl_s_bits, rl_s2_bits, rl_a, rl_r, rl_t: M_RL log rows (row = insert % log_cap);
      * sl_s_bits, sl_a: the reservoir before the rollout's inserts;
      * pend_x, pend_a, pend_pos: the rollout's SL inserts.
    Returns per agent: weights, iteration, epsilon, lr_br, temp, exploitability (last BR
    proxy), br_updates, ar_updates, reservoir (bits, a) after the update.
    max_updates: replay only the first max_updates BR and AR updates of each agent (the
    engine's nfsp_engine_set_update_limit); the counters still follow the full plan.
    trace(a, net, u, flat_weights): called after each replayed update u (net 0 = AR, 1 = BR).
    """
    c, B, E = cfg["c"], cfg["batch"], cfg["epochs"]
    k0, k1 = cfg["seed"] & M32, (cfg["seed"] >> 32) & M32
    out = []
    for a in (0, 1):
        st = state[a]
        P0 = st["rl_total"] - st["last_rl"]
        m_first = P0 // c + 1
        m_last = (P0 + st["last_rl"]) // c
        U = max(0, m_last - m_first + 1)
        m_br0 = max(m_first, B // c + 1)
        U_br = max(0, m_last - m_br0 + 1)
        log_cap = len(st["rl_s_bits"])
        ar = nn.MLP(nn.ACT_SOFTMAX, 64, weights=nn.unpack_weights(st["w"][0]))
        br_act = (nn.ACT_LINEAR_MSE if quirks & EXT_MSE_Q else nn.ACT_LINEAR) if quirks & EXT_LINEAR_Q \
            else nn.ACT_RELU
        br = nn.MLP(br_act, 64, weights=nn.unpack_weights(st["w"][1]))
        tg = nn.MLP(br_act, 64, weights=nn.unpack_weights(st["w"][2]))
        it, tc, eps = st["iteration"], st["br_updates"], st["epsilon"]
        it0 = it
        expl = None
        lim = lambda n: n if max_updates is None else min(n, max_updates)
        # ---- BR updates
        for u in range(lim(U_br)):
            m = m_br0 + u
            pm = m * c
            win = min(pm, cfg["rl_capacity"])
            rows = sample_distinct(B, pm - win, win, TAG_SAMPLE | (a * 2 + 1), m, k0, k1) % log_cap
            s, s2 = bits_to_x(st["rl_s_bits"][rows]), bits_to_x(st["rl_s2_bits"][rows])
            act = np.argmax(st["rl_a"][rows], axis=1)
            r = st["rl_r"][rows].astype(np.float64)
            t = st["rl_t"][rows].astype(bool)
            target = tg.predict(s).astype(np.float32)
            qn = tg.predict(s2).max(axis=1).astype(np.float64)
            terminal = t & (not (quirks & QUIRK_TERMINAL_BOOTSTRAP))
            vals = np.where(terminal, r, r + cfg["gamma"] * qn).astype(np.float32)
            expl = float(np.sum(target.max(axis=1).astype(np.float64)) / B)
            for k in range(B):
                target[0 if quirks & QUIRK_ROW0_TARGET else k][act[k]] = vals[k]
            lr = np.float32(cfg["lr_br"] / (1.0 + 0.003 * math.sqrt(it0 + 2 * u)))
            perms = np.stack([draw_perm(B, e, TAG_PERM | (a * 2 + 1), m, k0, k1) for e in range(E)])
            br.fit(s, target, lr, epochs=E, perms=perms)
            if (tc + u) % cfg["target_every"] == 0:
                tg.set_weights(br.get_weights())
            if trace is not None:
                trace(a, 1, u, br.flat())
            it += 2
            eps = cfg["epsilon"] if quirks & EXT_EPS_CONST else eps / it
        for u in range(lim(U_br), U_br):      # schedules of updates past the prefix
            it += 2
            eps = cfg["epsilon"] if quirks & EXT_EPS_CONST else eps / it
        # ---- AR updates, the reservoir as of each trigger
        n_sl = st["last_sl"]
        sl0 = st["sl_total"] - n_sl
        cap = cfg["sl_capacity"]
        slots = reservoir_slots(a, sl0, n_sl, cap, k0, k1, quirks)
        n_ar = 0
        for u, xb, ya, perms in ar_minibatches(cfg, state, a, quirks, slots, build_below=lim(U)):
            if xb is None:
                continue
            n_ar += 1
            if u >= lim(U):
                continue
            ar.fit(bits_to_x(xb), ya, np.float32(cfg["lr_ar"]), epochs=E, perms=perms)
            if trace is not None:
                trace(a, 0, u, ar.flat())
        # ---- the reservoir after the rollout's inserts (last writer per slot)
        res_x = np.array(st["sl_s_bits"], np.int64).copy()
        res_a = np.array(st["sl_a"], np.float32).copy()
        for q in range(n_sl):
            if slots[q] >= 0:
                res_x[slots[q]] = st["pend_x"][q]
                res_a[slots[q]] = st["pend_a"][q]
        out.append(dict(
            w={0: ar.flat(), 1: br.flat(), 2: tg.flat()}, iteration=it, epsilon=eps,
            lr_br=float(np.float32(cfg["lr_br"] / (1.0 + 0.003 * math.sqrt(it)))),
            temp=1.0 / (1.0 + 0.02 * math.sqrt(it)) if U_br else None,
            exploitability=expl, br_updates=st["br_updates"] + U_br, ar_updates=n_ar,
            U=U, U_br=U_br, res_x=res_x, res_a=res_a))
    return out
