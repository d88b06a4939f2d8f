#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by RUNNING THE REFERENCE in this
(build) container.  Never runs on the GPU box: /root/reference does not exist there,
the committed .npz files travel instead.

How the py2.7 reference is loaded under py3: each module's source is
read as text, a handful of expressions are rewritten in memory (no file is touched),
and the result is executed as a module:

  * ``import ConfigParser``            -> sys.modules alias of ``configparser``
  * implicit relative ``import deck`` / ``import cardmatrix`` -> pre-registered modules
  * py2 integer ``/`` at leduc/deck.py:37, leduc/newenv.py:39,106 -> ``//``
  * the ragged name table at leduc/cardmatrix.py:8-9 -> ``dtype=object`` (numpy >= 1.24)

Keras / TensorFlow / matplotlib are absent; for the rollout trace they are replaced
by stand-ins whose arithmetic is ``oracle/nn_oracle.py``.  That trace therefore pins
the reference's *control flow* (scheduler, play(), buffer traffic, update cadence and
schedules) -- the NN arithmetic itself stays "parity unpinned" against real Keras.

Outputs (all ``numpy.savez_compressed``, no pickles):
  env_kat.npz        exhaustive + random env known-answer table (newenv/deck)
  deal_seq.npz       deals drawn by the reference deck under CPython-3 ``random``
  buffers_trace.npz  ReplayBuffer / ReservoirBuffer insert + sample traces
  rollout_trace.npz  main.train + agent.py event log (hands, get_state, step, inserts,
                     samples, updates, schedules)
  do_action_kat.npz  Env.do_action / game_or_round_has_terminated called directly

Usage: python tests/golden/gen_golden.py   (CWD anywhere; writes next to this file)
"""
from __future__ import annotations

import configparser
import os
import random
import sys
import types
import zlib

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import nn_oracle as nn  # noqa: E402
sys.path.insert(0, HERE)
from tracefmt import Recorder, bits30, crc  # noqa: E402


# ---------------------------------------------------------------------------
# loading the reference
# ---------------------------------------------------------------------------
def _load(name, rel, patches=()):
    path = os.path.join(REF, rel)
    with open(path) as f:
        src = f.read()
    for old, new in patches:
        assert old in src, (rel, old)
        src = src.replace(old, new)
    mod = types.ModuleType(name)
    mod.__file__ = path
    sys.modules[name] = mod
    exec(compile(src, path, "exec"), mod.__dict__)
    return mod


def load_reference_env():
    sys.modules["ConfigParser"] = configparser
    cm = _load("cardmatrix", "leduc/cardmatrix.py",
               [("'Diamonds']])", "'Diamonds']], dtype=object)")])
    dk = _load("deck", "leduc/deck.py", [("self._size / 2", "self._size // 2")])
    ne = _load("newenv", "leduc/newenv.py",
               [("(self.decksize / self.suits)", "(self.decksize // self.suits)")])
    return cm, dk, ne


def load_reference_buffers():
    rb = _load("utils.replay_buffer", "utils/replay_buffer.py")
    rs = _load("utils.ReservoirBuffer", "utils/ReservoirBuffer.py")
    pkg = types.ModuleType("utils")
    pkg.__path__ = []
    pkg.replay_buffer, pkg.ReservoirBuffer = rb, rs
    sys.modules["utils"] = pkg
    return rb, rs


# ---------------------------------------------------------------------------
# Keras / TF / matplotlib stand-ins (arithmetic = oracle/nn_oracle.py)
# ---------------------------------------------------------------------------
STUB_INIT = {"rng": np.random.RandomState(0)}


def install_nn_stubs():
    class _Sym:
        def __init__(self, layers=()):
            self.layers = list(layers)

    class Dense:
        def __init__(self, units, activation=None, **kw):
            self.units, self.activation = units, activation

        def __call__(self, sym):
            return _Sym(sym.layers + [self])

    class _Var:
        def __init__(self, v):
            self.value = np.float32(v)

    class SGD:
        def __init__(self, lr=0.01, **kw):
            self.lr = _Var(lr)

    class Model:
        def __init__(self, inputs=None, outputs=None, name=None):
            d1, d2 = outputs.layers
            act = nn.ACT_RELU if d2.activation == "relu" else nn.ACT_SOFTMAX
            self.mlp = nn.MLP(act, d1.units, STUB_INIT["rng"])

        def compile(self, loss=None, optimizer=None, metrics=None):
            self.opt = optimizer

        def predict(self, x):
            return self.mlp.predict(x)

        def fit(self, x, y, epochs=1, verbose=0, callbacks=None):
            self.mlp.fit(x, y, self.opt.lr.value, epochs=epochs)

        def get_weights(self):
            return self.mlp.get_weights()

        def set_weights(self, ws):
            self.mlp.set_weights(ws)

    def mk(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    mk("keras.models", Sequential=object, Model=Model)
    mk("keras.layers.advanced_activations", LeakyReLU=object)
    layers = mk("keras.layers", Dense=Dense, Input=lambda shape=None, name=None: _Sym())
    layers.advanced_activations = sys.modules["keras.layers.advanced_activations"]
    mk("keras.optimizers", Adam=SGD, SGD=SGD)
    mk("keras.callbacks", TensorBoard=lambda **kw: None)
    mk("keras.backend", set_value=lambda var, v: setattr(var, "value", np.float32(v)),
       cast=lambda x, t: x)
    keras = mk("keras")
    keras.__path__ = []

    class _Sess:
        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

        def run(self, *a, **k):
            return None

    mk("tensorflow", Session=_Sess, set_random_seed=lambda s: None,
       global_variables_initializer=lambda: None)
    plt = mk("matplotlib.pyplot", plot=lambda *a, **k: None, show=lambda *a, **k: None)
    mpl = mk("matplotlib")
    mpl.pyplot = plt


def load_reference_main():
    cm, dk, ne = load_reference_env()
    rb, rs = load_reference_buffers()
    install_nn_stubs()
    leduc = types.ModuleType("leduc")
    leduc.__path__ = []
    leduc.newenv = ne
    sys.modules["leduc"] = leduc
    sys.modules["leduc.newenv"] = ne
    ag = _load("agent.agent", "agent/agent.py")
    agpkg = types.ModuleType("agent")
    agpkg.__path__ = []
    agpkg.agent = ag
    sys.modules["agent"] = agpkg
    mn = _load("refmain", "main.py")
    mn.time = types.SimpleNamespace(sleep=lambda s: None)
    return dk, ne, rb, rs, ag, mn


# ---------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------
def rigged_shuffle(ranks):
    """A replacement for deck.rshuffle whose three pops yield (P0, P1, public)."""
    def shuf(cards):
        pool = list(cards)
        picked = []
        for r in ranks:
            k = next(i for i, c in enumerate(pool) if c.rank == r)
            picked.append(pool.pop(k))
        cards[:] = pool + picked[::-1]
    return shuf


RANK_TRIPLES = [(a, b, c) for a in range(3) for b in range(3) for c in range(3)
                if not (a == b == c)]


# ---------------------------------------------------------------------------
# 1. env KAT
# ---------------------------------------------------------------------------
class NeedMore(Exception):
    pass


def snapshot(env, out):
    for p in (0, 1):
        s, a, r, s2, t = env.get_state(p)
        out.append((p, bits30(s), np.asarray(a, np.float64).reshape(3).copy(),
                    float(r), isinstance(r, (int,)) and not isinstance(r, bool),
                    bits30(s2), bool(t), int(env.round_index)))


def drive_hand(env, dealer, vecs, extra_step=None):
    """Run one hand under the main.train D/L/D scheduler (observe -> act), with the
    decision vectors ``vecs``; snapshot both players after reset and every step."""
    snaps, steps = [], []
    env.reset(dealer)
    snapshot(env, snaps)
    k = [0]

    def play(p, initial):
        if not initial and env.get_state(p)[4]:
            return True
        if k[0] >= len(vecs):
            raise NeedMore()
        env.step(np.asarray(vecs[k[0]], dtype=np.float64).reshape(1, 1, 3), p)
        steps.append(p)
        k[0] += 1
        snapshot(env, snaps)
        return False

    lh = 1 - dealer
    d_t = l_t = False
    first = True
    while not (d_t and l_t):
        rnd = env.round_index
        if not d_t:
            d_t = play(dealer, first)
            first = False
        if not l_t:
            l_t = play(lh, False)
        if rnd == env.round_index and not d_t:
            d_t = play(dealer, False)
    if k[0] != len(vecs):
        raise ValueError("unused actions")
    if extra_step is not None:                     # step after termination
        p, v = extra_step
        env.step(np.asarray(v, dtype=np.float64).reshape(1, 1, 3), p)
        steps.append(p)
        snapshot(env, snaps)
    return steps, snaps


def gen_env_kat(dk, ne):
    os.chdir(REF)
    env = ne.Env()
    onehot = np.eye(3)
    hands = []            # (dealer, r0, r1, rp, steps, vecs, snaps)

    def enum(dealer, ranks, prefix):
        dk.rshuffle = rigged_shuffle(ranks)
        try:
            steps, snaps = drive_hand(env, dealer, [onehot[i] for i in prefix])
        except NeedMore:
            for i in range(3):
                enum(dealer, ranks, prefix + [i])
            return
        hands.append((dealer, ranks, steps, [onehot[i] for i in prefix], snaps))

    for dealer in (0, 1):
        for ranks in RANK_TRIPLES:
            enum(dealer, ranks, [])
    n_exhaustive = len(hands)

    # random hands: fp32-representable vectors incl. ties, all-zero vectors, and a
    # step after termination
    rng = np.random.RandomState(20240607)
    levels = np.array([0.0, 0.25, 0.5, 0.75, 1.0])
    for h in range(4000):
        dealer = int(rng.randint(2))
        ranks = RANK_TRIPLES[rng.randint(len(RANK_TRIPLES))]
        dk.rshuffle = rigged_shuffle(ranks)
        vecs = []
        while True:
            try:
                extra = None
                if rng.rand() < 0.15:
                    extra = (int(rng.randint(2)), np.float32(rng.rand(3)).astype(np.float64))
                steps, snaps = drive_hand(env, dealer, vecs, extra)
                break
            except NeedMore:
                if rng.rand() < 0.5:
                    v = levels[rng.randint(5, size=3)]
                else:
                    v = np.float32(rng.rand(3)).astype(np.float64)
                vecs.append(v)
        if extra is not None:
            vecs = vecs + [extra[1]]
        hands.append((dealer, ranks, steps, vecs, snaps))

    H = len(hands)
    MAXS = 7
    dealer = np.array([h[0] for h in hands], np.uint8)
    ranks = np.array([h[1] for h in hands], np.uint8)
    nsteps = np.array([len(h[2]) for h in hands], np.uint8)
    step_p = np.full((H, MAXS), 255, np.uint8)
    step_v = np.zeros((H, MAXS, 3), np.float32)
    for i, h in enumerate(hands):
        step_p[i, :len(h[2])] = h[2]
        step_v[i, :len(h[3])] = np.asarray(h[3], np.float32)
        assert np.array_equal(np.asarray(h[3], np.float32).astype(np.float64), np.asarray(h[3]))
    snap_off = np.zeros(H + 1, np.int64)
    rows = []
    for i, h in enumerate(hands):
        rows.extend(h[4])
        snap_off[i + 1] = len(rows)
    snap = dict(
        p=np.array([r[0] for r in rows], np.uint8),
        s=np.array([r[1] for r in rows], np.uint32),
        a=np.array([r[2] for r in rows], np.float64),
        r=np.array([r[3] for r in rows], np.float64),
        r_is_int=np.array([r[4] for r in rows], np.uint8),
        s2=np.array([r[5] for r in rows], np.uint32),
        t=np.array([r[6] for r in rows], np.uint8),
        rnd=np.array([r[7] for r in rows], np.uint8),
    )
    np.savez_compressed(os.path.join(HERE, "env_kat.npz"), dealer=dealer, ranks=ranks,
                        nsteps=nsteps, step_p=step_p, step_v=step_v, snap_off=snap_off,
                        n_exhaustive=np.int64(n_exhaustive),
                        **{"snap_" + k: v for k, v in snap.items()})
    term = snap["t"][snap_off[1:] - 1] == 1
    print(f"env_kat: {H} hands ({n_exhaustive} exhaustive), {len(rows)} snapshots, "
          f"all terminal={bool(term.all())}")


# ---------------------------------------------------------------------------
# 2. deal sequences under CPython-3 random
# ---------------------------------------------------------------------------
def gen_deal_seq(dk, ne):
    os.chdir(REF)
    dk.rshuffle = random.shuffle
    out = {}
    for seed in (1234, 7, 99):
        random.seed(seed)
        env = ne.Env()
        deals = []
        for i in range(2000):
            env.reset(i & 1)
            p0 = int(np.argmax(env.specific_cards[0][0]))
            p1 = int(np.argmax(env.specific_cards[1][0]))
            pub = int(env.deck.pick_up().rank)
            deals.append((p0, p1, pub))
            # the extra pick_up above consumed no RNG; the deck is rebuilt each reset
        out[f"seed{seed}"] = np.array(deals, np.uint8)
    np.savez_compressed(os.path.join(HERE, "deal_seq.npz"), **out)
    print("deal_seq:", {k: v.shape for k, v in out.items()})


# ---------------------------------------------------------------------------
# 3. buffer traces
# ---------------------------------------------------------------------------
def gen_buffers(rb, rs):
    rec = {}
    # ReplayBuffer: cap 50, 180 inserts, sample 16 every 25 inserts (and a short one)
    buf = rb.ReplayBuffer(50, 7)
    samples = []
    for i in range(180):
        s = np.full((1, 30), float(i))
        buf.add(s, np.full((1, 1, 3), i + 0.5), float(i % 3), s + 1000.0, bool(i % 4 == 0))
        if i in (5, 24, 49, 50, 74, 99, 124, 149, 179):
            sb, ab, rbt, s2b, tb = buf.sample_batch(16)
            samples.append((i, sb[:, 0, 0].astype(np.int64), ab[:, 0, 0], rbt, s2b[:, 0, 0],
                            tb.astype(np.uint8)))
    rec["rl_at"] = np.array([x[0] for x in samples])
    rec["rl_len"] = np.array([len(x[1]) for x in samples])
    rec["rl_ids"] = np.concatenate([x[1] for x in samples])
    rec["rl_a"] = np.concatenate([x[2] for x in samples])
    rec["rl_r"] = np.concatenate([x[3] for x in samples])
    rec["rl_s2"] = np.concatenate([x[4] for x in samples])
    rec["rl_t"] = np.concatenate([x[5] for x in samples])
    rec["rl_final"] = np.array([e[0][0, 0] for e in buf.buffer], np.int64)
    # ReservoirBuffer: cap 40, 300 inserts, sample 12 at a few points
    res = rs.ReservoirBuffer(40, 11)
    samples = []
    for i in range(300):
        res.add(np.full((1, 1, 30), float(i)), np.full((1, 1, 3), i * 0.25))
        if i in (3, 39, 40, 99, 199, 299):
            sb, ab = res.sample_batch(12)
            samples.append((i, sb[:, 0, 0].astype(np.int64), ab[:, 0, 0]))
    rec["sl_at"] = np.array([x[0] for x in samples])
    rec["sl_len"] = np.array([len(x[1]) for x in samples])
    rec["sl_ids"] = np.concatenate([x[1] for x in samples])
    rec["sl_a"] = np.concatenate([x[2] for x in samples])
    rec["sl_final"] = np.array([e[0][0, 0] for e in res.buffer], np.int64)
    np.savez_compressed(os.path.join(HERE, "buffers_trace.npz"), **rec)
    print("buffers_trace:", {k: v.shape for k, v in rec.items()})


# ---------------------------------------------------------------------------
# 4. rollout trace: event log of main.train + agent.py (format: tracefmt.py)
# ---------------------------------------------------------------------------
ROLLOUT_EPISODES = 2500
ROLLOUT_INIT_SEED = 5


def gen_rollout(dk, ne, rb, rs, ag, mn):
    os.chdir(REF)
    dk.rshuffle = random.shuffle
    rec = Recorder()
    rec.wrap_classes(ne.Env, rb.ReplayBuffer, rs.ReservoirBuffer, ag.Agent)
    STUB_INIT["rng"] = np.random.RandomState(ROLLOUT_INIT_SEED)
    mn.Config.set("Common", "Episodes", str(ROLLOUT_EPISODES))
    import io
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        mn.main({"human": False})
    code, who, pay = rec.arrays()
    np.savez_compressed(os.path.join(HERE, "rollout_trace.npz"), code=code, who=who, pay=pay,
                        episodes=np.int64(ROLLOUT_EPISODES),
                        init_seed=np.int64(ROLLOUT_INIT_SEED))
    counts = {c: int((code == c).sum()) for c in range(10)}
    print("rollout_trace:", len(code), "events", counts)


# ---------------------------------------------------------------------------
# 5. do_action / game_or_round_has_terminated called directly
# ---------------------------------------------------------------------------
DO_VECS = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [0, 0.5, 0.5], [1, 0, 1]], np.float64)


def gen_do_action(dk, ne):
    """leduc/newenv.py:131-190 called directly (not through step): every sequence of 1..3
    do_action calls (vectors DO_VECS, players alternating from the dealer) from a fresh
    hand (round 0) and from round 1 (reached by step([C]), step([C])), both dealers.  Per
    call: do_action's return, game_or_round_has_terminated() (1 True, 0 False, -1 None),
    and the env state it changed."""
    import itertools
    os.chdir(REF)
    env = ne.Env()
    rows = dict(hand=[], dealer=[], pre=[], p=[], vec=[], fold=[], status=[], hist=[], pot_half=[],
                raises=[], round_raises=[], la=[])
    h = 0
    for dealer in (0, 1):
        for pre in (0, 1):
            for L in (1, 2, 3):
                for seq in itertools.product(range(len(DO_VECS)), repeat=L):
                    dk.rshuffle = rigged_shuffle((0, 1, 2))
                    env.reset(dealer)
                    p = dealer
                    if pre:
                        env.step(DO_VECS[1].reshape(1, 1, 3), p)
                        env.step(DO_VECS[1].reshape(1, 1, 3), 1 - p)
                        assert env.round_index == 1 and not env.terminated
                    for v in seq:
                        f = env.do_action(DO_VECS[v].reshape(1, 1, 3), p)
                        st = env.game_or_round_has_terminated()
                        flat = env.history.flatten()
                        rows["hand"].append(h); rows["dealer"].append(dealer); rows["pre"].append(pre)
                        rows["p"].append(p); rows["vec"].append(v); rows["fold"].append(bool(f))
                        rows["status"].append(1 if st is True else (-1 if st is None else 0))
                        rows["hist"].append(sum(1 << i for i in range(24) if flat[i]))
                        rows["pot_half"].append([int(round(2 * x)) for x in env.overall_raises])
                        rows["raises"].append([int(x) for x in env.raises])
                        rows["round_raises"].append(int(env.round_raises))
                        rows["la"].append(np.array(env.last_action[p], np.float64).reshape(3))   # a copy
                        p = 1 - p
                    h += 1
    out = {k: np.asarray(v) for k, v in rows.items()}
    out["vecs"] = DO_VECS
    np.savez_compressed(os.path.join(HERE, "do_action_kat.npz"), **out)
    print(f"do_action_kat: {h} sequences, {len(rows['hand'])} calls, "
          f"status counts {np.unique(out['status'], return_counts=True)}")


def main():
    import contextlib
    import io
    os.chdir(REF)                      # the reference reads ./config.ini at import time
    dk, ne, rb, rs, ag, mn = load_reference_main()
    with contextlib.redirect_stdout(io.StringIO()):   # the env's "tried to step" prints
        gen_env_kat(dk, ne)
    gen_deal_seq(dk, ne)
    gen_buffers(rb, rs)
    gen_rollout(dk, ne, rb, rs, ag, mn)


if __name__ == "__main__":
    if sys.argv[1:] == ["do_action"]:           # only the do_action fixture
        os.chdir(REF)
        _dk, _ne = load_reference_env()[1:]
        gen_do_action(_dk, _ne)
    else:
        main()
