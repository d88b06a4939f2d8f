"""The reference's self-play driver on top of the drop-in Env / Agent.

``train`` is main.train (main.py:21-75): dealer alternation from ``random.randint``,
eta policy draws (dealer first), the D/L/D scheduler (the dealer acts first in both
rounds), stats every 100 hands after 150.  ``make_main`` is main.main (main.py:127-146)
minus the TF session.  The per-decision work runs through libnfsp; this loop is the
host-side control the reference also runs in Python.
"""
from __future__ import annotations

import random

import numpy as np

from .agent import CFG, Agent
from .leduc import Env
from . import pyrandom


def play_hand(env, players, dealer, eta):
    lhand = 1 - dealer
    env.reset(dealer)
    policy = ["", ""]
    policy[dealer] = "a" if random.random() > eta else "b"
    policy[lhand] = "a" if random.random() > eta else "b"
    d_s = env.get_state(dealer)[3]
    first = True
    d_t = l_t = False
    while not (d_t and l_t):
        rnd = env.round_index
        if not d_t:
            d_t = players[dealer].play(policy[dealer], dealer, d_s if first else None)
            first = False
        if not l_t:
            l_t = players[lhand].play(policy[lhand], lhand)
        if rnd == env.round_index and not d_t:
            d_t = players[dealer].play(policy[dealer], dealer)
    return policy


def train(env, player1, player2, episodes=400000, eta=0.1, stats_every=100, plot: str | None = None):
    """Returns the exploitability-proxy curve main.train plots (main.py:73-75,122).  `plot`:
    a path prefix; the curve is written to <plot>.csv and <plot>.png (main.py:122-123 shows
    it with plt.show() instead)."""
    players = [player1, player2]
    dealer = pyrandom.randint(0, 1)
    curve = []
    for i in range(episodes):
        dealer = 1 - dealer
        play_hand(env, players, dealer, eta)
        if i > 150 and i % stats_every == 0:
            for pl in players:
                pl.sampled_actions()
            curve.append(players[0].average_payoff_br() + players[1].average_payoff_br())
    if plot:
        from .observability import save_curve
        save_curve(curve, plot + ".csv", plot + ".png", xlabel="report")
    return curve


def make_main(cfg=None, init_seed=0, quirks=None, verbose=False):
    c = dict(CFG, **(cfg or {}))
    env = Env(c["seed"], verbose=False)
    np.random.seed(c["seed"])
    rng = np.random.RandomState(init_seed)
    kw = {} if quirks is None else {"quirks": quirks}
    p1 = Agent(None, env.observation_space, env.action_space, "Player0", env, c, rng, **kw)
    p2 = Agent(None, env.observation_space, env.action_space, "Player1", env, c, rng, **kw)
    p1.verbose = p2.verbose = verbose
    return env, p1, p2
