#!/usr/bin/env python3
"""Kuhn policy probe: train the engine on Kuhn (16,384 lanes, C3 memories) and print, per
information state, the AR net's softmax and the BR net's Q-values beside the exact
exploitability.  Information-state observations come from the oracle Env.

    python tests/studies/kuhn_policy.py <quirks> <steps> [cfg_key=value ...]
    e.g. python tests/studies/kuhn_policy.py 120 15000
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import torch, __graft_entry__
import nfsp_oracle as orc, nn_oracle as nn
pkg = __graft_entry__.load_package()
quirks = int(sys.argv[1]); steps = int(sys.argv[2]); extra = dict(kv.split('=') for kv in sys.argv[3:])
cfg = dict(n_lanes=16384, rl_capacity=200000, sl_capacity=2000000, quirks=quirks)
for k, v in extra.items(): cfg[k] = float(v) if '.' in v else int(v)
eng = pkg.engine.SelfPlayEngine(seed=1234, game=pkg.native.GAME_KUHN, **cfg)
for k in range(steps): eng.step()
torch.cuda.synchronize()
print("exploit", eng.exploitability(0), eng.stats()["hands"])
E = np.eye(3)
def obs(dealer, ranks, seq, p):
    e = orc.Env(deal_source=lambda: ranks, game="kuhn"); e.reset(dealer)
    q = dealer
    for a in seq:
        e.step(E[a].reshape(1, 1, 3), q); q = 1 - q
    return e.obs(p).reshape(1, 30)
names = {0: "F", 1: "C", 2: "B"}
for a in (0, 1):
    ar = nn.MLP(nn.ACT_SOFTMAX, 64, weights=nn.unpack_weights(eng.get_weights(a, 0)))
    br = nn.MLP(nn.ACT_LINEAR if quirks & 32 else nn.ACT_RELU, 64, weights=nn.unpack_weights(eng.get_weights(a, 1)))
    for dealer in (0, 1):
        first = dealer == a
        seqs = [[]] if first else [[1], [2]]
        if first: seqs += [[1, 2]]
        for seq in seqs:
            for card in (0, 1, 2):
                other = (card + 1) % 3
                ranks = (card, other, 0) if a == 0 else (other, card, 0)
                x = obs(dealer, ranks, seq, a)
                p = ar.predict(x.reshape(1, 1, 30)).reshape(3)
                q = br.predict(x.reshape(1, 1, 30)).reshape(3)
                print(f"agent {a} {'first ' if first else 'second'} hist {''.join(names[s] for s in seq):3s} card {'AKQ'[card]}: "
                      f"AR F {p[0]:.3f} C {p[1]:.3f} B {p[2]:.3f} | Q {q[0]:+.2f} {q[1]:+.2f} {q[2]:+.2f}")


def memory_probe(eng, agent, dealer, card, seq, p_act=(1, 2)):
    """Mean reward and count of the M_RL transitions of `agent` from the information state
    (dealer, card, history seq) with a call / raise recorded (the last 200k inserts)."""
    import torch
    st = eng.stats()
    m = eng.memories(agent)
    n = int(min(st["rl_total"][agent], eng.cfg.rl_capacity))
    rows = (torch.arange(int(st["rl_total"][agent]) - n, int(st["rl_total"][agent]), device=m["rl_s"].device)
            % m["log_cap"])
    w = torch.ones(30, dtype=torch.int64, device=rows.device) << torch.arange(30, device=rows.device)
    sb = ((m["rl_s"][rows] != 0).long() * w).sum(1).cpu().numpy()
    act = m["rl_a"][rows].argmax(1).cpu().numpy()
    r = m["rl_r"][rows].cpu().numpy()
    other = (card + 1) % 3
    ranks = (card, other, 0) if agent == 0 else (other, card, 0)
    x = obs(dealer, ranks, seq, agent).reshape(30)
    want = int(sum(1 << i for i in range(30) if x[i]))
    sel = (sb == want) & np.isin(act, p_act)
    return int(sel.sum()), float(r[sel].mean()) if sel.any() else None


if len(sys.argv) > 1:
    for a, d in ((0, 0), (1, 1)):
        for card in (1,):
            print("memory", a, "dealer", d, "card K hist CB call:", memory_probe(eng, a, d, card, [1, 2]))

if len(sys.argv) > 1:
    for card in (0, 1, 2):
        counts = [memory_probe(eng, 0, 1, card, [1], p_act=(k,))[0] for k in (0, 1, 2)]
        print("memory agent 0 second (dealer 1) after check, card", "AKQ"[card], "F/C/B counts", counts)

if len(sys.argv) > 1:
    for card in (0, 2):
        for k in (1, 2):
            print("memory agent 0 second (dealer 1) after check, card", "AKQ"[card], "action", "FCB"[k],
                  "(count, mean r):", memory_probe(eng, 0, 1, card, [1], p_act=(k,)))
