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
