#!/usr/bin/env python3
"""Where does textbook NFSP's Kuhn plateau come from?  

Trains the engine on Kuhn (textbook extensions, low policy lag) and reports, at each
checkpoint, with the brute-force evaluator (oracle/exploit_oracle.py):
* expl        exploitability of the AR pair (softmax mixed strategies): BR_0 + BR_1;
* br_gap[i]   how far agent i's learned best response (the BR net's greedy policy) is from a
              true best response to the opponent's AR policy: BR_i - value of greedy(BR_i);
* anticip[i]  the same gap against the opponent's eta-mixture (eta BR + (1 - eta) AR), the
              policy NFSP's RL part actually faces;
* sl_gap[i]   how far the AR net is from the average of the BR policies: the L1 distance
              between the AR softmax and the greedy BR action, per information state
              (a one-sample proxy of the time average).

    python tests/studies/kuhn_diag.py --hands 40000000 --every 5000000 > profiles/r02_kuhn_diag.jsonl
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


class Mix:
    """eta * a + (1 - eta) * b, as an exploit_oracle policy."""
    def __init__(self, a, b, eta):
        self.a, self.b, self.eta = a, b, eta

    def probs(self, obs, legal):
        return self.eta * np.asarray(self.a.probs(obs, legal)) + (1 - self.eta) * np.asarray(self.b.probs(obs, legal))


def seat_value(i, pol_i, pol_o):
    import exploit_oracle as eo
    v0 = eo.on_policy_value0(pol_i if i == 0 else pol_o, pol_o if i == 0 else pol_i, game="kuhn")
    return v0 if i == 0 else -v0


def true_q(i, pol_o):
    """Q*(I, a) of seat i against pol_o: the expected return of taking a at information set
    I and best-responding afterwards, per unit of reach (exploit_oracle.best_response's
    recursion, keeping every action's value)."""
    import exploit_oracle as eo
    from collections import defaultdict
    out = {}

    def expand(entries):
        total, groups, stack = 0.0, defaultdict(list), list(entries)
        while stack:
            deal, dealer, acts, w = stack.pop()
            r = eo.replay(deal, dealer, acts, "kuhn")
            if r[0] == "terminal":
                total += w * float(r[1][i])
                continue
            _, seat, obs, legal = r
            if seat == i:
                groups[obs].append((deal, dealer, acts, w, legal))
                continue
            pr = pol_o.probs(obs, legal)
            for a in eo._legal_actions(legal):
                if pr[a] > 0.0:
                    stack.append((deal, dealer, acts + [a], w * pr[a]))
        return total, groups

    def value(obs, group):
        reach = sum(g[3] for g in group)
        vals = {}
        for a in eo._legal_actions(group[0][4]):
            t, g = expand([(d, dl, acts + [a], w) for d, dl, acts, w, _ in group])
            vals[a] = t + sum(value(o, gr) for o, gr in g.items())
        out[obs] = {a: v / reach for a, v in vals.items()}
        return max(vals.values())

    roots = [(deal, dealer, [], p / 2) for deal, p in eo.rank_deals("kuhn").items() for dealer in (0, 1)]
    t, g = expand(roots)
    for o, gr in g.items():
        value(o, gr)
    return out


def memory_returns(eng, a):
    """Agent a's M_RL (the last min(total, capacity) inserts): per (s bits, argmax a) the
    count and mean r of the TERMINAL transitions (their TD target is r itself)."""
    import torch
    st = eng.stats()
    m = eng.memories(a)
    tot = int(st["rl_total"][a])
    n = min(tot, int(eng.cfg.rl_capacity))
    rows = torch.arange(tot - n, tot, device=m["rl_s"].device) % m["log_cap"]
    w = torch.ones(30, dtype=torch.int64, device=rows.device) << torch.arange(30, device=rows.device)
    sb = ((m["rl_s"][rows] != 0).long() * w).sum(1).cpu().numpy()
    act = m["rl_a"][rows].argmax(1).cpu().numpy()
    r = m["rl_r"][rows].cpu().numpy()
    t = m["rl_t"][rows].cpu().numpy().astype(bool)
    out = {}
    for key in set(zip(sb[t].tolist(), act[t].tolist())):
        sel = t & (sb == key[0]) & (act == key[1])
        out[key] = (int(sel.sum()), float(r[sel].mean()))
    return out


def q_table(eng, a, pol_o):
    """Per information set of agent a: the BR net's Q, the true Q*, greedy vs best action,
    and the terminal returns in M_RL per action."""
    import nn_oracle as nn
    net = nn.MLP(nn.ACT_LINEAR, 64, weights=nn.unpack_weights(eng.get_weights(a, 1)))
    mem = memory_returns(eng, a)
    rows = []
    for obs, qs in sorted(true_q(a, pol_o).items()):
        x = np.array([[(obs >> k) & 1 for k in range(30)]], np.float32)
        q = net.predict(x).reshape(3)
        legal = list(qs)
        rows.append({"obs": obs, "card": int(next(r for r in range(3) if (obs >> (24 + r)) & 1)),
                     "hist_bits": obs & 0xFFFFFF, "q_net": [round(float(q[k]), 3) for k in legal],
                     "q_true": [round(qs[k], 3) for k in legal], "actions": legal,
                     "greedy": int(legal[int(np.argmax([q[k] for k in legal]))]),
                     "best": int(max(qs, key=qs.get)),
                     "mem_terminal": {int(k): mem.get((obs, k)) for k in (0, 1, 2)}})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hands", type=int, default=40_000_000)
    ap.add_argument("--every", type=int, default=5_000_000)
    ap.add_argument("--lanes", type=int, default=256)
    ap.add_argument("--quirks", type=int, default=248)
    ap.add_argument("--set", action="append", default=["lr_ar=0.005", "lr_br=0.1", "gamma=1.0"])
    ap.add_argument("--qtable", action="store_true", help="at the end, per-information-set Q")
    args = ap.parse_args()
    import torch
    import __graft_entry__
    import exploit_oracle as eo
    pkg = __graft_entry__.load_package()
    cfg = dict(n_lanes=args.lanes, rl_capacity=200_000, sl_capacity=2_000_000, quirks=args.quirks)
    for kv in args.set:
        k, v = kv.split("=")
        cfg[k] = float(v)
    eng = pkg.engine.SelfPlayEngine(seed=1234, game=pkg.native.GAME_KUHN, **cfg)
    eta = float(eng.cfg.eta)
    done = 0
    while done < args.hands:
        for _ in range(args.every // args.lanes):
            eng.step()
        done += (args.every // args.lanes) * args.lanes
        torch.cuda.synchronize()
        ar = [eo.Policy(eng.get_weights(a, 0), 0) for a in (0, 1)]
        br = [eo.Policy(eng.get_weights(a, 1), 1) for a in (0, 1)]      # greedy Q (argmax)
        rec = {"hands": int(eng.stats()["hands"]), "quirks": args.quirks, "set": args.set,
               "expl": eo.exploitability_of(ar[0], ar[1], game="kuhn")}
        for i in (0, 1):
            o = 1 - i
            best = eo.best_response(i, ar[o], game="kuhn")
            rec[f"br_gap{i}"] = best - seat_value(i, br[i], ar[o])
            mix = Mix(br[o], ar[o], eta)
            best_m = eo.best_response(i, mix, game="kuhn")
            rec[f"anticip_gap{i}"] = best_m - seat_value(i, br[i], mix)
            rec[f"ar_value{i}"] = seat_value(i, ar[i], ar[o])
        print(json.dumps(rec), flush=True)
    if args.qtable:
        ar = [eo.Policy(eng.get_weights(a, 0), 0) for a in (0, 1)]
        for a in (0, 1):
            for row in q_table(eng, a, ar[1 - a]):
                print(json.dumps({"agent": a, **row}), flush=True)


if __name__ == "__main__":
    main()
