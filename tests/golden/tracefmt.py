"""Event-log format shared by the golden generator (which records the REFERENCE)
and the tests (which record the oracle / the HIP drop-in through the same wrappers).

Test infrastructure only.  ``Recorder.wrap_classes`` instruments any implementation
of the Env / ReplayBuffer / ReservoirBuffer / Agent API (reference, oracle, HIP
drop-in) at class level; the resulting (code, who, payload) arrays are compared
event for event.
"""
from __future__ import annotations

import zlib

import numpy as np


def bits30(x) -> int:
    v = np.asarray(x, dtype=np.float64).reshape(-1)
    assert v.shape == (30,), v.shape
    assert np.all((v == 0) | (v == 1)), v
    return int(sum(int(v[i]) << i for i in range(30)))


def crc(*arrays) -> int:
    h = 0
    for a in arrays:
        h = zlib.crc32(np.ascontiguousarray(np.asarray(a, dtype=np.float64)).tobytes(), h)
    return h


EV_RESET, EV_GET, EV_STEP, EV_RL_ADD, EV_SL_ADD, EV_RL_SAMPLE, EV_SL_SAMPLE, \
    EV_BR_UPD, EV_AR_UPD, EV_STATS = range(10)
PAYLOAD = 8


class Recorder:
    """Wraps Env / buffer / agent methods of whichever implementation is passed."""

    def __init__(self):
        self.code, self.who, self.pay = [], [], []
        self.buf_ids = {}
        self._orig = []

    def ev(self, code, who, *vals):
        v = np.zeros(PAYLOAD)
        v[:len(vals)] = vals
        self.code.append(code)
        self.who.append(who)
        self.pay.append(v)

    def bid(self, buf):
        return self.buf_ids.setdefault(id(buf), len(self.buf_ids))

    def wrap_classes(self, env_cls, rb_cls, rs_cls, agent_cls):
        R = self

        def w(cls, name, fn):
            orig = cls.__dict__[name]
            R._orig.append((cls, name, orig))

            def inner(self, *a, **k):
                return fn(orig, self, *a, **k)
            setattr(cls, name, inner)

        def reset(orig, env, dealer):
            orig(env, dealer)
            s0 = bits30(env.get_state(0)[3])
            s1 = bits30(env.get_state(1)[3])
            R.ev(EV_RESET, dealer, s0, s1)

        def get_state(orig, env, p):
            out = orig(env, p)
            s, a, r, s2, t = out
            a3 = np.asarray(a, np.float64).reshape(3)
            R.ev(EV_GET, p, bits30(s), a3[0], a3[1], a3[2], float(r), bits30(s2), float(t))
            return out

        def step(orig, env, action, p):
            v = np.asarray(action, np.float64).reshape(3)
            orig(env, action, p)
            R.ev(EV_STEP, p, v[0], v[1], v[2], env.round_index)

        def rl_add(orig, buf, s, a, r, s2, t):
            orig(buf, s, a, r, s2, t)
            R.ev(EV_RL_ADD, R.bid(buf), buf.size(), float(r), float(t))

        def sl_add(orig, buf, s, a):
            orig(buf, s, a)
            R.ev(EV_SL_ADD, R.bid(buf), buf.size())

        def rl_sample(orig, buf, n):
            out = orig(buf, n)
            R.ev(EV_RL_SAMPLE, R.bid(buf), len(out[0]), crc(*out[:4]),
                 crc(np.asarray(out[4], np.float64)))
            return out

        def sl_sample(orig, buf, n):
            out = orig(buf, n)
            R.ev(EV_SL_SAMPLE, R.bid(buf), len(out[0]), crc(*out))
            return out

        def br_upd(orig, ag):
            orig(ag)
            lr = ag.sgd_br.lr.value if hasattr(ag, "sgd_br") else ag.cur_lr_br
            tw = ag.target_br_model.get_weights()
            R.ev(EV_BR_UPD, 0 if ag.name == "Player0" else 1, ag.iteration, ag.epsilon,
                 float(lr), float(np.average(ag.exploitability)), ag.temp,
                 crc(*ag.best_response_model.get_weights()), crc(*tw))

        def ar_upd(orig, ag):
            orig(ag)
            R.ev(EV_AR_UPD, 0 if ag.name == "Player0" else 1,
                 crc(*ag.avg_strategy_model.get_weights()))

        def stats(orig, ag):
            R.ev(EV_STATS, 0 if ag.name == "Player0" else 1, ag.played, ag.actions[0],
                 ag.actions[1], ag.actions[2], float(ag.reward),
                 float(ag.average_payoff_br()))
            orig(ag)

        w(env_cls, "reset", reset)
        w(env_cls, "get_state", get_state)
        w(env_cls, "step", step)
        w(rb_cls, "add", rl_add)
        w(rs_cls, "add", sl_add)
        w(rb_cls, "sample_batch", rl_sample)
        w(rs_cls, "sample_batch", sl_sample)

        # device-side drop-ins sample through sample_device (no host arrays): record
        # the event and its size; the content is checked by what follows it
        def dev_sample(code):
            def fn(orig, buf, n):
                out = orig(buf, n)
                R.ev(code, R.bid(buf), out.cap)
                return out
            return fn
        if "sample_device" in rb_cls.__dict__:
            w(rb_cls, "sample_device", dev_sample(EV_RL_SAMPLE))
        if "sample_device" in rs_cls.__dict__:
            w(rs_cls, "sample_device", dev_sample(EV_SL_SAMPLE))
        w(agent_cls, "update_best_response_network", br_upd)
        w(agent_cls, "update_avg_response_network", ar_upd)
        w(agent_cls, "sampled_actions", stats)

    def restore(self):
        for cls, name, orig in reversed(self._orig):
            setattr(cls, name, orig)
        self._orig = []

    def arrays(self):
        return (np.array(self.code, np.uint8), np.array(self.who, np.uint8),
                np.array(self.pay, np.float64))
