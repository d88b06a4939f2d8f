"""Drop-in for the reference's ``agent.agent.Agent`` (agent/agent.py:18-273) with the
networks, their updates and both memories on the GPU.

Preserved API: ``Agent(sess, state_dim, action_dim, name, env)``, ``play``,
``act_best_response``, ``boltzmann``, ``remember_for_rl``, ``remember_best_response``,
``update_strategy``, ``update_best_response_network``, ``update_avg_response_network``,
``update_br_target_network``, ``sampled_actions``, ``average_payoff_br``; attributes
``best_response_model`` / ``target_br_model`` / ``avg_strategy_model`` with
``predict``, ``get_weights``, ``set_weights``.

Preserved semantics: the play() observe/store/act/update order,
``np.average(a) != 0`` store rule, ``game_step % 128`` trigger, eps-greedy BR with the
global ``random`` and ``np.random.rand``, the BR/AR update schedules (iteration += 2,
temperature, target sync every TargetModelUpdateRate, lr decay, ``eps = eps/iteration``)
and, by default, the reference's target quirks (``quirks=native.QUIRKS_REFERENCE``).

Device work per call: predict -> ``nfsp_mlp_forward``; BR targets ->
``nfsp_br_targets``; fits -> ``nfsp_mlp_fit`` (the Keras fit shuffles are drawn from the
global ``np.random`` on the host, one ``shuffle(arange(n))`` per epoch, as Keras 2.x
does); memories -> ``buffers``.  Initial weights: Keras's glorot_uniform / zeros,
drawn from ``init_rng`` (TF's own initialiser RNG cannot be reproduced).
"""
from __future__ import annotations

import math
import random

import numpy as np
import torch

from . import native
from .buffers import ReplayBuffer, ReservoirBuffer

CFG = dict(hidden=64, lr_br=0.05, lr_ar=0.1, gamma=0.95, epsilon=0.06, batch=128, eta=0.1,
           target_every=150, buffer=40000, seed=1234)
OBS = 30


def glorot(rng, fan_in, fan_out):
    limit = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-limit, limit, size=(fan_in, fan_out)).astype(np.float32)


class DeviceMLP:
    """A 30 -> 64 -> 3 head whose packed weights live in HBM."""

    def __init__(self, act, hidden, rng, ctx):
        self.act, self.hidden, self.ctx = act, hidden, ctx
        self.dev = torch.device("cuda", torch.cuda.current_device())
        ws = [glorot(rng, OBS, hidden), np.zeros(hidden, np.float32),
              glorot(rng, hidden, 3), np.zeros(3, np.float32)]
        self.w = torch.zeros(OBS * hidden + hidden + hidden * 3 + 3, dtype=torch.float32,
                             device=self.dev)
        self.set_weights(ws)

    def get_weights(self):
        f = self.w.cpu().numpy()
        H = self.hidden
        o = 0
        W1 = f[o:o + OBS * H].reshape(OBS, H).copy(); o += OBS * H
        b1 = f[o:o + H].copy(); o += H
        W2 = f[o:o + 3 * H].reshape(H, 3).copy(); o += 3 * H
        b2 = f[o:o + 3].copy()
        return [W1, b1, W2, b2]

    def set_weights(self, ws):
        flat = np.concatenate([np.ravel(np.asarray(x, np.float32)) for x in ws])
        self.w.copy_(torch.from_numpy(flat))

    def predict_device(self, x_dev):
        B = x_dev.shape[0]
        y = torch.empty((B, 3), dtype=torch.float32, device=self.dev)
        self.ctx.call("nfsp_mlp_forward", native.ptr(self.w), self.hidden, self.act,
                      native.ptr(x_dev), native.ptr(y), B)
        return y

    def predict(self, x):
        x = np.asarray(x, np.float32)
        lead = x.shape[:-1]
        xd = torch.as_tensor(x.reshape(-1, OBS), device=self.dev).contiguous()
        return self.predict_device(xd).cpu().numpy().reshape(lead + (3,))

    def fit_device(self, x_dev, t_dev, lr, epochs=2, batch_size=32):
        """Keras ``fit`` (shuffle=True): permutations from the global np.random."""
        n = x_dev.shape[0]
        perms = []
        for _ in range(epochs):
            idx = np.arange(n)
            np.random.shuffle(idx)
            perms.append(idx)
        pd = torch.as_tensor(np.concatenate(perms).astype(np.int32), device=self.dev)
        self.ctx.call("nfsp_mlp_fit", native.ptr(self.w), self.hidden, self.act,
                      native.ptr(x_dev.contiguous()), native.ptr(t_dev.contiguous()), n,
                      native.ptr(pd), epochs, batch_size, native.F32(lr))
        return np.stack(perms)


class Agent:
    def __init__(self, sess, state_dim, action_dim, name, env, cfg=None, init_rng=None,
                 quirks=native.QUIRKS_REFERENCE):
        c = dict(CFG, **(cfg or {}))
        self.sess, self.s_dim, self.a_dim = sess, state_dim, action_dim
        self.name = name
        self.env = env
        self.ctx = env.ctx if hasattr(env, "ctx") else native.Context(1)
        self.quirks = quirks
        self.exploitability = 0
        self.iteration = 0
        self.minibatch_size = c["batch"]
        self.n_hidden = c["hidden"]
        self.lr_br = c["lr_br"]
        self.lr_ar = c["lr_ar"]
        self.cur_lr_br = np.float32(self.lr_br)
        self.epsilon = c["epsilon"]
        self.gamma = c["gamma"]
        self.eta = c["eta"]
        self.temp = (1 + 0.02 * np.sqrt(self.iteration)) ** (-1)
        self.target_model_update_rate = c["target_every"]
        self.target_br_model_update_count = 0
        self._rl_memory = ReplayBuffer(c["buffer"], c["seed"], self.ctx,
                                       alias=bool(quirks & native.QUIRK_ALIAS_RL))
        self._sl_memory = ReservoirBuffer(c["buffer"], c["seed"], self.ctx)
        rng = init_rng if init_rng is not None else np.random.RandomState(0)
        self.avg_strategy_model = DeviceMLP(native.ACT_SOFTMAX, self.n_hidden, rng, self.ctx)
        self.best_response_model = DeviceMLP(native.ACT_RELU, self.n_hidden, rng, self.ctx)
        self.target_br_model = DeviceMLP(native.ACT_RELU, self.n_hidden, rng, self.ctx)
        self.target_br_model.w.copy_(self.best_response_model.w)
        self.actions = np.zeros(3)
        self.played = 0
        self.reward = 0
        self.game_step = 0
        self._expl = torch.zeros(1, dtype=torch.float64, device=self.best_response_model.dev)

    # -- memories ---------------------------------------------------------------
    def remember_best_response(self, state, action):
        self._sl_memory.add(state, action)

    def remember_for_rl(self, state, action, reward, nextstate, terminal):
        self._rl_memory.add(state, action, reward, nextstate, terminal)

    # -- acting -----------------------------------------------------------------
    def act_best_response(self, state):
        if random.random() > self.epsilon:
            return self.best_response_model.predict(state)
        return np.random.rand(1, 1, 3)

    def boltzmann(self, actions):
        q = np.asarray(actions, np.float64)[0][0]
        e = np.exp(q / self.temp)
        bottom = 0.0
        for k in range(3):
            bottom += e[k]
        return (e / bottom).reshape(1, 1, 3)

    def play(self, policy, index, s2=None):
        if s2 is None:
            s, a, r, s2, t = self.env.get_state(index)
            self.reward += r
            if np.average(a) != 0:
                self.remember_for_rl(s, a, r, s2, t)
                self.game_step += 1
            if t:
                return t
        else:
            t = False
        x = np.reshape(s2, (1, 1, OBS))
        if policy == "a":
            a = self.avg_strategy_model.predict(x)
            self.env.step(a, index)
        else:
            a_t = self.act_best_response(x)
            a = self.boltzmann(a_t)
            self.env.step(a_t, index)
            self.remember_best_response(s2, a_t)
        self.played += 1
        if self.game_step % 128 == 0:
            self.update_strategy()
        self.actions[np.argmax(a)] += 1
        return t

    # -- learning ---------------------------------------------------------------
    def update_strategy(self):
        self.update_avg_response_network()
        self.update_best_response_network()

    verbose = True      # sampled_actions prints like the reference (agent/agent.py:197)

    def sampled_actions(self):
        if self.verbose:
            print("{} played {} times: Folds: {}, Calls: {}, Raises: {} - Reward: {}".format(
                self.name, self.played, self.actions[0], self.actions[1], self.actions[2],
                self.reward))
        self.actions = np.zeros(3)
        self.played = 0

    def average_payoff_br(self):
        return np.average(self.exploitability)

    def update_best_response_network(self):
        if self._rl_memory.size() <= self.minibatch_size:
            return
        self.iteration += 1
        b = self._rl_memory.sample_device(self.minibatch_size)
        n = b.cap
        target = torch.empty((n, 3), dtype=torch.float32, device=b.s.device)
        self.ctx.call("nfsp_br_targets", native.ptr(self.target_br_model.w), self.n_hidden,
                      native.ptr(b.s), native.ptr(b.a), native.ptr(b.r), native.ptr(b.s2),
                      native.ptr(b.t), n, native.F64(self.gamma), self.quirks & 3,
                      native.ptr(target), native.ptr(self._expl))
        self.exploitability = float(self._expl.item())
        self.best_response_model.fit_device(b.s, target, self.cur_lr_br)
        self.iteration += 1
        self.temp = (1 + 0.02 * np.sqrt(self.iteration)) ** (-1)
        self.update_br_target_network()
        self.cur_lr_br = np.float32(self.lr_br / (1 + 0.003 * math.sqrt(self.iteration)))
        self.epsilon = self.epsilon ** 1 / self.iteration

    def update_avg_response_network(self):
        if self._sl_memory.size() <= self.minibatch_size:
            return
        b = self._sl_memory.sample_device(self.minibatch_size)
        self.avg_strategy_model.fit_device(b.s, b.a, np.float32(self.lr_ar))

    def update_br_target_network(self):
        if self.target_br_model_update_count % self.target_model_update_rate == 0:
            self.target_br_model.w.copy_(self.best_response_model.w)
        self.target_br_model_update_count += 1
