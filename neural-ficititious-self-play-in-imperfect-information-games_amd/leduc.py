"""Drop-in for the reference's ``leduc.newenv.Env`` (leduc/newenv.py:8-349), backed by
the HIP env of libnfsp.

API preserved exactly: ``Env()``, ``reset(dealer)``, ``get_state(p) -> (s, a, r, s2, t)``,
``step(action, p)``, ``round_index``, ``observation_space == (1, 30)``,
``action_space == (3,)``, plus ``get_new_state`` as an alias (the name used by the
abandoned prototype, leduc/env.py:160).

Semantics preserved exactly, including the quirks main.train depends on:

* The deal consumes the global ``random`` like the reference deck: one
  ``random.shuffle`` of a 6-card deck per reset, P0 / P1 / public by ``pop()``
  (leduc/deck.py:42-50, leduc/newenv.py:85-86,109-114,221).  The shuffled ranks are
  injected into the device env (``nfsp_env_set_deal``).
* ``get_state`` returns ``s`` and ``a`` as VIEWS of host arrays ``env.s[p]`` /
  ``env.last_action[p]`` that the env rewrites in place on ``step`` and replaces on
  ``reset`` (leduc/newenv.py:88,101,119,126,136,202) -- the aliasing every stored RL
  tuple of the reference inherits.  ``r`` is the int ``0`` until the hand ends, then a
  float64.  ``s2`` is a fresh [1,1,30] float64 array.
* A step after the end only rewrites ``s[p]`` and prints the reference's warning
  (leduc/newenv.py:346-348).

Every transition is computed by the device (``nfsp_env_step``); the host arrays are
refreshed from the device state after each step.
"""
from __future__ import annotations

import random

import numpy as np
import torch

from . import deck
from . import native
from . import pyrandom

# numpy view of the device `Hand` struct (csrc/nfsp_device.h), 64 bytes
HAND_DTYPE = np.dtype([
    ("hist", "<u4"), ("s", "<u4", (2,)), ("warn", "<u4"), ("la", "<f4", (2, 3)),
    ("rew", "<f4", (2,)), ("rank", "u1", (3,)), ("dealer", "u1"), ("rnd", "u1"),
    ("term", "u1"), ("raises0", "u1"), ("raises1", "u1"), ("slot", "u1"), ("ndone", "u1"),
    ("done0", "u1"), ("done1", "u1"), ("done2", "u1"), ("c0", "u1"), ("c1", "u1"),
    ("pad", "u1")])
assert HAND_DTYPE.itemsize == 64

OBS_DIM = 30
_BITS = (1 << np.arange(OBS_DIM, dtype=np.uint64))


def bits_to_obs(b: int) -> np.ndarray:
    return ((np.uint64(b) & _BITS) != 0).astype(np.float64)


def deal_from_global_random():
    """One reference deal (leduc/newenv.py:85-86,106-114,221): a new deck shuffled with the
    global ``random``, then P0, P1 and the public card picked up from its end."""
    d = deck.Deck(6)
    d.shuffle()
    return d.pick_up().rank, d.pick_up().rank, d.pick_up().rank


class Env:
    """Single Leduc env on the GPU with the reference's Python API."""

    def __init__(self, seed: int = 1234, verbose: bool = True):
        self.ctx = native.Context(1, seed)
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.verbose = verbose
        # device I/O staging: floats s[30] a[3] r s2[30] | byte t
        self._io = torch.zeros(65, dtype=torch.float32, device=self.dev)
        self._t = torch.zeros(1, dtype=torch.uint8, device=self.dev)
        self._act = torch.zeros(3, dtype=torch.float32, device=self.dev)
        self._small = torch.zeros(4, dtype=torch.uint8, device=self.dev)
        self._hand = torch.zeros(64, dtype=torch.uint8, device=self.dev)
        self.dealer = 0
        self._rnd = 0
        self._term = False
        self.warnings = 0
        self.s = np.array([[np.zeros(OBS_DIM)], [np.zeros(OBS_DIM)]])
        self.last_action = np.zeros((2, 3))

    # -- reference properties -----------------------------------------------
    @property
    def round_index(self):
        return self._rnd

    @property
    def action_space(self):
        return (3,)

    @property
    def observation_space(self):
        return (1, OBS_DIM)

    @property
    def terminated(self):
        return self._term

    # -- API ------------------------------------------------------------------
    def reset(self, dealer, ranks=None):
        """``ranks`` (P0, P1, public) overrides the global-random deal (tests)."""
        self.dealer = dealer
        r0, r1, rp = deal_from_global_random() if ranks is None else ranks
        self._small.copy_(torch.tensor([r0, r1, rp, dealer & 1], dtype=torch.uint8))
        p = self._small.data_ptr()
        self.ctx.call("nfsp_env_set_deal", native.P(p))
        self.ctx.call("nfsp_env_reset", native.P(p + 3))
        self.s = np.array([[np.zeros(OBS_DIM)], [np.zeros(OBS_DIM)]])
        self.last_action = np.zeros((2, 3))
        self._rnd = 0
        self._term = False

    def get_state(self, p_index):
        p = int(p_index)
        base = self._io.data_ptr()
        self.ctx.call("nfsp_env_get_state", p, None, native.P(base), native.P(base + 120),
                      native.P(base + 132), native.P(base + 136), native.ptr(self._t))
        io = self._io.cpu().numpy()
        t = bool(self._t.item())
        s2 = io[34:64].astype(np.float64).reshape(1, 1, OBS_DIM)
        r = np.float64(io[33]) if t else 0
        return self.s[p], self.last_action[p].reshape(1, 1, 3), r, s2, t

    get_new_state = get_state

    def do_action(self, action, p_index):
        """Env.do_action (leduc/newenv.py:131-178) alone, on the device: records the action
        (argmax, illegal raise -> call) without ending the round or the hand; True on a fold."""
        p = int(p_index)
        a = np.asarray(action, dtype=np.float32).reshape(3)
        self._act.copy_(torch.from_numpy(a))
        self.ctx.call("nfsp_env_do_action", native.ptr(self._act), p, None, None, native.ptr(self._t))
        fold = bool(self._t.item())
        self.last_action[p] = a
        return fold

    def game_or_round_has_terminated(self):
        """leduc/newenv.py:180-190 on the device's actions_done: True, False, or the
        reference's None for a length-2 / -3 sequence that does not end the round."""
        self.ctx.call("nfsp_env_round_status", native.ptr(self._small))
        v = int(self._small[0].item())
        return True if v == 1 else (None if v == 255 else False)

    def step(self, action, p_index):
        p = int(p_index)
        a = np.asarray(action, dtype=np.float32).reshape(3)
        self._act.copy_(torch.from_numpy(a))
        self.ctx.call("nfsp_env_step", native.ptr(self._act), p, None, None)
        self.ctx.call("nfsp_env_export", native.ptr(self._hand))
        h = np.frombuffer(self._hand.cpu().numpy().tobytes(), dtype=HAND_DTYPE)[0]
        self.s[p][0][:] = bits_to_obs(int(h["s"][p]))
        if int(h["warn"]) > self.warnings:
            self.warnings = int(h["warn"])
            if self.verbose:
                print("Player{} tried to step while self.terminated is {}".format(p, self._term))
            return
        self.last_action[p] = h["la"][p]
        self._rnd = int(h["rnd"])
        self._term = bool(h["term"])
