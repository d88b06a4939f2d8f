"""Batched self-play: the fused hot path (``nfsp_engine_*`` / ``nfsp_rollout``).

``SelfPlayEngine`` owns one ``nfsp_engine`` (n_lanes hands in flight, both agents'
networks and memories in HBM).  ``step()`` = one hand per lane through the fused
rollout kernel + the deterministic insert + the learner at the reference cadence
(one update_strategy per ``inserts_per_update`` RL inserts of an agent,
agent/agent.py:153).  Configuration keys mirror config.ini:

    reference (config C1)   n_lanes=1,   rl_capacity=40_000,  sl_capacity=40_000
    C2                      n_lanes=65_536
    C3                      n_lanes=1_048_576, rl_capacity=200_000, sl_capacity=2_000_000
                            (slices=16: the 1M lanes advance in 16 slices of 65,536, the
                            learner consuming each slice before the next acts)
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import native

NP = 30 * 64 + 64 + 64 * 3 + 3
NET_AR, NET_BR, NET_TARGET = 0, 1, 2

PRESETS = {
    "reference": dict(n_lanes=1, rl_capacity=40_000, sl_capacity=40_000),
    "c2": dict(n_lanes=65_536, rl_capacity=40_000, sl_capacity=40_000),
    "c3": dict(n_lanes=1_048_576, rl_capacity=200_000, sl_capacity=2_000_000),
}


def glorot_net(rng: np.random.RandomState, hidden: int = 64) -> np.ndarray:
    """Keras defaults: glorot_uniform kernels, zero biases; packed like nfsp.h."""
    def g(fi, fo):
        lim = np.sqrt(6.0 / (fi + fo))
        return rng.uniform(-lim, lim, size=(fi, fo)).astype(np.float32)
    return np.concatenate([g(30, hidden).ravel(), np.zeros(hidden, np.float32),
                           g(hidden, 3).ravel(), np.zeros(3, np.float32)])


def make_cfg(L, **cfg) -> native.EngineCfg:
    c = native.EngineCfg()
    native.check(L.nfsp_engine_default_cfg(C.byref(c)), "nfsp_engine_default_cfg")
    for k, v in cfg.items():
        if not hasattr(c, k):
            raise KeyError(k)
        setattr(c, k, v)
    return c


class SelfPlayEngine:
    def __init__(self, ctx: native.Context | None = None, init_seed: int = 0, game: int = native.GAME_LEDUC,
                 _borrow=None, **cfg):
        self.ctx = ctx if ctx is not None else native.Context(1, game=game)
        L = self.ctx.L
        self.L = L
        self.dev = torch.device("cuda", torch.cuda.current_device())
        if _borrow is not None:            # a replica of an EngineGroup: (group, handle, cfg)
            self._owner, self.h, self.cfg = _borrow
            self._init_weights(init_seed)
            return
        self._owner = None
        c = make_cfg(L, **cfg)
        self.cfg = c
        h = native.P()
        native.check(L.nfsp_engine_create(self.ctx.h, C.byref(c), C.byref(h)), "nfsp_engine_create")
        self.h = h
        self._init_weights(init_seed)

    def _init_weights(self, init_seed):
        # initial weights in the reference's construction order: per agent AR, BR, target
        # (the target is drawn, then overwritten with BR: agent/agent.py:67-72)
        rng = np.random.RandomState(init_seed)
        for a in (0, 1):
            ar = glorot_net(rng)
            br = glorot_net(rng)
            glorot_net(rng)
            self.set_weights(a, NET_AR, ar)
            self.set_weights(a, NET_BR, br)
            self.set_weights(a, NET_TARGET, br)

    # -- weights ------------------------------------------------------------------
    def _wptr(self, agent, net):
        p = native.P()
        native.check(self.L.nfsp_engine_weights(self.h, agent, net, C.byref(p)), "weights")
        return p.value

    def weights_tensor(self, agent, net) -> torch.Tensor:
        """A torch view (no copy) of the device weights of (agent, net)."""
        return _wrap_device(self._wptr(agent, net), NP, torch.float32, self.dev, self)

    def get_weights(self, agent, net) -> np.ndarray:
        return self.weights_tensor(agent, net).cpu().numpy().copy()

    def set_weights(self, agent, net, flat):
        self.weights_tensor(agent, net).copy_(torch.as_tensor(np.asarray(flat, np.float32)))

    # -- hot path -----------------------------------------------------------------
    def rollout(self):
        native.check(self.L.nfsp_rollout(self.h), "nfsp_rollout")

    def rollout_with(self, w_flat: np.ndarray, eps):
        """Test hook (nfsp_rollout_with): the next slice's rollout acting with the given nets
        ([2][3][NP] flat, as weights_tensor packs them) and epsilons."""
        w = torch.as_tensor(np.asarray(w_flat, np.float32).reshape(-1), device=self.dev)
        assert w.numel() == 6 * NP
        e = (C.c_double * 2)(float(eps[0]), float(eps[1]))
        native.check(self.L.nfsp_rollout_with(self.h, C.c_void_p(w.data_ptr()), e), "nfsp_rollout_with")
        torch.cuda.synchronize(self.dev)       # w is a temporary

    def update(self):
        native.check(self.L.nfsp_engine_update(self.h), "nfsp_engine_update")

    def step(self):
        """One hand on every lane: ``cfg.slices`` x (rollout of the next slice + update)."""
        native.check(self.L.nfsp_engine_step(self.h), "nfsp_engine_step")

    def stats(self) -> dict:
        s = native.EngineStats()
        native.check(self.L.nfsp_engine_get_stats(self.h, C.byref(s)), "nfsp_engine_get_stats")
        return s.to_dict()

    KERNELS = ("k_rollout", "k_scan", "k_commit", "learner", "learner_prep", "k_br_targets",
               "k_chain3_br", "k_chain3_ar", "br_stream_a0", "br_stream_a1", "ar_exchange")

    def set_timing(self, on=True):
        native.check(self.L.nfsp_engine_set_timing(self.h, int(bool(on))), "set_timing")

    def timings(self) -> dict:
        """{kernel: (total ms, launches)} since the last call (HIP events, ctx stream)."""
        ms = (native.F64 * len(self.KERNELS))()
        n = (native.I64 * len(self.KERNELS))()
        native.check(self.L.nfsp_engine_get_timings(self.h, ms, n), "get_timings")
        return {k: (ms[i], n[i]) for i, k in enumerate(self.KERNELS)}

    # -- inspection (tests) -------------------------------------------------------
    def memories(self, agent):
        rl, sl = native.Records(), native.Records()
        cap = native.I64()
        px, pa, pp = native.P(), native.P(), native.P()
        native.check(self.L.nfsp_engine_memories(self.h, agent, C.byref(rl), C.byref(cap),
                                                  C.byref(sl), C.byref(px), C.byref(pa),
                                                  C.byref(pp)), "nfsp_engine_memories")
        n = cap.value
        d = self.dev
        out = dict(
            log_cap=n,
            rl_s=_wrap_device(rl.s, n * 30, torch.float32, d, self).view(n, 30),
            rl_a=_wrap_device(rl.a, n * 3, torch.float32, d, self).view(n, 3),
            rl_r=_wrap_device(rl.r, n, torch.float32, d, self),
            rl_s2=_wrap_device(rl.s2, n * 30, torch.float32, d, self).view(n, 30),
            rl_t=_wrap_device(rl.t, n, torch.uint8, d, self),
            sl_s=_wrap_device(sl.s, sl.cap * 30, torch.float32, d, self).view(sl.cap, 30),
            sl_a=_wrap_device(sl.a, sl.cap * 3, torch.float32, d, self).view(sl.cap, 3),
        )
        pc = 4 * self.slice_lanes
        out["pend_x"] = _wrap_device(px.value, pc, torch.int32, d, self)
        out["pend_a"] = _wrap_device(pa.value, pc * 3, torch.float32, d, self).view(pc, 3)
        out["pend_pos"] = _wrap_device(pp.value, pc, torch.int64, d, self)
        return out

    def last_update(self, agent, role):
        rows, perms = native.P(), native.P()
        native.check(self.L.nfsp_engine_last_update(self.h, agent, role, C.byref(rows),
                                                     C.byref(perms)), "last_update")
        B, E = self.cfg.batch, self.cfg.epochs
        return (_wrap_device(rows.value, B, torch.int64, self.dev).cpu().numpy(),
                _wrap_device(perms.value, E * B, torch.int32, self.dev).view(E, B).cpu().numpy())

    @property
    def slice_lanes(self) -> int:
        """Lanes per rollout (cfg.slices: n_lanes / slices)."""
        return self.cfg.n_lanes // self.cfg.slices

    def last_slice(self) -> tuple:
        """(global id of the first lane, hand index g) of the last rollout: rollout k plays
        slice k % slices with the lanes' hand index k // slices (include/nfsp.h cfg.slices)."""
        k = self.stats()["rollouts"] - 1
        return (k % self.cfg.slices) * self.slice_lanes, k // self.cfg.slices

    def lane_counts(self) -> np.ndarray:
        """[n_lanes / slices, 4] (RL agent 0, RL agent 1, SL agent 0, SL agent 1) records of each
        lane's hand in the last rollout (its slice's lanes; nfsp_engine_lane_counts;
        synchronises)."""
        p = native.P()
        native.check(self.L.nfsp_engine_lane_counts(self.h, C.byref(p)), "lane_counts")
        torch.cuda.synchronize(self.dev)
        c = _wrap_device(p.value, self.slice_lanes, torch.int32, self.dev).cpu().numpy()
        c = c.astype(np.int64) & 0xFFFF
        return np.stack([(c >> (4 * k)) & 15 for k in range(4)], axis=1)

    def snapshot(self, parity: int):
        """(acting nets [2][3][NP] flat, (eps0, eps1)) of snapshot `parity` (cfg.slice_lag 2,
        nfsp_engine_snapshot): after a pipelined step of K slices, parity (K - 1) & 1 is what
        the last slice acted with."""
        p = native.P()
        eps = (C.c_double * 2)()
        native.check(self.L.nfsp_engine_snapshot(self.h, int(parity), C.byref(p), eps), "snapshot")
        torch.cuda.synchronize(self.dev)
        w = _wrap_device(p.value, 6 * NP, torch.float32, self.dev, self).cpu().numpy().copy()
        return w, (eps[0], eps[1])

    def set_exchange(self, every: int, scale: float, comm=None, fn=None):
        """The cross-shard exchange of the AR nets (nfsp_engine_set_exchange): after every
        ``every``-th learner call (slice), W_AR = W0 + (sum over shards of W_AR - W0) * scale on
        the AR chain stream, by the RCCL communicator ``comm`` or the host callback ``fn``
        (a ``native.EXCHANGE_FN``; kept alive here).  W0 = the AR nets now.  every 0: off."""
        self._xchg_fn = fn
        native.check(self.L.nfsp_engine_set_exchange(self.h, int(every), float(scale), comm, fn, None),
                     "nfsp_engine_set_exchange")

    def exchanges(self) -> int:
        n = native.I64()
        native.check(self.L.nfsp_engine_exchanges(self.h, C.byref(n)), "nfsp_engine_exchanges")
        return n.value

    def set_update_limit(self, max_updates: int):
        """Test hook (nfsp_engine_set_update_limit): the chains run only a prefix of each
        learner call's updates."""
        native.check(self.L.nfsp_engine_set_update_limit(self.h, int(max_updates)), "set_update_limit")

    loss_log = False

    def set_loss_log(self, on=True):
        native.check(self.L.nfsp_engine_set_loss_log(self.h, int(bool(on))), "set_loss_log")
        self.loss_log = bool(on)

    def losses(self) -> dict:
        """Keras epoch losses of the last learner call (nfsp_engine_losses), keyed like the
        reference's TensorBoard log dirs (agent/agent.py:84-88): Player{a}rl = BR, Player{a}sl = AR."""
        out = (C.c_double * 8)()
        native.check(self.L.nfsp_engine_losses(self.h, out), "nfsp_engine_losses")
        d = {}
        for a in (0, 1):
            for n, tag in ((0, "sl"), (1, "rl")):
                d[f"Player{a}{tag}/loss_mean"] = out[(2 * a + n) * 2]
                d[f"Player{a}{tag}/loss_last"] = out[(2 * a + n) * 2 + 1]
        return d

    def exploitability(self, mode: int = 0) -> dict:
        """Exact exploitability of the two agents' current AR nets (nfsp_exploitability):
        mode 0 = softmax mixed strategies, 1 = the argmax the env executes."""
        return exploitability(self.ctx, self._wptr(0, NET_AR), self._wptr(1, NET_AR), mode)

    def close(self):
        if getattr(self, "h", None) and getattr(self, "_owner", None) is None:
            self.L.nfsp_engine_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class EngineGroup:
    """R replicas of the engine stepped together (``nfsp_group_*``, include/nfsp.h): each an
    independent main.train over ``n_lanes`` lanes with its own memories and nets (seed + r,
    initial nets from ``init_seed + r`` -- replica r is bit-identical to
    ``SelfPlayEngine(seed=seed + r, init_seed=init_seed + r)``), their SGD chains in shared
    launches.  ``avg_ar``: the AR nets are averaged over the replicas after every step (C4's
    exchange on device, shards.AvgPolicyAllReduce); ``set_exchange`` for other cadences (e.g.
    after every slice, shards.AvgPolicyExchange's).  ``slice_lag=2``: every replica's slice j
    acts with the nets slice j - 2 left (a pipelined engine's arithmetic; executed pipelined --
    slice j + 1's rollout, plan and prep overlap slice j's chains -- unless the BR nets are
    exchanged or ``set_sched(serial=1)``)."""

    def __init__(self, replicas: int, ctx: native.Context | None = None, init_seed: int = 0,
                 game: int = native.GAME_LEDUC, avg_ar: bool = False, **cfg):
        self.ctx = ctx if ctx is not None else native.Context(1, game=game)
        self.L = self.ctx.L
        self.cfg = make_cfg(self.L, **cfg)
        h = native.P()
        native.check(self.L.nfsp_group_create(self.ctx.h, C.byref(self.cfg), int(replicas),
                                              native.GROUP_AVG_AR if avg_ar else 0, C.byref(h)),
                     "nfsp_group_create")
        self.h = h
        self.R = int(replicas)
        self.replicas = []
        for r in range(self.R):
            e = native.P()
            native.check(self.L.nfsp_group_engine(self.h, r, C.byref(e)), "nfsp_group_engine")
            c = native.EngineCfg.from_buffer_copy(self.cfg)
            c.seed = self.cfg.seed + r
            self.replicas.append(SelfPlayEngine(self.ctx, init_seed=init_seed + r, _borrow=(self, e, c)))

    def step(self):
        native.check(self.L.nfsp_group_step(self.h), "nfsp_group_step")

    def average_ar(self):
        native.check(self.L.nfsp_group_average_ar(self.h), "nfsp_group_average_ar")

    def set_exchange(self, nets: int = native.XCHG_AR, every: int = 1, scale: float | None = None):
        """nfsp_group_set_exchange: after every ``every``-th slice, the ``nets``
        (native.XCHG_AR | XCHG_BR) of all replicas <- W0 + (sum_r W_r - W0) * scale (default
        1 / R, the mean); every 0: off.  The next exchange of a net not exchanged before copies
        replica 0's instead."""
        scale = 1.0 / self.R if scale is None else float(scale)
        native.check(self.L.nfsp_group_set_exchange(self.h, int(nets), int(every), scale),
                     "nfsp_group_set_exchange")

    def sched(self) -> dict:
        """The group's BR-round / slice schedule (nfsp_group_get_sched)."""
        sc = native.GroupSched()
        native.check(self.L.nfsp_group_get_sched(self.h, C.byref(sc)), "nfsp_group_get_sched")
        return {k: int(getattr(sc, k)) for k, _ in sc._fields_}

    def set_sched(self, **kw):
        """nfsp_group_set_sched: change br_cap / br_pace / br_streams / serial / br_persist
        from the next learner call (the rest stay as they are).  No SGD step changes."""
        cur = self.sched()
        for k in kw:
            if k not in cur:
                raise KeyError(k)
        cur.update(kw)
        native.check(self.L.nfsp_group_set_sched(self.h, C.byref(native.GroupSched(**cur))),
                     "nfsp_group_set_sched")

    def check(self):
        """nfsp_group_check: synchronise the group's streams; raises if a k_br_persist wait
        expired (sched br_persist)."""
        native.check(self.L.nfsp_group_check(self.h), "nfsp_group_check")

    def rounds(self) -> int:
        n = native.I64()
        native.check(self.L.nfsp_group_rounds(self.h, C.byref(n)), "nfsp_group_rounds")
        return n.value

    def set_trace(self, on=True):
        """Start (and clear) / stop the learner-plan trace (nfsp_group_set_trace)."""
        native.check(self.L.nfsp_group_set_trace(self.h, int(bool(on))), "nfsp_group_set_trace")

    def trace(self) -> np.ndarray:
        """The traced learner calls' update counts, [call][replica][agent][AR, BR]."""
        n = native.I64()
        native.check(self.L.nfsp_group_trace(self.h, None, 0, C.byref(n)), "nfsp_group_trace")
        buf = (native.I32 * max(n.value, 1))()
        native.check(self.L.nfsp_group_trace(self.h, buf, n.value, C.byref(n)), "nfsp_group_trace")
        return np.frombuffer(buf, np.int32, count=n.value).reshape(-1, self.R, 2, 2).copy()

    def stats(self) -> dict:
        """Per-replica stats summed (counters) and listed (``replicas``)."""
        per = [e.stats() for e in self.replicas]
        out = {"replicas": per}
        for k in ("hands", "rollouts"):
            out[k] = sum(p[k] for p in per)
        for k in ("rl_total", "sl_total", "br_updates", "ar_updates", "last_rl", "last_sl"):
            out[k] = [sum(p[k][a] for p in per) for a in (0, 1)]
        out["exploitability"] = [float(np.mean([p["exploitability"][a] for p in per])) for a in (0, 1)]
        return out

    KERNELS = SelfPlayEngine.KERNELS

    def set_timing(self, on=True):
        native.check(self.L.nfsp_group_set_timing(self.h, int(bool(on))), "set_timing")

    def timings(self) -> dict:
        ms = (native.F64 * len(self.KERNELS))()
        n = (native.I64 * len(self.KERNELS))()
        native.check(self.L.nfsp_group_get_timings(self.h, ms, n), "get_timings")
        return {k: (ms[i], n[i]) for i, k in enumerate(self.KERNELS)}

    def exploitability(self, mode: int = 0, replica: int = 0) -> dict:
        return self.replicas[replica].exploitability(mode)

    def exploitability_all(self, mode: int = 0) -> list:
        """Exact exploitability of every replica's AR pair in one launch
        (nfsp_exploitability_batch, one workgroup per replica)."""
        w0 = [e._wptr(0, NET_AR) for e in self.replicas]
        w1 = [e._wptr(1, NET_AR) for e in self.replicas]
        return exploitability_batch(self.ctx, w0, w1, mode)

    def close(self):
        if getattr(self, "h", None):
            for e in self.replicas:
                e.h = None
            self.L.nfsp_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def exploitability(ctx, dev_w_ar0: int, dev_w_ar1: int, mode: int = 0) -> dict:
    """nfsp_exploitability on two packed AR nets given as device pointers."""
    out = (C.c_double * 4)()
    native.check(ctx.L.nfsp_exploitability(ctx.h, dev_w_ar0, dev_w_ar1, mode, out), "nfsp_exploitability")
    return {"br0": out[0], "br1": out[1], "exploitability": out[2], "value0": out[3]}


def exploitability_batch(ctx, dev_w_ar0: list, dev_w_ar1: list, mode: int = 0) -> list:
    """nfsp_exploitability_batch on n pairs of packed AR nets (lists of device pointers)."""
    n = len(dev_w_ar0)
    assert len(dev_w_ar1) == n
    a0 = (C.c_void_p * max(n, 1))(*dev_w_ar0)
    a1 = (C.c_void_p * max(n, 1))(*dev_w_ar1)
    out = (C.c_double * (4 * max(n, 1)))()
    native.check(ctx.L.nfsp_exploitability_batch(ctx.h, a0, a1, n, mode, out), "nfsp_exploitability_batch")
    return [{"br0": out[4 * k], "br1": out[4 * k + 1], "exploitability": out[4 * k + 2], "value0": out[4 * k + 3]}
            for k in range(n)]


def _wrap_device(addr, numel, dtype, device, owner=None) -> torch.Tensor:
    """Zero-copy torch view of device memory owned by libnfsp.  ``owner`` (the engine) is
    referenced by the view's array-interface object, which torch keeps alive with the tensor:
    the engine -- and so the memory -- outlives every view of it."""
    if numel == 0:
        return torch.empty(0, dtype=dtype, device=device)

    class _Holder:
        pass
    h = _Holder()
    h.owner = owner
    esize = torch.empty(0, dtype=dtype).element_size()
    h.__cuda_array_interface__ = {
        "shape": (int(numel),), "typestr": torch.empty(0, dtype=dtype).numpy().dtype.str,
        "data": (int(addr), False), "version": 2, "strides": (esize,)}
    return torch.as_tensor(h, device=device)
