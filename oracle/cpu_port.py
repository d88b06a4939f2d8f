"""TEST INFRASTRUCTURE ONLY -- ctypes binding of oracle/nfsp_cpu.cpp (the C++ restatement
of main.train).  Only tests/ and bench.py's cpu_baseline leg import this module.

``CpuGame`` mirrors ``nfsp_oracle.make_main`` + ``nfsp_oracle.train``; ``bench`` runs
independent replicas on host threads (the CPU side of bench.py).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libnfsp_cpu.so")


class Cfg(C.Structure):
    _fields_ = [("rl_capacity", C.c_int64), ("sl_capacity", C.c_int64),
                ("lr_br", C.c_double), ("lr_ar", C.c_double), ("gamma", C.c_double),
                ("epsilon", C.c_double), ("eta", C.c_double),
                ("batch", C.c_int32), ("target_every", C.c_int32),
                ("seed", C.c_int64), ("init_seed", C.c_int64),
                ("quirks", C.c_int32), ("game", C.c_int32), ("workload", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("hands", C.c_int64)] + [
        (n, C.c_int64 * 2) for n in ("rl_inserts", "sl_inserts", "rl_size", "sl_size", "iteration",
                                     "br_updates", "ar_updates", "game_step", "played")] + [
        ("actions", (C.c_double * 3) * 2)] + [
        (n, C.c_double * 2) for n in ("reward", "epsilon", "lr_br", "temp", "exploitability")] + [
        ("warnings", C.c_int64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        L.nfsp_cpu_create.restype = C.c_void_p
        L.nfsp_cpu_create.argtypes = [C.POINTER(Cfg)]
        L.nfsp_cpu_destroy.argtypes = [C.c_void_p]
        L.nfsp_cpu_train.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p]
        L.nfsp_cpu_get_stats.argtypes = [C.c_void_p, C.POINTER(Stats)]
        L.nfsp_cpu_weights.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
        L.nfsp_cpu_rl.restype = C.c_int64
        L.nfsp_cpu_rl.argtypes = [C.c_void_p, C.c_int32, C.c_int64] + [C.c_void_p] * 5
        L.nfsp_cpu_sl.restype = C.c_int64
        L.nfsp_cpu_sl.argtypes = [C.c_void_p, C.c_int32, C.c_int64, C.c_void_p, C.c_void_p]
        L.nfsp_cpu_bench.restype = C.c_int64
        L.nfsp_cpu_bench.argtypes = [C.POINTER(Cfg), C.c_int32, C.c_double, C.POINTER(C.c_double)]
        assert L.nfsp_cpu_cfg_size() == C.sizeof(Cfg) and L.nfsp_cpu_stats_size() == C.sizeof(Stats)
        _lib = L
    return _lib


WORKLOADS = {"c": 0, "a": 1, "b": 2}     # (c) end to end, (a) env + scheduler, (b) play


def make_cfg(cfg=None, init_seed=0, quirks=True, game="leduc", rl_capacity=None, sl_capacity=None,
             workload="c"):
    """nfsp_oracle.DEFAULT_CFG (+ overrides) as the C struct; both memories default to cfg buffer."""
    import nfsp_oracle as orc
    c = dict(orc.DEFAULT_CFG, **(cfg or {}))
    return Cfg(rl_capacity=rl_capacity or c["buffer"], sl_capacity=sl_capacity or c["buffer"],
               lr_br=c["lr_br"], lr_ar=c["lr_ar"], gamma=c["gamma"], epsilon=c["epsilon"],
               eta=c["eta"], batch=c["batch"], target_every=c["target_every"], seed=c["seed"],
               init_seed=init_seed, quirks=int(bool(quirks)), game=1 if game == "kuhn" else 0,
               workload=WORKLOADS[workload])


class CpuGame:
    """make_main(cfg, init_seed, quirks) + train(...) of nfsp_oracle, in C++."""

    def __init__(self, cfg: Cfg):
        self.L = lib()
        self.cfg = cfg
        self.h = self.L.nfsp_cpu_create(C.byref(cfg))

    def train(self, episodes: int, stats_every: int = 100):
        curve = np.zeros(max(1, episodes // max(stats_every, 1) + 1))
        n = C.c_int64()
        self.L.nfsp_cpu_train(self.h, episodes, stats_every, curve.ctypes.data, C.addressof(n))
        return list(curve[:n.value])

    def stats(self) -> dict:
        st = Stats()
        self.L.nfsp_cpu_get_stats(self.h, C.byref(st))
        out = {}
        for name, _ in Stats._fields_:
            v = getattr(st, name)
            if name == "actions":
                out[name] = [list(v[0]), list(v[1])]
            elif hasattr(v, "__len__"):
                out[name] = list(v)
            else:
                out[name] = v
        return out

    def weights(self, agent: int, net: int) -> np.ndarray:
        w = np.zeros(2179, np.float32)
        assert self.L.nfsp_cpu_weights(self.h, agent, net, w.ctypes.data) == 0
        return w

    def rl(self, agent: int):
        n = int(self.cfg.rl_capacity)
        s, s2 = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        a, r, t = np.zeros((n, 3)), np.zeros(n), np.zeros(n, np.uint8)
        k = self.L.nfsp_cpu_rl(self.h, agent, n, s.ctypes.data, a.ctypes.data, r.ctypes.data,
                               s2.ctypes.data, t.ctypes.data)
        return s[:k], a[:k], r[:k], s2[:k], t[:k]

    def sl(self, agent: int):
        n = int(self.cfg.sl_capacity)
        s, a = np.zeros(n, np.uint32), np.zeros((n, 3))
        k = self.L.nfsp_cpu_sl(self.h, agent, n, s.ctypes.data, a.ctypes.data)
        return s[:k], a[:k]

    def close(self):
        if self.h:
            self.L.nfsp_cpu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def bench(cfg: Cfg, threads: int, seconds: float):
    """Independent replicas (seed + i) on `threads` host threads -> (hands, wall seconds)."""
    el = C.c_double()
    hands = lib().nfsp_cpu_bench(C.byref(cfg), threads, seconds, C.byref(el))
    return int(hands), el.value
