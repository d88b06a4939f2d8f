"""ctypes binding of libnfsp (include/nfsp.h).

The product path is this library: every Env / Agent / buffer operation of the package
ends in one of these entry points.  There is no CPU fallback -- if the library or a
GPU is missing, ``lib()`` raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NFSP_LIB", os.path.join(HERE, "libnfsp.so"))

OK, EINVAL, EHIP, ENOMEM = 0, -1, -2, -3
GAME_LEDUC = 0
GAME_KUHN = 1     # the Kuhn swap-in (include/nfsp.h NFSP_GAME_KUHN)
ACT_RELU, ACT_SOFTMAX = 0, 1
QUIRK_TERMINAL_BOOTSTRAP, QUIRK_ROW0_TARGET, QUIRK_ALIAS_RL = 1, 2, 4
QUIRKS_REFERENCE = 7
# textbook-NFSP extensions (include/nfsp.h NFSP_EXT_*; not the reference's algorithm)
EXT_SL_ONEHOT, EXT_RESERVOIR, EXT_LINEAR_Q, EXT_EPS_CONST, EXT_SAMPLE_AR = 8, 16, 32, 64, 128
TEXTBOOK = EXT_SL_ONEHOT | EXT_RESERVOIR | EXT_LINEAR_Q | EXT_EPS_CONST | EXT_SAMPLE_AR
EXT_MSE_Q = 256
TEXTBOOK_MSE = TEXTBOOK | EXT_MSE_Q
TEXTBOOK_MSE_DECAY = TEXTBOOK_MSE & ~EXT_EPS_CONST      # epsilon / iteration, as the reference

P = C.c_void_p
I32, I64, U32, U64, F32, F64 = C.c_int, C.c_int64, C.c_uint, C.c_uint64, C.c_float, C.c_double


class Records(C.Structure):
    """``nfsp_records``: device column pointers of an M_RL / M_SL table."""
    _fields_ = [("s", P), ("a", P), ("r", P), ("s2", P), ("t", P), ("cap", I64)]


class EngineCfg(C.Structure):
    """``nfsp_engine_cfg``"""
    _fields_ = [("n_lanes", C.c_int32), ("hidden", C.c_int32), ("rl_capacity", I64),
                ("sl_capacity", I64), ("batch", C.c_int32), ("inserts_per_update", C.c_int32),
                ("target_every", C.c_int32), ("epochs", C.c_int32), ("fit_batch", C.c_int32),
                ("quirks", C.c_uint32), ("eta", F32), ("lr_br", F32), ("lr_ar", F32),
                ("gamma", F64), ("epsilon", F64), ("seed", U64), ("slices", C.c_int32),
                ("slice_lag", C.c_int32), ("sched", C.c_uint32)]


class GroupSched(C.Structure):
    """``nfsp_group_sched``: how a group schedules its BR rounds and slices (no result changes)"""
    _fields_ = [("br_cap", C.c_int32), ("br_pace", C.c_int32), ("br_streams", C.c_int32),
                ("serial", C.c_int32), ("br_persist", C.c_int32)]


class EngineStats(C.Structure):
    """``nfsp_engine_stats``"""
    _fields_ = [("hands", I64), ("rollouts", I64), ("rl_total", I64 * 2), ("sl_total", I64 * 2),
                ("rl_size", I64 * 2), ("sl_size", I64 * 2), ("last_rl", I64 * 2),
                ("last_sl", I64 * 2), ("br_updates", I64 * 2), ("ar_updates", I64 * 2),
                ("iteration", I64 * 2), ("target_syncs", I64 * 2), ("actions", (I64 * 3) * 2),
                ("reward", F64 * 2), ("epsilon", F64 * 2), ("temp", F64 * 2), ("lr_br", F64 * 2),
                ("exploitability", F64 * 2)]

    def to_dict(self):
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            if isinstance(v, (int, float)):
                out[name] = v
            elif name == "actions":
                out[name] = [list(v[0]), list(v[1])]
            else:
                out[name] = list(v)
        return out


PP = C.POINTER(P)
# name -> (restype, argtypes); must list every symbol include/nfsp.h declares
SIGNATURES = {
    "nfsp_last_error": (C.c_char_p, []),
    "nfsp_version": (I32, []),
    "nfsp_device_count": (I32, [C.POINTER(I32)]),
    "nfsp_create": (I32, [C.POINTER(P), I32, U64, I32, I32]),
    "nfsp_destroy": (I32, [P]),
    "nfsp_set_stream": (I32, [P, P]),
    "nfsp_synchronize": (I32, [P]),
    "nfsp_num_envs": (I32, [P]),
    "nfsp_env_set_deal": (I32, [P, P]),
    "nfsp_env_reset": (I32, [P, P]),
    "nfsp_env_set_deal_mode": (I32, [P, I32, U64]),
    "nfsp_deal_mt": (I32, [I32, U64, I64, P]),
    "nfsp_env_get_state": (I32, [P, I32, P, P, P, P, P, P]),
    "nfsp_env_step": (I32, [P, P, I32, P, P]),
    "nfsp_env_round": (I32, [P, P]),
    "nfsp_env_do_action": (I32, [P, P, I32, P, P, P]),
    "nfsp_env_round_status": (I32, [P, P]),
    "nfsp_env_export": (I32, [P, P]),
    "nfsp_mlp_forward": (I32, [P, P, I32, I32, P, P, I64]),
    "nfsp_mlp_fit": (I32, [P, P, I32, I32, P, P, I32, P, I32, I32, F32]),
    "nfsp_br_targets": (I32, [P, P, I32, P, P, P, P, P, I32, F64, U32, P, P]),
    "nfsp_buf_insert": (I32, [P, C.POINTER(Records), C.POINTER(Records), P, I64]),
    "nfsp_buf_sample": (I32, [P, C.POINTER(Records), P, I64, C.POINTER(Records)]),
    "nfsp_engine_default_cfg": (I32, [C.POINTER(EngineCfg)]),
    "nfsp_engine_create": (I32, [P, C.POINTER(EngineCfg), C.POINTER(P)]),
    "nfsp_engine_destroy": (I32, [P]),
    "nfsp_engine_weights": (I32, [P, I32, I32, PP]),
    "nfsp_rollout": (I32, [P]),
    "nfsp_rollout_with": (I32, [P, P, P]),
    "nfsp_engine_update": (I32, [P]),
    "nfsp_engine_step": (I32, [P]),
    "nfsp_engine_get_stats": (I32, [P, C.POINTER(EngineStats)]),
    "nfsp_engine_memories": (I32, [P, I32, C.POINTER(Records), C.POINTER(I64), C.POINTER(Records),
                                   PP, PP, PP]),
    "nfsp_engine_last_update": (I32, [P, I32, I32, PP, PP]),
    "nfsp_engine_lane_counts": (I32, [P, PP]),
    "nfsp_exploitability": (I32, [P, P, P, I32, P]),
    "nfsp_exploitability_batch": (I32, [P, P, P, I32, I32, P]),
    "nfsp_engine_set_loss_log": (I32, [P, I32]),
    "nfsp_engine_losses": (I32, [P, P]),
    "nfsp_engine_set_timing": (I32, [P, I32]),
    "nfsp_engine_get_timings": (I32, [P, C.POINTER(F64), C.POINTER(I64)]),
    "nfsp_engine_set_update_limit": (I32, [P, I64]),
    "nfsp_engine_snapshot": (I32, [P, I32, PP, P]),
    "nfsp_group_create": (I32, [P, C.POINTER(EngineCfg), I32, U32, C.POINTER(P)]),
    "nfsp_group_destroy": (I32, [P]),
    "nfsp_group_engine": (I32, [P, I32, C.POINTER(P)]),
    "nfsp_group_step": (I32, [P]),
    "nfsp_group_average_ar": (I32, [P]),
    "nfsp_group_set_timing": (I32, [P, I32]),
    "nfsp_group_get_timings": (I32, [P, C.POINTER(F64), C.POINTER(I64)]),
    "nfsp_group_rounds": (I32, [P, C.POINTER(I64)]),
    "nfsp_group_check": (I32, [P]),
    "nfsp_group_set_trace": (I32, [P, I32]),
    "nfsp_group_trace": (I32, [P, C.POINTER(I32), I64, C.POINTER(I64)]),
    "nfsp_group_set_exchange": (I32, [P, U32, I32, F32]),
    "nfsp_group_default_sched": (I32, [C.POINTER(GroupSched)]),
    "nfsp_group_set_sched": (I32, [P, C.POINTER(GroupSched)]),
    "nfsp_group_get_sched": (I32, [P, C.POINTER(GroupSched)]),
    "nfsp_engine_set_exchange": (I32, [P, I32, F32, P, P, P]),
    "nfsp_engine_exchanges": (I32, [P, C.POINTER(I64)]),
    "nfsp_rccl_ready": (I32, [I32]),
    "nfsp_rccl_unique_id": (I32, [P]),
    "nfsp_rccl_comm_create": (I32, [P, I32, I32, I32, C.POINTER(P)]),
    "nfsp_rccl_comm_destroy": (I32, [P]),
}
# int (*nfsp_exchange_fn)(void* user, float* dev_sum, int64_t n)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, P, P, I64)
GROUP_AVG_AR = 1
XCHG_AR, XCHG_BR = 1, 2
DEAL_PHILOX, DEAL_PY3_MT, DEAL_PY2_MT = 0, 1, 2
GROUP_MAX_REPLICAS = 256

_LIB = None


class NativeError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """dlopen libnfsp and bind every signature (no GPU needed)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise NativeError(f"libnfsp not built: {path} is missing (run __graft_entry__.build())")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def lib():
    """The library, on a machine that has a HIP device; raises otherwise (no fallback)."""
    L = load()
    n = I32(0)
    rc = L.nfsp_device_count(C.byref(n))
    if rc != OK or n.value < 1:
        raise NativeError("libnfsp needs a HIP device (none visible): "
                          + L.nfsp_last_error().decode())
    return L


def check(rc: int, what: str = ""):
    if rc != OK:
        raise NativeError(f"{what} failed ({rc}): {load().nfsp_last_error().decode()}")


def ptr(t) -> P:
    """Device pointer of a torch tensor (or None -> NULL)."""
    return None if t is None else P(t.data_ptr())


def stream_handle():
    import torch
    return P(torch.cuda.current_stream().cuda_stream)


class Context:
    """Owns one ``nfsp_ctx`` (n envs on the current device), bound to torch's stream."""

    def __init__(self, n_envs: int, seed: int = 1234, device: int | None = None, game: int = GAME_LEDUC):
        import torch
        L = lib()
        self.L = L
        dev = torch.cuda.current_device() if device is None else device
        h = P()
        check(L.nfsp_create(C.byref(h), int(n_envs), int(seed) & (2**64 - 1), int(game), dev),
              "nfsp_create")
        self.h = h
        self.n = int(n_envs)
        check(L.nfsp_set_stream(h, stream_handle()), "nfsp_set_stream")

    def call(self, name, *args):
        check(getattr(self.L, name)(self.h, *args), name)

    def close(self):
        if getattr(self, "h", None):
            self.L.nfsp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
