#!/usr/bin/env python3
"""Learner-chain cycle split inside the engine (diagnostic).

Builds libnfsp with -DNFSP_CHAIN_STAMPS into build/, runs the C3 engine through it and
reads the chains' accumulated s_memtime phase cycles (shader clock) next to their
HIP-event durations: cycles / event time = the effective shader clock while the chain ran.

    python tools/chain_clock.py [--lanes N] [--steps K]
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PHASES = ["fwd-mfma", "layer2+po", "barrier", "loss+gb2", "bwd+dW1", "update+load"]


def build():
    import __graft_entry__ as g
    out = os.path.join(REPO, "build", "libnfsp_stamps.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    srcs = [os.path.join(g.CSRC, f) for f in sorted(os.listdir(g.CSRC)) if f.endswith(".hip")]
    if not os.path.exists(out) or any(os.path.getmtime(s) > os.path.getmtime(out) for s in srcs):
        subprocess.check_call([g.HIPCC, *g.HIPFLAGS, "-DNFSP_CHAIN_STAMPS", "-shared", "-o", out, *srcs])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=1_048_576)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    lib = build()
    if args.build_only:
        return
    os.environ["NFSP_LIB"] = lib
    import torch
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    eng = pkg.engine.SelfPlayEngine(n_lanes=args.lanes, rl_capacity=200_000, sl_capacity=2_000_000, seed=1234)
    L = C.CDLL(lib)
    L.nfsp_debug_chain_stamps.argtypes = [C.c_void_p]
    buf = (C.c_ulonglong * 320)()          # [8][4][10]: RELU * 2 + block
    for _ in range(2):
        eng.step()
    torch.cuda.synchronize()
    L.nfsp_debug_chain_stamps(buf)          # reset
    eng.set_timing(True)
    eng.timings()
    for _ in range(args.steps):
        eng.step()
    torch.cuda.synchronize()
    t = eng.timings()
    assert L.nfsp_debug_chain_stamps(buf) == 0
    st = [[[buf[(b * 4 + w) * 10 + k] for k in range(10)] for w in range(4)] for b in range(4)]
    for b, (name, key) in enumerate([("AR block 0", "k_chain3_ar"), ("AR block 1", "k_chain3_ar"),
                                     ("BR (all segments)", "k_chain3_br")]):
        w0 = st[b][0]
        steps = w0[9]
        if not steps:
            continue
        cyc = w0[8]
        ms = t[key][0]
        print(f"{name}: {steps} steps, {cyc / steps:.0f} cycles/step, kernel events {ms:.1f} ms "
              f"-> {ms * 1e3 / steps:.3f} us/step, effective clock {cyc / (ms * 1e-3) / 1e9:.2f} GHz"
              + ("" if b < 2 else " (BR: sum over agents' segments, clock approximate)"))
        print("   phases/step: " + " ".join(f"{p}={w0[k] / steps:.0f}" for k, p in enumerate(PHASES)))


if __name__ == "__main__":
    main()
