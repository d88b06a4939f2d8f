#!/usr/bin/env python3
"""Instruction census of the SGD chain's step loop (k_chain3), from the gfx950 assembly of
the two translation units as __graft_entry__ builds them (learner.hip: BR, chain_ar.hip: AR).

For each chain it counts the instructions of the loop body (one SGD step) by class and
prices their issue with the per-instruction constants of MI355X_MICROARCH.md ('vector-
instruction ISSUE cost, one wave's stream on one SIMD'): VALU 4 cycles, transcendental
(v_exp / v_log / v_rcp / v_rsq / v_sqrt) 8, v_mfma_f32_16x16x32_bf16 8 (it holds the SIMD's
vector issue for 8 of its 16 cycles), s_nop 4; LDS / VMEM / SALU / waitcnt / branch 1.
bench.py divides that issue estimate by the measured cycles per step: the fraction of a
step one wave spends issuing (the chain is one wave per SIMD, so nothing else fills it).

    python tools/chain_census.py > profiles/r04_chain_census.json
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

KERNELS = {"br": ("learner.hip", "_ZN4nfsp5chain8k_chain3ILi1ELi0E"),
           "ar": ("chain_ar.hip", "_ZN4nfsp5chain8k_chain3ILi0ELi0E")}
TRANS = ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32")


def asm(src):
    import __graft_entry__ as g
    out = os.path.join(tempfile.mkdtemp(), os.path.basename(src) + ".s")
    subprocess.check_call([g.HIPCC, *g.HIPFLAGS, *g.FILE_FLAGS.get(src, []), "--cuda-device-only", "-S",
                           os.path.join(g.CSRC, src), "-o", out], stderr=subprocess.DEVNULL)
    return open(out).read().split("\n")


def loop_body(lines, kernel):
    """The step loop's instructions from its header to its back edge.  Blocks placed after the
    back edge (the AR chain's rarely taken clipped-softmax block) are not counted: the census
    is the common path."""
    start = next(i for i, l in enumerate(lines) if l.startswith(kernel))
    stop = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    best = None
    for h in [i for i in range(start, stop) if "Loop Header" in lines[i]]:
        lab = lines[h].split(":")[0]
        end = next((i for i in range(h, stop)
                    if re.search(r"s_(cbranch_\w+|branch)\s+" + re.escape(lab) + r"\s*$", lines[i])), None)
        if end is None:
            continue
        body = [l.strip() for l in lines[h + 1:end + 1]
                if l.strip() and not l.strip().startswith((";", "."))]
        if best is None or len(body) > len(best):
            best = body
    return best


def price(op):
    if op.startswith("v_mfma"):
        return "mfma", 8
    if op.startswith(TRANS):
        return "trans", 8
    if op.startswith("v_dot2"):        # two passes (MI355X_MICROARCH: ~10 beside MFMAs)
        return "dot2", 8
    if op.startswith("v_"):
        return "valu", 4
    if op == "s_nop":
        return "nop", 4
    if op.startswith("ds_"):
        return "lds", 1
    if op.startswith(("global_", "buffer_")):
        return "vmem", 1
    return "salu/other", 1


def main():
    out = {"source": "tools/chain_census.py (gfx950 assembly with the build's flags)",
           "prices": "MI355X_MICROARCH.md issue costs: VALU 4, transcendental 8, v_dot2 8, "
                     "MFMA 16x16x32 8, s_nop 4, other 1 cycle"}
    for name, (src, kern) in KERNELS.items():
        body = loop_body(asm(src), kern)
        ops = collections.Counter(l.split()[0] for l in body)
        cls = collections.Counter()
        cyc = collections.Counter()
        for op, n in ops.items():
            k, c = price(op)
            cls[k] += n
            cyc[k] += n * c
        # the loop may hold several SGD steps (k_chain3 unrolls by 4 when the steps per update
        # are a multiple of 4): one s_barrier per step
        steps = max(ops.get("s_barrier", 1), 1)
        out[name] = {"instructions": len(body), "steps_per_iteration": steps,
                     "instructions_per_step": len(body) / steps,
                     "by_class": {k: v / steps for k, v in cls.items()},
                     "issue_cycles": {k: v / steps for k, v in cyc.items()},
                     "issue_cycles_per_step": sum(cyc.values()) / steps}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
