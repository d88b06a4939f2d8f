#!/usr/bin/env python3
"""Static MFMA hazard scan of the SGD chains (k_chain3) in the gfx950 code the build produces.

The SGD chain (agent/agent.py:241-264, fit of the BR / AR nets) runs its layer products on
v_mfma_f32_16x16x32_bf16 and the rest on VALU.  An MFMA reads its sources and writes its result
registers while later instructions of the wave issue; the hardware does not interlock a VALU
write to those registers, so enough independent instructions ("wait states") must separate them.

Two rules, checked on every k_chain3 instance of both chain translation units, straight-line
and across each loop's back edge:

1. the compiler's own model (LLVM, ROCm 7.2, gfx950; this MFMA is a 4-pass XDL op there --
   probed: `s_nop 7` before a VALU reads its result, `s_nop 2` before a VALU overwrites its
   SrcC): no VALU write to SrcC within 3 states, none to the result within 8.  The compiler
   pads what it sees; this catches inline-asm VALU (the chains' split3 / bwd statements),
   which it does not see;
2. the empirical rule from round 4 (csrc/chain3.h PK_* notes): packed f32
   (v_pk_fma/mul/add_f32) must not write any register of an MFMA (sources or result) within
   PK_WINDOW = 32 states.  The compiler allows packed writes at 3 / 8 states like scalar ones,
   but the packed layer-2 builds (PK_L2, whose packed FMAs land 3-24 states after MFMAs that
   read or write the same registers) gave run-to-run different weights -- the AR chain alone,
   the BR chain when 4 chain workgroups shared a CU (4 waves per SIMD: an MFMA can wait behind
   3 others on the SIMD's matrix core, 3 x 8 states, plus its own 8).  In the shipped chains the
   nearest packed write to an MFMA's registers is 76 states after it (AR; none in the BR).

tests/test_mfma_hazards.py asserts both rules on the shipped build and that rule 2 flags the
dropped PK_L2 builds (-DNFSP_PK_AR=13, -DNFSP_PK_BR=5).

    python tools/mfma_hazards.py [--define NFSP_PK_AR=13] [--json]
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SRCC_WAR = 3          # compiler model: VALU write of an MFMA's SrcC, wait states after issue
DST_WAW = 8           # compiler model: VALU write (or read) of its result
PK_WINDOW = 32        # empirical: packed-f32 writes of any MFMA register
PACKED = ("v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32")
SOURCES = {"br": "learner.hip", "ar": "chain_ar.hip", "brlin": "chain_brlin.hip"}
KERNEL_PREFIX = "_ZN4nfsp5chain8k_chain3"


def is_chain_kernel(name: str) -> bool:
    """A k_chain3 instance, or the persistent group BR kernel that runs the chain body inlined
    (learner.hip k_br_persist)."""
    return name.startswith(KERNEL_PREFIX) or "k_br_persist" in name
_REG = re.compile(r"\b([vas])(?:(\d+)|\[(\d+):(\d+)\])")


def regs(tok: str) -> set:
    """VGPR / AGPR numbers named by one operand ('v5', 'v[4:7]', 'a[0:3]'); SGPRs ignored."""
    out = set()
    for m in _REG.finditer(tok):
        kind = m.group(1)
        if kind == "s":
            continue
        lo = int(m.group(2) if m.group(2) is not None else m.group(3))
        hi = int(m.group(2) if m.group(2) is not None else m.group(4))
        out |= {(kind, r) for r in range(lo, hi + 1)}
    return out


def operands(line: str) -> list:
    body = line.split(None, 1)
    if len(body) < 2:
        return []
    # operands are comma-separated; modifiers (op_sel:[..], offset:..) follow the last one
    return [t.strip() for t in re.split(r",(?![^\[]*\])", body[1])]


def wait_states(line: str) -> int:
    op = line.split()[0]
    if op == "s_nop":
        return int(line.split()[1], 0) + 1
    return 1


def vgpr_writes(line: str) -> set:
    """VGPRs the instruction writes (its first operand), for VALU / LDS / VMEM-load forms."""
    op = line.split()[0]
    if op.startswith("v_mfma"):
        return set()
    if op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return set()                      # scalar destination (vcc / exec / SGPR)
    if op.startswith(("v_", "ds_read", "ds_load", "global_load", "buffer_load", "flat_load", "scratch_load")):
        ops = operands(line)
        return regs(ops[0]) if ops else set()
    if op.startswith("ds_") and not op.startswith(("ds_write", "ds_store", "ds_swizzle", "ds_bpermute",
                                                    "ds_permute", "ds_nop")):
        ops = operands(line)              # other LDS forms with a VGPR return value
        return regs(ops[0]) if ops else set()
    if op.startswith(("ds_swizzle", "ds_bpermute", "ds_permute")):
        ops = operands(line)
        return regs(ops[0]) if ops else set()
    return set()


def functions(asm_lines: list) -> dict:
    """The k_chain3 kernels of compiler assembly (-S): name -> (instructions, loops), loops as
    (first, last + 1) index ranges of the loop bodies (label ... backward branch to it)."""
    out = {}
    i = 0
    while i < len(asm_lines):
        l = asm_lines[i]
        if is_chain_kernel(l.split(":")[0]) and l.split(":")[0].endswith("E") and not l.startswith("."):
            name = l.split(":")[0]
            ins, labels, loops = [], {}, []
            j = i + 1
            while not asm_lines[j].startswith(".Lfunc_end"):
                t = asm_lines[j].split(";")[0].strip()
                j += 1
                if not t or t.startswith("."):
                    if t.endswith(":"):
                        labels[t[:-1]] = len(ins)
                    continue
                if t.endswith(":"):
                    labels[t[:-1]] = len(ins)
                    continue
                m = re.match(r"s_(cbranch_\w+|branch)\s+(\S+)$", t)
                if m and m.group(2) in labels:             # a backward branch: a loop
                    loops.append((labels[m.group(2)], len(ins)))
                ins.append(t)
            out[name] = (ins, loops)
            i = j
        i += 1
    return out


def functions_disassembled(text: str) -> dict:
    """The same from `llvm-objdump -d` of a code object (the built library's device image):
    instruction lines carry their address in the trailing comment, branches their target."""
    out = {}
    name, ins, addr_ix, loops = None, [], {}, []
    for line in text.split("\n") + [""]:
        m = re.match(r"^([0-9a-f]+) <(\S+)>:", line)
        if m or not line.strip():
            if name and is_chain_kernel(name) and ins:
                out[name] = (ins, loops)
            if m:
                name, ins, addr_ix, loops = m.group(2), [], {}, []
            continue
        if name is None or "//" not in line:
            continue
        t, comment = line.split("//", 1)
        t = t.strip()
        am = re.match(r"\s*([0-9A-Fa-f]+):", comment)
        if not t or not am:
            continue
        addr = int(am.group(1), 16)
        addr_ix[addr] = len(ins)
        bm = re.match(r"s_(cbranch_\w+|branch)\b", t)
        tm = re.search(r"<(\S+?)(?:\+0x([0-9a-f]+))?>", comment)
        if bm and tm and tm.group(1) == name:
            base = min(addr_ix)                          # the function's first instruction
            target = base + int(tm.group(2) or "0", 16)
            if target in addr_ix and target <= addr:
                loops.append((addr_ix[target], len(ins)))
            t = bm.group(0)                              # the offset operand is not needed
        ins.append(t)
    return out


def scan_sequence(ins: list) -> list:
    """Every violation as (rule, mfma index, writer index, wait states between, writer opcode):
    rule "srcc" / "dst" (the compiler model) or "packed" (the empirical packed-f32 rule).
    Memory loads are not writers here (their data returns hundreds of cycles later)."""
    found = []
    horizon = max(SRCC_WAR, DST_WAW, PK_WINDOW)
    for i, l in enumerate(ins):
        if not l.startswith("v_mfma"):
            continue
        ops = operands(l)
        dst, srca, srcb, srcc = (regs(o) for o in ops[:4])
        every = dst | srca | srcb | srcc
        states = 0
        for j in range(i + 1, len(ins)):
            op = ins[j].split()[0]
            if op.startswith("v_") and not op.startswith("v_mfma"):
                w = vgpr_writes(ins[j])
                if w & srcc and states < SRCC_WAR:
                    found.append(("srcc", i, j, states, op))
                if w & dst and states < DST_WAW:
                    found.append(("dst", i, j, states, op))
                if op in PACKED and w & every and states < PK_WINDOW:
                    found.append(("packed", i, j, states, op))
            states += wait_states(ins[j])
            # a conditional branch falls through into what follows: keep scanning
            if states >= horizon or op.startswith(("s_branch", "s_endpgm", "s_setpc")):
                break
    return found


def scan_kernel(ins: list, loops: list) -> dict:
    hits = scan_sequence(ins)
    # each loop again across its back edge: the body followed by its own start
    for first, last in loops:
        loop = ins[first:last]                       # without the back edge: the wrap is straight-line
        wrap = scan_sequence(loop + loop[:96])
        hits += [(r, i, j, st, op) for (r, i, j, st, op) in wrap if j >= len(loop)]
    by = collections.Counter((h[0], h[3], h[4]) for h in hits)
    return {"mfma": sum(1 for l in ins if l.startswith("v_mfma")), "loops": len(loops),
            "violations": {r: sum(1 for h in hits if h[0] == r) for r in ("srcc", "dst", "packed")},
            "detail": [{"rule": r, "states": s, "writer": w, "n": n} for (r, s, w), n in sorted(by.items())]}


def asm(src: str, defines: list) -> list:
    import __graft_entry__ as g
    out = os.path.join(tempfile.mkdtemp(), os.path.basename(src) + ".s")
    subprocess.check_call([g.HIPCC, *g.HIPFLAGS, *g.FILE_FLAGS.get(src, []), *["-D" + d for d in defines],
                           "--cuda-device-only", "-S", os.path.join(g.CSRC, src), "-o", out],
                          stderr=subprocess.DEVNULL)
    with open(out) as f:
        return f.read().split("\n")


def scan(defines=(), chains=tuple(SOURCES)) -> dict:
    """{chain: {kernel: scan_kernel(...)}} for the chain kernels compiled (-S) with `defines`."""
    return {c: {name: scan_kernel(*f) for name, f in functions(asm(SOURCES[c], list(defines))).items()}
            for c in chains}


def scan_library(lib: str) -> dict:
    """{kernel: scan_kernel(...)} for every k_chain3 in a built library's gfx950 code objects
    (llvm-objdump --offloading extracts them, -d disassembles)."""
    llvm = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    d = tempfile.mkdtemp()
    copy = os.path.join(d, os.path.basename(lib))
    with open(lib, "rb") as f, open(copy, "wb") as g:
        g.write(f.read())
    subprocess.check_call([llvm, "--offloading", copy], cwd=d, stdout=subprocess.DEVNULL)
    res = {}
    for co in sorted(os.listdir(d)):
        if "gfx950" not in co:
            continue
        dis = subprocess.run([llvm, "-d", "--mcpu=gfx950", "--no-show-raw-insn", os.path.join(d, co)],
                             capture_output=True, text=True, check=True).stdout
        for name, f in functions_disassembled(dis).items():
            res[name] = scan_kernel(*f)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--define", action="append", default=[])
    ap.add_argument("--lib", default=None, help="scan a built library instead of compiling")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    res = {"lib": scan_library(a.lib)} if a.lib else scan(a.define)
    if a.json:
        print(json.dumps(res, indent=1))
        return
    for c, ks in res.items():
        for k, r in ks.items():
            print(f"{c} {k[len(KERNEL_PREFIX):]}: {r['mfma']} MFMAs, violations {r['violations']}")
            for d in r["detail"]:
                print(f"    {d['rule']:6s} at {d['states']} states by {d['writer']} x{d['n']}")


if __name__ == "__main__":
    main()
