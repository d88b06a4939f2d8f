"""Static MFMA hazard check of the shipped SGD chains (tools/mfma_hazards.py): the gfx950 code
objects inside the built libnfsp.so are disassembled and every k_chain3 instance (BR, AR,
linear-Q BR; with and without the loss log; one-engine and group-table forms) is scanned for
VGPR writes to the registers of an in-flight v_mfma_f32_16x16x32_bf16:

* the compiler's model: no VALU write to SrcC within 3 wait states, none to the result within
  8 -- catches inline-asm VALU the compiler cannot pad;
* the empirical packed-f32 rule: no v_pk_fma/mul/add_f32 write of any MFMA register within
  32 states (the packed layer-2 variants that broke determinism in round 4 violate it).

The chains are the reference's fit (agent/agent.py:241-264).  No GPU needed."""
import os
import sys

import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))


@pytest.fixture(scope="module")
def hz():
    import mfma_hazards
    return mfma_hazards


def test_shipped_library_has_no_mfma_register_hazards(pkg, hz):
    import __graft_entry__
    __graft_entry__.build()
    res = hz.scan_library(pkg.native.LIB_PATH)
    # 3 chain nets x (loss log on / off) x (one engine / group table), + the MSE-Q form, + the
    # persistent group BR kernel (the chain body inlined)
    assert len(res) == 17, sorted(res)
    assert any("k_br_persist" in k for k in res), sorted(res)
    for name, r in res.items():
        assert r["mfma"] >= 80 and r["loops"] >= 1, (name, r)
        assert r["violations"] == {"srcc": 0, "dst": 0, "packed": 0}, (name, r["detail"])


def test_scan_flags_the_dropped_packed_layer2_builds(hz):
    """The PK_L2 builds round 4 dropped (AR: different weights on every run; BR: replicas that
    differed from standalone engines under CU sharing, gpurun_out/r04l.log) violate the
    packed-f32 rule in their production kernels; the compiler-model rules hold in both."""
    res = hz.scan(defines=["NFSP_PK_AR=13", "NFSP_PK_BR=5"], chains=("br", "ar"))
    for chain in ("br", "ar"):
        prod = {k: r for k, r in res[chain].items() if "ELi0ELi0E" in k or "ELi0ELi1E" in k}
        assert len(prod) == 2
        for name, r in prod.items():
            assert r["violations"]["packed"] > 0, (chain, name)
            assert r["violations"]["srcc"] == r["violations"]["dst"] == 0, (chain, name)


def test_scanner_sees_a_planted_hazard(hz):
    """The rules on a hand-written sequence: a packed write 10 states after the MFMA, a scalar
    SrcC write at 2 states, a result write at 5 -- and a loop's wrap across its back edge."""
    ins = ["v_mfma_f32_16x16x32_bf16 v[0:3], v[8:11], v[12:15], v[4:7]",
           "v_mov_b32_e32 v4, 0",                       # SrcC at 0 states
           "s_nop 3",
           "v_add_f32_e32 v1, v20, v21",                # result at 5 states
           "s_nop 4",
           "v_pk_fma_f32 v[12:13], v[20:21], v[22:23], v[24:25]",   # SrcB at 11 states, packed
           "s_nop 7", "s_nop 7", "s_nop 7", "s_nop 7",
           "v_pk_fma_f32 v[2:3], v[20:21], v[22:23], v[24:25]"]     # beyond 32 states
    r = hz.scan_kernel(ins, [])
    assert r["violations"] == {"srcc": 1, "dst": 1, "packed": 1}, r
    loop = ["v_pk_mul_f32 v[4:5], v[20:21], v[22:23]", "s_nop 0",
            "v_mfma_f32_16x16x32_bf16 v[0:3], v[8:11], v[12:15], v[4:7]"]
    r = hz.scan_kernel(loop, [(0, 3)])                  # the wrap: MFMA, then the next iteration's pk
    assert r["violations"]["packed"] == 1 and r["violations"]["srcc"] == 1, r
