"""The SGD chain's step-record layout and its LDS reads, checked on the host (no GPU).

csrc/engine_internal.h StepRec / fa_slot and csrc/chain3.h k_chain3: the prep kernels store
each minibatch's observations as bf16 0/1 MFMA fragments fa[g][fa_slot(g, s)] (16 bytes per
sample s and lane row g); the chain reads

* the layer-1 operand X (sample-major) with 16-byte reads fa[g][c ^ 12 (g & 1)], and
* the dW1 operand X^T (input-major, K = samples) with ds_read_b64_tr_b16 from the same image.

This restates the gfx950 transposed read (cdna_hip_programming.md T10: per 16-lane group,
lane 4q + p supplies the address of row q, columns 4p .. 4p + 3; lane i receives column i of
the four rows, row q in element q) and the LDS bank rules (MI355X_MICROARCH.md §LDS), and
checks that every lane receives exactly the operand the chain's MFMAs assume, and the
conflict degrees the design states (row reads conflict-free, transposed reads 2-way).
"""
import numpy as np

ONE = 0x3F80          # bf16 1.0
BIAS_IN = 30          # CHAIN_BIAS_IN: input 30 is the constant 1


def fa_slot(g, s):
    return s ^ (12 * (g & 1))


def k_input(g, j):
    """layer-1 K slot 8g + j <-> input 4g + j (j < 4) or 16 + 4g + j - 4"""
    return 4 * g + j if j < 4 else 16 + 4 * g + j - 4


def fa_image(x):
    """The fa part of a StepRec as 16-bit words: [g][slot][8] (emit_recs)."""
    img = np.zeros((4, 32, 8), np.uint16)
    for s in range(32):
        for g in range(4):
            for j in range(8):
                img[g, fa_slot(g, s), j] = ONE if (x[s] >> k_input(g, j)) & 1 else 0
    return img


def tr_read(words, addr):
    """ds_read_b64_tr_b16 of a wave: addr[l] = byte offset supplied by lane l (8-byte aligned,
    4 contiguous 16-bit elements of one row); returns out[l][q] (4 elements per lane)."""
    out = np.zeros((64, 4), np.uint16)
    for grp in range(4):
        for i in range(16):
            p = i // 4
            for q in range(4):
                a = addr[16 * grp + 4 * q + p]
                out[16 * grp + i, q] = words[a // 2 + (i % 4)]
    return out


def tr_offsets():
    """chain3.h: tr_off = 512 (c & 3) + 16 fa_slot(c & 3, 4g + (c >> 2)), lane l = 16g + c"""
    return np.array([512 * (c & 3) + 16 * fa_slot(c & 3, 4 * g + (c >> 2))
                     for g in range(4) for c in range(16)])


def test_fa_slot_is_an_involution_per_row():
    for g in range(4):
        slots = [fa_slot(g, s) for s in range(32)]
        assert sorted(slots) == list(range(32))
        assert all(fa_slot(g, fa_slot(g, s)) == s for s in range(32))


def test_row_reads_give_the_layer1_operand():
    rng = np.random.RandomState(5)
    x = (rng.randint(0, 1 << 30, size=32) | (1 << BIAS_IN)).astype(np.int64)
    img = fa_image(x)
    for g in range(4):
        for c in range(16):
            sw = 12 * (g & 1)
            for half, s in ((0, c), (1, 16 + c)):      # fa0: sample c, fa1: sample 16 + c
                got = img[g, s ^ sw]
                want = [ONE if (x[s] >> k_input(g, j)) & 1 else 0 for j in range(8)]
                assert list(got) == want


def test_transposed_reads_give_the_dw1_operand():
    """ba0 lane (g, c): input c of samples 4g + j (j < 4) and 16 + 4g + j - 4; ba1: input
    16 + c -- the four reads at tr_off, +256, +8, +264 (chain3.h tr_pair)."""
    rng = np.random.RandomState(11)
    for trial in range(20):
        x = (rng.randint(0, 1 << 30, size=32) | (1 << BIAS_IN)).astype(np.int64)
        words = fa_image(x).reshape(-1)
        off = tr_offsets()
        lo0, hi0 = tr_read(words, off), tr_read(words, off + 256)
        lo1, hi1 = tr_read(words, off + 8), tr_read(words, off + 264)
        for l in range(64):
            g, c = l >> 4, l & 15
            for j in range(8):
                smp = 4 * g + j if j < 4 else 16 + 4 * g + j - 4
                got0 = (lo0 if j < 4 else hi0)[l, j & 3]
                got1 = (lo1 if j < 4 else hi1)[l, j & 3]
                assert got0 == (ONE if (x[smp] >> c) & 1 else 0), (trial, l, j)
                assert got1 == (ONE if (x[smp] >> (16 + c)) & 1 else 0), (trial, l, j)


def _ways(addrs_bytes, nbytes, lanes, modulus=64):
    """worst bank multiplicity over distinct dword addresses of one lane group"""
    banks = {}
    for l in lanes:
        for k in range(nbytes // 4):
            dw = addrs_bytes[l] // 4 + k
            banks.setdefault(dw % modulus, set()).add(dw)
    return max(len(v) for v in banks.values())


def test_bank_conflicts_as_stated():
    # 16-byte row reads fa[g][c ^ sw] (and the +16-sample read): ds_read_b128 lane groups
    groups = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
              list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
              list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
              list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]
    for plus in (0, 16):
        row = [512 * (l >> 4) + 16 * ((((l & 15) + plus)) ^ (12 * ((l >> 4) & 1))) for l in range(64)]
        assert max(_ways(row, 16, grp) for grp in groups) == 1
    # the transposed reads: 2 lane groups of 32, 2-way at worst (4-way without the swizzle)
    off = tr_offsets()
    for extra in (0, 256, 8, 264):
        a = off + extra
        assert max(_ways(a, 8, range(h * 32, h * 32 + 32)) for h in (0, 1)) == 2
    plain = np.array([512 * (c & 3) + 16 * (4 * g + (c >> 2)) for g in range(4) for c in range(16)])
    assert max(_ways(plain, 8, range(h * 32, h * 32 + 32)) for h in (0, 1)) == 4
