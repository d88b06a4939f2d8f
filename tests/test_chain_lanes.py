"""The SGD chain's loss-lane layout and its 32-sample sums, checked on the host (no GPU).

csrc/chain3.h k_chain3 (round 4): every wave computes the loss of the 32 minibatch samples in
its 64 lanes, lane (g, c) = 16 g + c holding sample

    ls(g, c) = 4 ((g & 2) | ((g & 1) ^ (c >> 3))) + (c & 3) + 16 ((c >> 2) & 1)

so that the backward can take the gradients of its slot j (samples 4g + j and 16 + 4g + j - 4,
the rows of the sample-major Z1 layout) from lane j of its own row by DPP row_newbcast:j
(bwd_dpp).  The gb2 sums and the loss log add the 32 per-sample values in round 3's exact order
(tot32 / tot32_pair), although round 3 held sample c in lane c of rows 0 / 1 and 16 + c in rows
2 / 3.  This restates the cross-lane operations on float32 lane vectors and checks both claims
bit for bit:

* row_ror:k (DPP 0x120 + k): lane c of a 16-lane row reads lane (c - k) mod 16;
* quad_perm [2,3,0,1] (0x4E) / [1,0,3,2] (0xB1): lane c reads c ^ 2 / c ^ 1;
* v_permlane32_swap(a, b): a' = [a_lo, b_lo], b' = [a_hi, b_hi] (halves of 32 lanes), so
  a' + b' adds lane l and l ^ 32 of a in lanes 0..31 and of b in lanes 32..63.
"""
import numpy as np


def ls(g, c):
    return 4 * ((g & 2) | ((g & 1) ^ (c >> 3))) + (c & 3) + 16 * ((c >> 2) & 1)


LS = np.array([ls(l >> 4, l & 15) for l in range(64)])


def ror(x, k):
    """DPP row_ror:k on a 64-lane vector"""
    out = np.empty_like(x)
    for l in range(64):
        row, c = l & ~15, l & 15
        out[l] = x[row + ((c - k) % 16)]
    return out


def qperm(x, xor):
    return x[np.arange(64) ^ xor]


def swap32_sum(a, b):
    """r = permlane32_swap(a, b); r[0] + r[1]"""
    r0 = np.concatenate([a[:32], b[:32]])
    r1 = np.concatenate([a[32:], b[32:]])
    return (r0 + r1).astype(np.float32)


def tot_rows(x):
    x = (x + ror(x, 8)).astype(np.float32)
    x = (x + qperm(x, 2)).astype(np.float32)
    x = (x + qperm(x, 1)).astype(np.float32)
    return (x + ror(x, 4)).astype(np.float32)


def tot32(x):
    return tot_rows(swap32_sum(x, x))


def tot32_pair(a, b):
    return tot_rows(swap32_sum(a, b))


def round3_rows(d):
    """round 3's lane layout (sample c in lane c of rows 0 / 1, 16 + c in rows 2 / 3) and its
    per-row sums: DPP x + row_ror(x) for 8, 4, 2, 1 (bound_ctrl: every lane has a source)"""
    x = np.array([d[16 * ((l >> 4) >> 1) + (l & 15)] for l in range(64)], np.float32)
    for k in (8, 4, 2, 1):
        x = (x + ror(x, k)).astype(np.float32)
    return x


def round3_total(d):
    """round 3's 32-sample total: the row sums of rows g and g ^ 2 added (the U swap)"""
    x = round3_rows(d)
    return swap32_sum(x, x)


def _vectors(rng, n):
    for i in range(n):
        scale = 10.0 ** rng.uniform(-9, 3)
        v = (rng.standard_normal(32) * scale).astype(np.float32)
        if i % 3 == 1:
            v[rng.random(32) < 0.5] = 0.0          # masked gradients (ReLU / Huber zeros)
        if i % 3 == 2:
            v *= (10.0 ** rng.uniform(-6, 6, 32)).astype(np.float32)   # mixed magnitudes
        yield v.astype(np.float32)


def test_every_backward_slot_finds_its_sample_in_lane_j_of_its_row():
    for g in range(4):
        for j in range(8):
            assert LS[16 * g + j] == 4 * g + (j & 3) + 16 * (j >> 2)


def test_rows_g_and_g_xor_1_hold_the_same_16_samples_and_every_sample_twice():
    for g in (0, 2):
        a, b = set(LS[16 * g:16 * g + 16]), set(LS[16 * (g + 1):16 * (g + 2)])
        assert len(a) == 16 and a == b
    assert sorted(np.bincount(LS, minlength=32)) == [2] * 32
    # rows 0 / 1 and rows 2 / 3 split the samples by bit 3 (the s, s ^ 8 pairs are cross-row)
    assert set(LS[:32]) == {s for s in range(32) if not s & 8}


def test_tot32_adds_in_round_3s_order_bit_for_bit():
    rng = np.random.default_rng(7)
    for d in _vectors(rng, 300):
        new = tot32(d[LS])
        old = round3_total(d)
        assert np.array_equal(new.view(np.uint32), np.full(64, old[0]).view(np.uint32)), (new, old)
        assert np.all(old == old[0])


def test_tot32_pair_gives_rows_01_the_first_total_and_rows_23_the_second():
    rng = np.random.default_rng(11)
    vs = list(_vectors(rng, 200))
    for a, b in zip(vs[::2], vs[1::2]):
        got = tot32_pair(a[LS], b[LS])
        ta, tb = round3_total(a)[0], round3_total(b)[0]
        assert np.array_equal(got[:32].view(np.uint32), np.full(32, ta).view(np.uint32))
        assert np.array_equal(got[32:].view(np.uint32), np.full(32, tb).view(np.uint32))


def test_the_loss_log_total_matches_round_3s():
    """round 3 zeroed rows 1 and 3 before its row sums and took sum_x32(sum_x16(.)); the
    32 distinct (non-negative) loss terms give the same float as tot32 of the duplicated lanes"""
    rng = np.random.default_rng(3)
    for i in range(200):
        L = np.abs(rng.standard_normal(32) * 10.0 ** rng.uniform(-4, 2)).astype(np.float32)
        x = np.array([L[16 * ((l >> 4) >> 1) + (l & 15)] if ((l >> 4) & 1) == 0 else 0.0
                      for l in range(64)], np.float32)
        for k in (8, 4, 2, 1):
            x = (x + ror(x, k)).astype(np.float32)
        x16 = (x + x[np.arange(64) ^ 16]).astype(np.float32)
        old = swap32_sum(x16, x16)
        assert np.array_equal(tot32(L[LS]).view(np.uint32), old.view(np.uint32))
