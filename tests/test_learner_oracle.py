"""CPU checks of the learner oracle's sampling primitives (oracle/learner_oracle.py), against
brute-force restatements of the kernels' definitions (csrc/engine_internal.h)."""
import numpy as np

import learner_oracle as LO
from rollout_oracle import philox4x32


def test_draw_perm_is_rank_order_of_keys():
    for e in (0, 1):
        p = LO.draw_perm(128, e, LO.TAG_PERM | 3, 12345, 7, 9)
        keys = []
        for b in range(128):
            x, _, _, _ = philox4x32(np.uint32(LO.TAG_PERM | 3), np.uint32(12345), np.uint32(0),
                                    np.uint32((e << 8) | b), 7, 9)
            keys.append((int(x) & 0xFFFFFF00) | b)
        rank = [sum(k < keys[b] for k in keys) for b in range(128)]
        for b in range(128):
            assert p[rank[b]] == b


def test_sample_distinct_draws_and_redraws():
    lo, win = 100, 130                  # 128 of 130: many redraws
    s = LO.sample_distinct(128, lo, win, LO.TAG_SAMPLE | 1, 77, 5, 6)
    assert len(set(s.tolist())) == 128 and s.min() >= lo and s.max() < lo + win
    # the first pick is the first draw of lane 0 (nothing earlier can collide with it)
    x, y, _, _ = philox4x32(np.uint32(LO.TAG_SAMPLE | 1), np.uint32(77), np.uint32(0), np.uint32(0), 5, 6)
    assert s[0] == lo + ((int(x) << 32) | int(y)) % win


def test_reservoir_slots_append_then_replace():
    cap = 50
    sl = LO.reservoir_slots(1, 40, 30, cap, 3, 4)
    assert sl[:10].tolist() == list(range(40, 50))          # append while count < N
    assert all(-1 <= v < cap and v != 0 for v in sl[10:])    # j in [1, N], kept iff j < N


def test_reservoir_slots_algorithm_r_is_uniform():
    """NFSP_EXT_RESERVOIR (Algorithm R): after K inserts into N slots every insert survives
    with probability N / K; the reference's rule (utils/ReservoirBuffer.py:22-28) replaces on
    almost every insert, so its survivors are the last few hundred."""
    cap, K, trials = 40, 400, 120
    early_tb = late_tb = early_ref = 0
    for t in range(trials):
        for ext, acc in ((LO.EXT_RESERVOIR, "tb"), (0, "ref")):
            slots = LO.reservoir_slots(0, 0, K, cap, 1000 + t, 7, ext)
            owner = np.arange(cap)
            for q in range(cap, K):
                if slots[q] >= 0:
                    owner[slots[q]] = q
            kept = set(owner.tolist())
            early = sum(q in kept for q in range(1, 101))   # item 0 sits in the reference's
            # never-replaced slot 0
            late = sum(q in kept for q in range(K - 100, K))
            if acc == "tb":
                early_tb += early
                late_tb += late
            else:
                early_ref += early
    p = cap / K                          # 0.1 per insert
    assert abs(early_tb / (100 * trials) - p) < 0.02 and abs(late_tb / (100 * trials) - p) < 0.02
    assert early_ref / (100 * trials) < 0.005
