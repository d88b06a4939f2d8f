"""The drop-in's Python-semantics switch (nfsp_amd.pyrandom; SURVEY §8(b) deal_mode).

Mode 3 is CPython 3's ``random`` itself, which the golden fixtures pin.  Mode 2 restates
CPython 2.7's integer methods (Lib/random.py 2.7: ``int(random() * n)``).  There is no
Python 2 in the image, so mode 2 is checked against that published algorithm draw for draw
(parity unpinned otherwise).
"""
import random

import numpy as np
import pytest


@pytest.fixture
def pr(pkg):
    m = pkg.pyrandom
    yield m
    m.set_python_semantics(3)


def test_mode3_is_cpython3(pr):
    pr.set_python_semantics(3)
    random.seed(11)
    a = list(range(6)); pr.shuffle(a)
    s = pr.sample(range(40000), 128)
    r = pr.randrange(1, 40001)
    d = pr.randint(0, 1)
    random.seed(11)
    b = list(range(6)); random.shuffle(b)
    assert a == b and s == random.sample(range(40000), 128)
    assert r == random.randrange(1, 40001) and d == random.randint(0, 1)


def test_mode2_follows_python27(pr):
    pr.set_python_semantics(2)
    random.seed(1234)
    a = list(range(6)); pr.shuffle(a)
    small = pr.sample(range(200), 128)          # n <= setsize (21 + 4^5): pool branch
    big = pr.sample(range(40000), 128)          # set branch
    ri = pr.randint(0, 1)
    rr = pr.randrange(1, 40001)
    random.seed(1234)
    u = random.random
    b = list(range(6))
    for i in range(5, 0, -1):                   # one draw per swap
        j = int(u() * (i + 1))
        b[i], b[j] = b[j], b[i]
    pool, want_small = list(range(200)), []
    for i in range(128):
        j = int(u() * (200 - i))
        want_small.append(pool[j])
        pool[j] = pool[200 - i - 1]
    seen, want_big = set(), []
    for _ in range(128):
        j = int(u() * 40000)
        while j in seen:
            j = int(u() * 40000)
        seen.add(j)
        want_big.append(j)
    assert a == b and small == want_small and big == want_big
    assert ri == int(u() * 2) and rr == 1 + int(u() * 40000)


def test_dropin_deal_follows_the_mode(pr, pkg):
    leduc = pkg.leduc
    for mode in (3, 2):
        pr.set_python_semantics(mode)
        random.seed(5)
        got = [leduc.deal_from_global_random() for _ in range(20)]
        random.seed(5)
        want = []
        for _ in range(20):
            cards = list(range(6))
            pr.shuffle(cards)
            want.append((cards[5] >> 1, cards[4] >> 1, cards[3] >> 1))
        assert got == want


def test_dropin_deck_deals_like_the_reference(pkg):
    """leduc.deck (the drop-in Deck) against the reference's own deals (deal_seq.npz: the
    reference Env reset + deck, CPython-3 random, 3 seeds): P0, P1 and the public card."""
    from conftest import golden
    pkg.pyrandom.set_python_semantics(3)
    for seed in (1234, 7, 99):
        ref = golden("deal_seq.npz")[f"seed{seed}"]
        random.seed(seed)
        for i in range(len(ref)):
            d = pkg.deck.Deck()
            d.shuffle()
            got = (d.pick_up().rank, d.pick_up().rank, d.pick_up().rank)
            assert got == tuple(int(x) for x in ref[i]), (seed, i)
    c = pkg.deck.Card(0, 1)
    assert c.rank == 0 and str(c) == "Ace Spades 0 1"
    assert pkg.deck.Deck().fake_pub_card().rank == -1
    assert len(pkg.deck.Deck()._cards) == 6


def test_capi_mt_deals_match_the_reference(pkg):
    """The C-ABI's host MT19937 deals (nfsp_deal_mt, the engine of nfsp_env_set_deal_mode):
    PY3_MT against the reference's own deals (deal_seq.npz, 3 seeds x 2,000 resets), PY2_MT
    against the CPython 2.7 shuffle restated in nfsp_amd.pyrandom.  Host code only: no GPU."""
    import ctypes as C
    from conftest import golden
    L = pkg.native.load()
    for seed in (1234, 7, 99):
        ref = golden("deal_seq.npz")[f"seed{seed}"]
        out = np.zeros((len(ref), 3), np.uint8)
        assert L.nfsp_deal_mt(pkg.native.DEAL_PY3_MT, seed, len(ref), out.ctypes.data_as(C.c_void_p)) == 0
        assert np.array_equal(out, ref), seed
    pr = pkg.pyrandom
    for seed in (0, 5, 2 ** 40 + 3):
        out = np.zeros((300, 3), np.uint8)
        assert L.nfsp_deal_mt(pkg.native.DEAL_PY2_MT, seed, 300, out.ctypes.data_as(C.c_void_p)) == 0
        pr.set_python_semantics(2)
        try:
            random.seed(seed)
            want = []
            for _ in range(300):
                cards = list(range(6))
                pr.shuffle(cards)
                want.append((cards[5] >> 1, cards[4] >> 1, cards[3] >> 1))
        finally:
            pr.set_python_semantics(3)
        assert np.array_equal(out, np.array(want, np.uint8)), seed
    assert L.nfsp_deal_mt(0, 1, 1, out.ctypes.data_as(C.c_void_p)) != 0     # PHILOX: refused
