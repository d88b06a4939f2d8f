"""GPU parity of the batched env C-ABI against the reference's env known-answer table
(3,408 exhaustive + 4,000 random hands, tests/golden/env_kat.npz): every hand runs
in its own env of ONE ctx, stepped in lock-step through nfsp_env_step, and every
get_state of both players after every step must match bit for bit."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def bits_of(x):
    x = x.reshape(x.shape[0], 30).cpu().numpy()
    assert np.all((x == 0) | (x == 1))
    return (x.astype(np.uint64) << np.arange(30, dtype=np.uint64)).sum(axis=1)


def test_env_kat_batched(pkg):
    nat = pkg.native
    kat = golden("env_kat.npz")
    H = len(kat["dealer"])
    ctx = nat.Context(H, seed=1)
    dev = "cuda"
    ranks = torch.as_tensor(kat["ranks"], device=dev).contiguous()
    dealer = torch.as_tensor(kat["dealer"], device=dev).contiguous()
    ctx.call("nfsp_env_set_deal", nat.ptr(ranks))
    ctx.call("nfsp_env_reset", nat.ptr(dealer))
    off = kat["snap_off"]
    s = torch.empty((H, 30), device=dev)
    a = torch.empty((H, 3), device=dev)
    r = torch.empty(H, device=dev)
    s2 = torch.empty((H, 30), device=dev)
    t = torch.empty(H, dtype=torch.uint8, device=dev)
    rnd = torch.empty(H, dtype=torch.uint8, device=dev)
    nsteps = kat["nsteps"].astype(np.int64)
    for k in range(int(nsteps.max()) + 1):
        if k > 0:
            live = nsteps >= k
            mask = torch.as_tensor(live.astype(np.uint8), device=dev)
            players = torch.as_tensor(np.where(live, kat["step_p"][:, k - 1], 0).astype(np.uint8),
                                      device=dev)
            act = torch.as_tensor(kat["step_v"][:, k - 1], device=dev).contiguous()
            ctx.call("nfsp_env_step", nat.ptr(act), 0, nat.ptr(players), nat.ptr(mask))
        ctx.call("nfsp_env_round", nat.ptr(rnd))
        sel = np.nonzero(nsteps >= k)[0]
        for p in (0, 1):
            ctx.call("nfsp_env_get_state", p, None, nat.ptr(s), nat.ptr(a), nat.ptr(r),
                     nat.ptr(s2), nat.ptr(t))
            row = off[sel] + 2 * k + p
            assert np.array_equal(bits_of(s)[sel], kat["snap_s"][row].astype(np.uint64)), (k, p)
            assert np.array_equal(bits_of(s2)[sel], kat["snap_s2"][row].astype(np.uint64)), (k, p)
            assert np.array_equal(a.cpu().numpy()[sel].astype(np.float64), kat["snap_a"][row])
            assert np.array_equal(r.cpu().numpy()[sel].astype(np.float64), kat["snap_r"][row])
            assert np.array_equal(t.cpu().numpy()[sel], kat["snap_t"][row])
    last = off[1:] - 1
    assert np.array_equal(rnd.cpu().numpy(), kat["snap_rnd"][last])


def test_env_philox_deals_are_valid_and_uniform(pkg):
    """Device-drawn deals: a legal 6-card deal (no rank 3 times), P0/P1/public
    marginals uniform over ranks; deterministic per (seed, reset)."""
    nat = pkg.native
    n = 1 << 16
    ctx = nat.Context(n, seed=99)
    dealer = torch.zeros(n, dtype=torch.uint8, device="cuda")
    ctx.call("nfsp_env_reset", nat.ptr(dealer))
    hb = torch.empty((n, 64), dtype=torch.uint8, device="cuda")
    ctx.call("nfsp_env_export", nat.ptr(hb))
    rk = hb[:, 48:51].cpu().numpy()
    assert rk.max() <= 2
    assert not np.any((rk[:, 0] == rk[:, 1]) & (rk[:, 1] == rk[:, 2]))
    for c in range(3):
        freq = np.bincount(rk[:, c], minlength=3) / n
        assert np.allclose(freq, 1 / 3, atol=0.01)
    ctx2 = nat.Context(n, seed=99)
    ctx2.call("nfsp_env_reset", nat.ptr(dealer))
    hb2 = torch.empty_like(hb)
    ctx2.call("nfsp_env_export", nat.ptr(hb2))
    assert torch.equal(hb, hb2)


def test_dropin_env_matches_oracle_with_global_random(pkg):
    """leduc.Env drop-in: the deal consumes the global `random` like the reference
    deck (tests/golden/deal_seq.npz), transitions come from the device."""
    import random
    ref = golden("deal_seq.npz")["seed1234"]
    env = pkg.leduc.Env(verbose=False)
    random.seed(1234)
    for i in range(200):
        env.reset(i & 1)
        s0 = env.get_state(0)[3].reshape(30)
        s1 = env.get_state(1)[3].reshape(30)
        assert int(np.argmax(s0[24:27])) == ref[i][0]
        assert int(np.argmax(s1[24:27])) == ref[i][1]


@pytest.mark.gpu
def test_dropin_do_action_matches_reference_kat(pkg):
    """Env.do_action / game_or_round_has_terminated called directly (do_action_kat.npz, made
    by running the reference) through the drop-in Env: nfsp_env_do_action /
    nfsp_env_round_status on the device; state read back from nfsp_env_export."""
    from test_oracle_golden import _replay_do_action
    leduc, native = pkg.leduc, pkg.native

    def make(dealer):
        e = leduc.Env(verbose=False)
        e.reset(dealer, (0, 1, 2))
        return e

    def state(e, p):
        e.ctx.call("nfsp_env_export", native.ptr(e._hand))
        h = np.frombuffer(e._hand.cpu().numpy().tobytes(), dtype=leduc.HAND_DTYPE)[0]
        return (int(h["hist"]) & 0xFFFFFF, (int(h["c0"]), int(h["c1"])),
                (int(h["raises0"]), int(h["raises1"])), int(h["slot"]), h["la"][p])
    assert _replay_do_action(make, state) == 1720


@pytest.mark.gpu
def test_env_reset_mt_deal_mode_deals_like_the_reference(pkg):
    """nfsp_env_set_deal_mode(PY3_MT, seed): nfsp_env_reset deals env 0..n-1 of every reset
    from CPython 3's shuffle of random.seed(seed) -- the reference's deals (deal_seq.npz)."""
    ref = golden("deal_seq.npz")["seed7"]
    n = 500
    ctx = pkg.native.Context(n)
    ctx.call("nfsp_env_set_deal_mode", pkg.native.DEAL_PY3_MT, 7)
    dealer = torch.zeros(n, dtype=torch.uint8, device="cuda")
    hb = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    for k in range(4):
        ctx.call("nfsp_env_reset", pkg.native.ptr(dealer))
        ctx.call("nfsp_env_export", pkg.native.ptr(hb))
        torch.cuda.synchronize()
        ranks = hb.view(n, 64)[:, 48:51].cpu().numpy()
        assert np.array_equal(ranks, ref[k * n:(k + 1) * n]), k
