"""GPU parity of the network kernels against oracle/nn_oracle.py.

Tolerances (north_star: "network outputs match within a stated fp32 tolerance"):
* predict, ReLU head: BIT-EXACT (same fixed summation order, no FMA contraction);
* predict, softmax head: |delta| <= 1e-6 (device expf vs numpy exp, ~1 ulp);
* fit (8 SGD steps): weights |delta| <= 1e-5 (parallel gradient sums);
* BR targets: |delta| <= 1e-6, exploitability proxy |delta| <= 1e-6.
"""
import numpy as np
import pytest
import torch

import nfsp_oracle as orc
import nn_oracle as nn

pytestmark = pytest.mark.gpu


def dev(x, dtype=None):
    return torch.as_tensor(np.ascontiguousarray(x), device="cuda", dtype=dtype)


def make(pkg, act, seed):
    ctx = pkg.native.Context(1)
    m = pkg.agent.DeviceMLP(act, 64, np.random.RandomState(seed), ctx)
    o = nn.MLP(act, 64, weights=m.get_weights())
    return m, o


@pytest.mark.parametrize("B", [1, 7, 128, 5000])
def test_predict_relu_bit_exact(pkg, B):
    m, o = make(pkg, nn.ACT_RELU, B)
    rng = np.random.RandomState(B)
    x = (rng.rand(B, 1, 30) < 0.3).astype(np.float32)
    assert np.array_equal(m.predict(x), o.predict(x))


def test_predict_relu_nonbinary_inputs_bit_exact(pkg):
    m, o = make(pkg, nn.ACT_RELU, 5)
    x = np.random.RandomState(0).randn(300, 1, 30).astype(np.float32)
    assert np.array_equal(m.predict(x), o.predict(x))


@pytest.mark.parametrize("B", [1, 128, 4096])
def test_predict_softmax(pkg, B):
    m, o = make(pkg, nn.ACT_SOFTMAX, 10 + B)
    x = (np.random.RandomState(B).rand(B, 1, 30) < 0.3).astype(np.float32)
    y, yo = m.predict(x), o.predict(x)
    assert np.abs(y - yo).max() <= 1e-6
    assert np.allclose(y.sum(-1), 1.0, atol=1e-6)


@pytest.mark.parametrize("act", [nn.ACT_RELU, nn.ACT_SOFTMAX])
def test_fit_matches_keras_restatement(pkg, act):
    m, o = make(pkg, act, 21 + act)
    rng = np.random.RandomState(4)
    x = (rng.rand(128, 30) < 0.3).astype(np.float32)
    if act == nn.ACT_RELU:
        t = (rng.rand(128, 3) * 3).astype(np.float32)      # regression targets
    else:
        t = rng.rand(128, 3).astype(np.float32)            # unnormalised SL targets
    np.random.seed(5)
    perms = m.fit_device(dev(x), dev(t), 0.1)
    o.fit(x, t, np.float32(0.1), perms=perms)
    for a, b in zip(m.get_weights(), o.get_weights()):
        assert np.abs(a - b).max() <= 1e-5


def test_fit_ce_clip_edge(pkg):
    """A saturated softmax (p < 1e-7) exercises the clip mask of the CE gradient."""
    m, o = make(pkg, nn.ACT_SOFTMAX, 3)
    ws = m.get_weights()
    ws[3] = np.array([40.0, 0.0, -40.0], np.float32)
    m.set_weights(ws)
    o.set_weights(ws)
    x = np.zeros((32, 30), np.float32)
    t = np.ones((32, 3), np.float32)
    perms = m.fit_device(dev(x), dev(t), 0.1, epochs=1)
    o.fit(x, t, np.float32(0.1), perms=perms, epochs=1)
    for a, b in zip(m.get_weights(), o.get_weights()):
        assert np.abs(a - b).max() <= 1e-5


@pytest.mark.parametrize("quirks", [3, 0])
def test_br_targets(pkg, quirks):
    nat = pkg.native
    m, o = make(pkg, nn.ACT_RELU, 77)
    rng = np.random.RandomState(8)
    n = 128
    s = (rng.rand(n, 30) < 0.3).astype(np.float32)
    s2 = (rng.rand(n, 30) < 0.3).astype(np.float32)
    a = rng.rand(n, 3).astype(np.float32)
    r = (rng.randint(-10, 11, size=n) * 0.5).astype(np.float32)
    t = (rng.rand(n) < 0.3).astype(np.uint8)
    out = torch.empty((n, 3), device="cuda")
    ex = torch.zeros(1, dtype=torch.float64, device="cuda")
    ds, da, dr, ds2, dt = dev(s), dev(a), dev(r), dev(s2), dev(t)
    m.ctx.call("nfsp_br_targets", nat.ptr(m.w), 64, nat.ptr(ds), nat.ptr(da), nat.ptr(dr),
               nat.ptr(ds2), nat.ptr(dt), n, nat.F64(0.95), quirks, nat.ptr(out), nat.ptr(ex))
    ag = orc.Agent.__new__(orc.Agent)
    ag.target_br_model, ag.gamma, ag.quirks = o, 0.95, quirks == 3
    tb = t.astype(bool)          # np.bool_ entries: `t is True` never holds (quirk)
    tgt, expl = ag.br_targets(s.reshape(n, 1, 30), a.reshape(n, 1, 3), r.astype(np.float64),
                              s2.reshape(n, 1, 30), tb)
    assert np.abs(out.cpu().numpy() - tgt.reshape(n, 3)).max() <= 1e-6
    assert abs(ex.item() - expl) <= 1e-6
