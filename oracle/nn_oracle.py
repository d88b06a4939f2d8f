"""TEST INFRASTRUCTURE ONLY -- numpy fp32 restatement of the Keras semantics the
reference's networks rely on.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module; the product path
(the HIP library) never does.

Parity status: **unpinned against real Keras/TF** (neither is installed and the
reference ships no NN test vectors).  This file *is* the NN
oracle: the HIP kernels are checked against it within ``NN_ATOL``.

Reference call sites restated here (``/root/reference``):

* ``agent/agent.py:90-107``  BR / target-BR net: Dense(64, relu) -> Dense(3, relu),
  loss = the ``huber_loss`` closure (py2: ``1/2 == 0``; the gradient is the plain
  Huber gradient either way), optimizer SGD(lr=LearningRateBR).
* ``agent/agent.py:109-116`` AR net: Dense(64, relu) -> Dense(3, softmax),
  loss = ``categorical_crossentropy`` (Keras/TF: output normalised by its sum,
  clipped to [1e-7, 1-1e-7], ``-sum(t*log(p))``), optimizer SGD(lr=LearningRateAR).
* ``model.predict`` / ``model.fit(x, y, epochs=2)`` call sites at
  ``agent/agent.py:126,143,219,230,243,261``: Keras 2.x ``fit`` defaults are
  batch_size=32 and shuffle=True, one ``np.random.shuffle(arange(n))`` per epoch,
  plain SGD ``w <- w - lr*g`` (no momentum, no decay).
* Keras default initialisers: glorot_uniform kernels (limit sqrt(6/(fan_in+fan_out))),
  zero biases.  TF's own RNG cannot be reproduced; weights are drawn from a
  caller-provided ``numpy.random.RandomState`` and parity is defined given equal
  weights.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
NN_ATOL = 1e-5            # |delta| bound on forward outputs
CE_EPS = F32(1e-7)        # keras.backend.epsilon()
N_IN, N_OUT = 30, 3

ACT_RELU = 0              # BR / target-BR output activation (agent/agent.py:103)
ACT_SOFTMAX = 1           # AR output activation (agent/agent.py:112)
ACT_LINEAR = 2            # BR head under the engine's NFSP_EXT_LINEAR_Q (not the reference)
ACT_LINEAR_MSE = 3        # ... with NFSP_EXT_MSE_Q: the same head, Keras mean_squared_error


def glorot_uniform(rng: np.random.RandomState, fan_in: int, fan_out: int) -> np.ndarray:
    """Keras ``glorot_uniform`` kernel, drawn from ``rng`` in float64 then cast."""
    limit = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-limit, limit, size=(fan_in, fan_out)).astype(F32)


def dense_seq(x2d: np.ndarray, W: np.ndarray, b: np.ndarray) -> np.ndarray:
    """``x @ W + b`` in float32 with a FIXED summation order: acc starts at +0,
    adds ``x[:, i] * W[i]`` for i = 0, 1, ... (separate multiply and add roundings),
    then adds the bias.  The order makes a row's result independent of the batch
    it is predicted in, and is the order the HIP forward kernels use (no FMA
    contraction), so forwards agree bit for bit."""
    x2d = np.asarray(x2d, dtype=F32)
    acc = np.zeros((x2d.shape[0], W.shape[1]), F32)
    for i in range(W.shape[0]):
        acc = acc + x2d[:, i:i + 1] * W[i]
    return (acc + b).astype(F32)


def softmax3(z: np.ndarray) -> np.ndarray:
    """Keras softmax on the last axis: exp(z - max) / ((e0 + e1) + e2)."""
    z = np.asarray(z, dtype=F32)
    e = np.exp(z - z.max(axis=-1, keepdims=True)).astype(F32)
    s = (e[..., 0:1] + e[..., 1:2]) + e[..., 2:3]
    return (e / s).astype(F32)


class MLP:
    """30 -> H (relu) -> 3 (relu | softmax), Keras weight order [W1, b1, W2, b2]."""

    def __init__(self, act: int, n_hidden: int = 64, rng: np.random.RandomState | None = None,
                 weights=None):
        self.act = act
        self.n_hidden = n_hidden
        if weights is not None:
            self.set_weights(weights)
        else:
            rng = rng if rng is not None else np.random.RandomState(0)
            self.W1 = glorot_uniform(rng, N_IN, n_hidden)
            self.b1 = np.zeros(n_hidden, F32)
            self.W2 = glorot_uniform(rng, n_hidden, N_OUT)
            self.b2 = np.zeros(N_OUT, F32)

    # -- Keras Model API -------------------------------------------------
    def get_weights(self):
        return [self.W1.copy(), self.b1.copy(), self.W2.copy(), self.b2.copy()]

    def set_weights(self, ws):
        self.W1, self.b1, self.W2, self.b2 = (np.array(w, dtype=F32, copy=True) for w in ws)

    def flat(self) -> np.ndarray:
        """Packed layout used by the device: W1[30,H] | b1[H] | W2[H,3] | b2[3]."""
        return np.concatenate([self.W1.ravel(), self.b1, self.W2.ravel(), self.b2]).astype(F32)

    def _forward(self, x2d: np.ndarray):
        z1 = dense_seq(x2d, self.W1, self.b1)
        h = np.maximum(z1, F32(0))
        z2 = dense_seq(h, self.W2, self.b2)
        if self.act == ACT_RELU:
            y = np.maximum(z2, F32(0))
        elif self.act in (ACT_LINEAR, ACT_LINEAR_MSE):
            y = z2
        else:
            y = softmax3(z2)
        return z1, h, z2, y.astype(F32)

    def predict(self, x) -> np.ndarray:
        """``model.predict`` on ``[B, 1, 30]`` (or any ``[..., 30]``) -> same leading shape x 3."""
        x = np.asarray(x, dtype=F32)
        lead = x.shape[:-1]
        y = self._forward(x.reshape(-1, N_IN))[3]
        return y.reshape(lead + (N_OUT,))

    # -- training --------------------------------------------------------
    def grads(self, x2d: np.ndarray, t2d: np.ndarray):
        """Gradients of the Keras loss of this head on one minibatch."""
        m = x2d.shape[0]
        z1, h, z2, y = self._forward(x2d)
        if self.act in (ACT_RELU, ACT_LINEAR):
            # Huber (agent/agent.py:91-99); mean over the 3 outputs, then over the batch.
            e = t2d - y
            dldy = np.where(np.abs(e) > F32(1.0), np.sign(e), e).astype(F32)
            dldy = -dldy / F32(3 * m)
            dz2 = dldy * (z2 > 0).astype(F32) if self.act == ACT_RELU else dldy
        elif self.act == ACT_LINEAR_MSE:
            # mean_squared_error: mean over the 3 outputs of e^2, then over the batch
            e = t2d - y
            dz2 = (-(e * F32(2.0)) / F32(3 * m)).astype(F32)
        else:
            # categorical_crossentropy, TF backend, from_logits=False.
            S = y.sum(axis=-1, keepdims=True)
            p = y / S
            if getattr(self, "clip_probe", None) is not None:   # tests: where the clip mask sits
                self.clip_probe(p)
            pc = np.clip(p, CE_EPS, F32(1.0) - CE_EPS)
            mask = ((p >= CE_EPS) & (p <= F32(1.0) - CE_EPS)).astype(F32)
            dldp = (-t2d / pc) * mask / F32(m)
            dldy = dldp / S - (dldp * y).sum(axis=-1, keepdims=True) / (S * S)
            dz2 = y * (dldy - (dldy * y).sum(axis=-1, keepdims=True))
        dz2 = dz2.astype(F32)
        gW2 = h.T @ dz2
        gb2 = dz2.sum(axis=0)
        dh = dz2 @ self.W2.T
        if getattr(self, "relu_probe", None) is not None:    # tests: how close a ReLU is to its kink
            self.relu_probe(z1)
        dz1 = dh * (z1 > 0).astype(F32)
        gW1 = x2d.T @ dz1
        gb1 = dz1.sum(axis=0)
        return gW1.astype(F32), gb1.astype(F32), gW2.astype(F32), gb2.astype(F32)

    def loss(self, x2d: np.ndarray, t2d: np.ndarray) -> float:
        """The Keras loss value of one minibatch (what the TensorBoard callbacks log,
        agent/agent.py:84-88,243,264): BR huber_loss as the reference runs it under py2
        (agent/agent.py:91-99: ``1 / 2 == 0``, so the linear term is |e|), mean over the 3
        outputs then the batch; AR categorical cross-entropy on the normalised, clipped
        softmax, mean over the batch."""
        y = self._forward(x2d)[3].astype(np.float64)
        t = t2d.astype(np.float64)
        if self.act in (ACT_RELU, ACT_LINEAR):
            e = t - y
            v = np.where(np.abs(e) > 1.0, np.abs(e), 0.5 * e * e)
            return float(v.mean(axis=-1).mean())
        if self.act == ACT_LINEAR_MSE:
            return float(((t - y) ** 2).mean(axis=-1).mean())
        p = y / y.sum(axis=-1, keepdims=True)
        pc = np.clip(p, float(CE_EPS), 1.0 - float(CE_EPS))
        return float((-(t * np.log(pc)).sum(axis=-1)).mean())

    def sgd_step(self, x2d, t2d, lr):
        gW1, gb1, gW2, gb2 = self.grads(x2d, t2d)
        lr = F32(lr)
        self.W1 = (self.W1 - lr * gW1).astype(F32)
        self.b1 = (self.b1 - lr * gb1).astype(F32)
        self.W2 = (self.W2 - lr * gW2).astype(F32)
        self.b2 = (self.b2 - lr * gb2).astype(F32)

    def fit(self, x, t, lr, epochs: int = 2, batch_size: int = 32, shuffle_rng=None, perms=None,
            epoch_losses=None):
        """Keras 2.x ``fit_loop``: per epoch ``np.random.shuffle(index_array)``, then
        consecutive slices of ``batch_size``, one SGD step each.

        ``perms`` (``[epochs, n]`` int) overrides the shuffle draws; otherwise they are
        taken from ``shuffle_rng`` (default: the global ``np.random``) and returned so
        a device run can replay the identical order.
        """
        x2d = np.asarray(x, dtype=F32).reshape(-1, N_IN)
        t2d = np.asarray(t, dtype=F32).reshape(-1, N_OUT)
        n = x2d.shape[0]
        used = []
        for ep in range(epochs):
            if perms is not None:
                idx = np.asarray(perms[ep])
            else:
                idx = np.arange(n)
                (shuffle_rng if shuffle_rng is not None else np.random).shuffle(idx)
            used.append(idx.copy())
            ls = []
            for b0 in range(0, n, batch_size):
                sel = idx[b0:b0 + batch_size]
                if epoch_losses is not None:          # Keras: batch loss before its update
                    ls.append(self.loss(x2d[sel], t2d[sel]))
                self.sgd_step(x2d[sel], t2d[sel], lr)
            if epoch_losses is not None:
                epoch_losses.append(float(np.mean(ls)))
        return np.stack(used)


def pack_weights(ws) -> np.ndarray:
    W1, b1, W2, b2 = ws
    return np.concatenate([np.ravel(W1), b1, np.ravel(W2), b2]).astype(F32)


def unpack_weights(flat: np.ndarray, n_hidden: int = 64):
    flat = np.asarray(flat, dtype=F32)
    o = 0
    W1 = flat[o:o + N_IN * n_hidden].reshape(N_IN, n_hidden); o += N_IN * n_hidden
    b1 = flat[o:o + n_hidden]; o += n_hidden
    W2 = flat[o:o + n_hidden * N_OUT].reshape(n_hidden, N_OUT); o += n_hidden * N_OUT
    b2 = flat[o:o + N_OUT]
    return [W1.copy(), b1.copy(), W2.copy(), b2.copy()]


def n_params(n_hidden: int = 64) -> int:
    return N_IN * n_hidden + n_hidden + n_hidden * N_OUT + N_OUT
