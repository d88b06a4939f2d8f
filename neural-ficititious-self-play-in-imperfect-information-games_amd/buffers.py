"""Drop-ins for the reference memories, with the records living in HBM.

* ``ReplayBuffer``    -- M_RL, utils/replay_buffer.py:18-59 (FIFO, ``random.sample``)
* ``ReservoirBuffer`` -- M_SL, utils/ReservoirBuffer.py:6-43 (append until full, then
  ``j = randrange(1, N+1)`` replaces slot ``j`` iff ``j < N``; slot 0 is never replaced)

Both constructors re-seed the global ``random`` like the reference
(utils/replay_buffer.py:27, utils/ReservoirBuffer.py:15) and draw every slot / sample
index from it in the same order, so a drop-in run consumes the reference's RNG stream
call for call.  The row copies themselves are ``nfsp_buf_insert`` / ``nfsp_buf_sample``.

View aliasing (``NFSP_QUIRK_ALIAS_RL``): the reference deque stores the views it is
handed, so an RL tuple's ``s``/``a`` keep changing until the env replaces its arrays at
the next reset.  ``ReplayBuffer`` reproduces that: records whose ``s`` is a view of a
live array stay *pending* on the host (sampled with their current values) and are
written to HBM once a record backed by a different array arrives.
"""
from __future__ import annotations

import random

import numpy as np
import torch

from . import native
from . import pyrandom

OBS = 30


def _base_ptr(x):
    b = x
    while isinstance(b, np.ndarray) and b.base is not None and isinstance(b.base, np.ndarray):
        b = b.base
    return b.__array_interface__["data"][0] if isinstance(b, np.ndarray) else id(b)


class _Table:
    """Device record columns + an nfsp_records descriptor."""

    def __init__(self, cap, rl, dev):
        self.cap = int(cap)
        self.s = torch.zeros((self.cap, OBS), dtype=torch.float32, device=dev)
        self.a = torch.zeros((self.cap, 3), dtype=torch.float32, device=dev)
        self.r = torch.zeros(self.cap, dtype=torch.float32, device=dev) if rl else None
        self.s2 = torch.zeros((self.cap, OBS), dtype=torch.float32, device=dev) if rl else None
        self.t = torch.zeros(self.cap, dtype=torch.uint8, device=dev) if rl else None
        self.rec = native.Records(native.ptr(self.s), native.ptr(self.a), native.ptr(self.r),
                                  native.ptr(self.s2), native.ptr(self.t), self.cap)


class _DeviceMemory:
    rl = True

    def __init__(self, buffer_size, random_seed=123, ctx=None):
        self.buffer_size = int(buffer_size)
        self.count = 0
        random.seed(random_seed)
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.ctx = ctx if ctx is not None else native.Context(1)
        self.table = _Table(self.buffer_size, self.rl, self.dev)
        self._stage = None

    def _staging(self, n):
        if self._stage is None or self._stage.cap < n:
            self._stage = _Table(max(n, 8), self.rl, self.dev)
        return self._stage

    def _write(self, slots, s, a, r=None, s2=None, t=None):
        """Copy host rows into table slots (one H2D per column + one insert kernel)."""
        n = len(slots)
        st = self._staging(n)
        st.s[:n].copy_(torch.as_tensor(np.asarray(s, np.float32).reshape(n, OBS)))
        st.a[:n].copy_(torch.as_tensor(np.asarray(a, np.float32).reshape(n, 3)))
        if self.rl:
            st.r[:n].copy_(torch.as_tensor(np.asarray(r, np.float32).reshape(n)))
            st.s2[:n].copy_(torch.as_tensor(np.asarray(s2, np.float32).reshape(n, OBS)))
            st.t[:n].copy_(torch.as_tensor(np.asarray(t, np.uint8).reshape(n)))
        sl = torch.as_tensor(np.asarray(slots, np.int64), device=self.dev)
        self.ctx.call("nfsp_buf_insert", native.C.byref(self.table.rec), native.C.byref(st.rec),
                      native.ptr(sl), n)

    def _gather(self, idx):
        k = len(idx)
        out = _Table(k, self.rl, self.dev)
        if k:
            it = torch.as_tensor(np.asarray(idx, np.int64), device=self.dev)
            self.ctx.call("nfsp_buf_sample", native.C.byref(self.table.rec), native.ptr(it), k,
                          native.C.byref(out.rec))
        return out

    def size(self):
        return self.count


class ReplayBuffer(_DeviceMemory):
    """M_RL with the reference's FIFO + sampling semantics."""
    rl = True

    def __init__(self, buffer_size, random_seed=123, ctx=None, alias=True):
        super().__init__(buffer_size, random_seed, ctx)
        self.alias = alias
        self.total = 0          # tuples ever added (logical)
        self.flushed = 0        # tuples written to HBM (tuple k lives at slot k % cap)
        self.pending = []       # (s_view, a_view, r, s2, t, base) not yet written
        self._pending_base = None

    def _flush(self):
        if not self.pending:
            return
        n = len(self.pending)
        slots = [(self.flushed + i) % self.buffer_size for i in range(n)]
        self._write(slots, [np.asarray(p[0]) for p in self.pending],
                    [np.asarray(p[1]) for p in self.pending], [p[2] for p in self.pending],
                    [p[3] for p in self.pending], [p[4] for p in self.pending])
        self.flushed += n
        self.pending = []
        self._pending_base = None

    def add(self, s, a, r, s2, t):
        s = np.reshape(s, (1, OBS))
        a = np.reshape(a, (1, 3))
        s2 = None if s2 is None else np.array(np.reshape(s2, (1, OBS)))
        base = _base_ptr(s)
        if not self.alias or (self.pending and base != self._pending_base):
            self._flush()
        self.pending.append((s, a, float(r), s2, bool(t)))
        self._pending_base = base
        self.total += 1
        if self.count < self.buffer_size:
            self.count += 1
        if not self.alias or len(self.pending) >= self.buffer_size:
            self._flush()

    def _logical_rows(self, logical):
        """Map deque positions to (device slots, pending entries)."""
        first = self.total - self.count
        dev_pos, dev_slot, pen_pos, pen = [], [], [], []
        for i, l in enumerate(logical):
            k = first + l
            if k < self.flushed:
                dev_pos.append(i)
                dev_slot.append(k % self.buffer_size)
            else:
                pen_pos.append(i)
                pen.append(self.pending[k - self.flushed])
        return dev_pos, dev_slot, pen_pos, pen

    def sample_device(self, batch_size):
        """``sample_batch`` returning the batch as device tensors (s [k,30], a [k,3],
        r [k], s2 [k,30], t [k])."""
        k = min(self.count, batch_size)
        logical = pyrandom.sample(range(self.count), k)
        dev_pos, dev_slot, pen_pos, pen = self._logical_rows(logical)
        out = _Table(k, True, self.dev)
        if dev_slot:
            g = self._gather(dev_slot)
            pos = torch.as_tensor(dev_pos, device=self.dev)
            out.s[pos] = g.s
            out.a[pos] = g.a
            out.r[pos] = g.r
            out.s2[pos] = g.s2
            out.t[pos] = g.t
        if pen:
            pos = torch.as_tensor(pen_pos, device=self.dev)
            out.s[pos] = torch.as_tensor(np.array([np.asarray(p[0]).reshape(OBS) for p in pen],
                                                  np.float32), device=self.dev)
            out.a[pos] = torch.as_tensor(np.array([np.asarray(p[1]).reshape(3) for p in pen],
                                                  np.float32), device=self.dev)
            out.r[pos] = torch.as_tensor([p[2] for p in pen], dtype=torch.float32,
                                         device=self.dev)
            out.s2[pos] = torch.as_tensor(np.array([np.asarray(p[3]).reshape(OBS) for p in pen],
                                                   np.float32), device=self.dev)
            out.t[pos] = torch.as_tensor([p[4] for p in pen], dtype=torch.uint8, device=self.dev)
        return out

    def sample_batch(self, batch_size):
        """Reference return shapes: s [k,1,30], a [k,1,3], r [k], s2 [k,1,30], t [k] bool."""
        o = self.sample_device(batch_size)
        k = o.cap
        return (o.s.cpu().numpy().astype(np.float64).reshape(k, 1, OBS),
                o.a.cpu().numpy().astype(np.float64).reshape(k, 1, 3),
                o.r.cpu().numpy().astype(np.float64),
                o.s2.cpu().numpy().astype(np.float64).reshape(k, 1, OBS),
                o.t.cpu().numpy().astype(bool))


class ReservoirBuffer(_DeviceMemory):
    """M_SL with the reference's replacement rule (j in [1, N], replace iff j < N)."""
    rl = False

    def add(self, s, a):
        if self.count < self.buffer_size:
            slot = self.count
            self.count += 1
        else:
            j = pyrandom.randrange(1, self.buffer_size + 1)
            if j >= self.buffer_size:
                return
            slot = j
        self._write([slot], np.reshape(s, (1, OBS)), np.reshape(a, (1, 3)))

    def sample_device(self, batch_size):
        k = min(self.count, batch_size)
        return self._gather(pyrandom.sample(range(self.count), k))

    def sample_batch(self, batch_size):
        o = self.sample_device(batch_size)
        k = o.cap
        return (o.s.cpu().numpy().astype(np.float64).reshape(k, 1, OBS),
                o.a.cpu().numpy().astype(np.float64).reshape(k, 1, 3))
