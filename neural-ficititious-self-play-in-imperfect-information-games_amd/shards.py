"""Multi-GPU self-play shards (BASELINE.json configs[3] = C4).

One process per GPU, each with its own ``SelfPlayEngine`` (its own hands, memories and
learner; seeds 1234 + rank).  Hands never cross GPUs.  The one exchange is the all-reduce of
the average-policy (AR) gradient steps of both agents.

``AvgPolicyExchange`` (what bench.py runs at N > 1) does it inside the engine, after every
lane slice's learner (nfsp_engine_set_exchange): the reference learns inside its hand loop
(main.py:27-67, an update every 128 RL inserts, agent/agent.py:153-154), so the shards' AR
copies are merged every 65,536 hands per rank rather than once per 1M-hand step.  On RCCL the
collective is enqueued by libnfsp itself on the AR chain stream (ncclAllReduce on a
communicator of its own), behind the slice's AR chain and before the snapshot the rollout two
slices on acts with -- no host round trip.  Over gloo (CPU rehearsals, co-resident tests) a
host callback sums the deltas through the process group instead, with the same arithmetic.

``AvgPolicyAllReduce`` is the per-step exchange of round 3 from the host, between steps:

* ``AvgPolicyAllReduce(tensors, dist)`` first broadcasts rank 0's AR nets, so every shard's
  AR nets start equal;
* ``__call__()``, once per engine step: every rank holds the AR weights W_r its learner
  reached from the common W0 by its own SGD steps (agent/agent.py:255-264 at the reference
  cadence).  The accumulated gradient steps D_r = W_r - W0 (= -sum of lr * grad) are
  all-reduced (SUM, 2 x 2,179 f32 = 17.4 KB in one call), and every rank sets
  W = W0 + sum(D_r) / world.  With plain SGD (no momentum, agent/agent.py:116) that is the
  data-parallel update of one AR net over all shards' minibatches, exchanged once per
  engine step instead of once per SGD step (local SGD).  The BR nets stay per shard (the
  SURVEY §8(e) default).

Why once per engine step, not once per SGD step: the SGD chain takes ~1 us per step and an
xGMI all-reduce >= 10 us, over ~190k sequential steps per engine step.

The tensors are torch views of device memory (``SelfPlayEngine.weights_tensor``) or, in
the CPU tests, plain CPU tensors; ``sync`` orders the engine's streams before and after
the collective (``torch.cuda.synchronize`` on a GPU).
"""
from __future__ import annotations

import ctypes as C
import sys
import traceback
from typing import Callable, Sequence

import torch


def ar_nets_digest(engine) -> str:
    """sha256 of both agents' AR nets as they are now (synchronises the device): equal on
    every rank after an exchange that worked (bench.py checks it over the ranks)."""
    import hashlib
    from .engine import NET_AR
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for a in (0, 1):
        h.update(engine.get_weights(a, NET_AR).tobytes())
    return h.hexdigest()


class AvgPolicyAllReduce:
    def __init__(self, tensors: Sequence[torch.Tensor], dist, src: int = 0,
                 sync: Callable[[], None] = lambda: None):
        if not tensors:
            raise ValueError("AvgPolicyAllReduce: no tensors")
        dev = tensors[0].device
        if any(t.device != dev or t.dtype != torch.float32 or not t.is_contiguous() for t in tensors):
            raise ValueError("AvgPolicyAllReduce: contiguous f32 tensors on one device expected")
        self.tensors = list(tensors)
        self.dist = dist
        self.world = dist.get_world_size()
        self.sync = sync
        self.sizes = [t.numel() for t in self.tensors]
        self.calls = 0
        sync()
        self.flat = torch.cat([t.reshape(-1) for t in self.tensors])   # staging: one collective
        # RCCL works on the device buffer; gloo (CPU rehearsals) on a host copy
        self.host = dist.get_backend() == "gloo" and self.flat.is_cuda
        self._collective(lambda x: dist.broadcast(x, src=src))
        self._scatter(self.flat)
        self.base = self.flat.clone()                                   # W0 of the next exchange
        sync()

    def _collective(self, op):
        if self.host:
            x = self.flat.cpu()
            op(x)
            self.flat.copy_(x)
        else:
            op(self.flat)

    def _scatter(self, flat):
        off = 0
        for t, n in zip(self.tensors, self.sizes):
            t.view(-1).copy_(flat[off:off + n])
            off += n

    def __call__(self):
        """All-reduce the AR gradient steps taken since the last call; every rank ends with
        the same AR nets W0 + mean_r(W_r - W0)."""
        self.sync()                                  # the learner's writes to W_r are done
        torch.cat([t.reshape(-1) for t in self.tensors], out=self.flat)
        self.flat.sub_(self.base)                    # D_r
        self._collective(self.dist.all_reduce)       # sum_r D_r (identical on every rank)
        self.base.add_(self.flat, alpha=1.0 / self.world)
        self._scatter(self.base)
        self.sync()                                  # the next rollout reads the new nets
        self.calls += 1


class AvgPolicyExchange:
    """The AR exchange inside the engine, every ``every`` learner calls (slices): W0 + gain x
    the mean over ranks of (W_r - W0) after each slice's AR chain (include/nfsp.h
    nfsp_engine_set_exchange, scale = gain / world).  gain 1 is plain model averaging
    (data-parallel SGD of one net over every shard's minibatches, exchanged per slice); gain g
    is a server step g x the mean of the shards' steps.  ``transport``: "rccl"
    (libnfsp's own communicator, the collective on the AR chain stream), "host" (the process
    group's all-reduce from a host callback: gloo), or "auto" (rccl under the nccl backend,
    host otherwise)."""

    def __init__(self, engine, dist, every: int = 1, transport: str = "auto", gain: float = 1.0,
                 src: int = 0):
        from . import native
        from .engine import NET_AR, _wrap_device
        self.engine, self.dist, self.every, self.gain = engine, dist, int(every), float(gain)
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        backend = dist.get_backend()
        self.transport = ("rccl" if backend == "nccl" else "host") if transport == "auto" else transport
        self._wrap, self._dev = _wrap_device, engine.dev
        # the common start: rank 0's AR nets everywhere (one broadcast)
        torch.cuda.synchronize()
        views = [engine.weights_tensor(a, NET_AR) for a in (0, 1)]
        flat = torch.cat([v.reshape(-1) for v in views])
        if backend == "gloo":
            x = flat.cpu()
            dist.broadcast(x, src=src)
            flat.copy_(x)
        else:
            dist.broadcast(flat, src=src)
        off = 0
        for v in views:
            v.copy_(flat[off:off + v.numel()])
            off += v.numel()
        torch.cuda.synchronize()
        self.bytes_per_call = 4 * flat.numel()
        self.comm = None
        self._fn = None
        L = engine.L
        self.fallback = None
        if self.transport == "rccl":
            # 1. every rank loads RCCL and selects its device (nfsp_rccl_ready) and the ranks
            #    agree on the result (MIN) BEFORE anyone calls ncclCommInitRank, which blocks
            #    until all ranks joined: a rank that cannot use RCCL never strands the others;
            # 2. rank 0's id to every rank; 3. the communicator, its success agreed the same way.
            # Unless every step worked on every rank, all ranks take the host transport
            # together and `fallback` says why (bench.py refuses that under RCCL at N > 1
            # unless --allow-host-fallback).
            dev = "cuda" if backend == "nccl" else "cpu"
            why = ""
            ready = int(L.nfsp_rccl_ready(torch.cuda.current_device()) == native.OK)
            uid = (C.c_uint8 * 128)()
            if ready and self.rank == src:
                ready = int(L.nfsp_rccl_unique_id(uid) == native.OK)
            if not ready:
                why = L.nfsp_last_error().decode()
            flag = torch.tensor([ready], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            rc = native.EINVAL
            comm = native.P()
            if int(flag.item()) == 1:
                t = torch.tensor(list(uid), dtype=torch.uint8, device=dev)
                dist.broadcast(t, src=src)
                uid = (C.c_uint8 * 128)(*t.cpu().tolist())
                rc = L.nfsp_rccl_comm_create(uid, self.world, self.rank, torch.cuda.current_device(), C.byref(comm))
                if rc != native.OK:
                    why = L.nfsp_last_error().decode()
            elif ready:
                why = "another rank could not load RCCL or select its device"
            good = torch.tensor([1 if rc == native.OK else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(good, op=dist.ReduceOp.MIN)
            if int(good.item()) == 1:
                self.comm = comm
                engine.set_exchange(self.every, self.gain / self.world, comm=comm)
            else:
                if rc == native.OK:
                    L.nfsp_rccl_comm_destroy(comm)
                self.fallback = "rccl setup failed on some rank: " + (why or "another rank failed")
                print(f"AvgPolicyExchange: {self.fallback}; using the host transport", file=sys.stderr)
                self.transport = "host"
        if self.transport == "host":
            self._fn = native.EXCHANGE_FN(self._host_sum)
            engine.set_exchange(self.every, self.gain / self.world, fn=self._fn)
        elif self.transport != "rccl":
            raise ValueError(f"unknown transport {transport!r}")

    def _host_sum(self, _user, ptr, n):
        """nfsp_exchange_fn: the engine synchronised its AR stream; leave the sum over ranks
        of the [2][NP] deltas at ptr (device), complete on return."""
        try:
            t = self._wrap(ptr, n, torch.float32, self._dev)
            if self.dist.get_backend() == "gloo":
                x = t.cpu()
                self.dist.all_reduce(x)
                t.copy_(x)
            else:
                self.dist.all_reduce(t)
            torch.cuda.synchronize()
            return 0
        except BaseException:           # never unwind through the C caller
            traceback.print_exc(file=sys.stderr)
            return 1

    @property
    def calls(self) -> int:
        return self.engine.exchanges()

    def close(self):
        if self.engine.h is not None:
            self.engine.set_exchange(0, 1.0)
        if self.comm is not None:
            self.engine.L.nfsp_rccl_comm_destroy(self.comm)
            self.comm = None
