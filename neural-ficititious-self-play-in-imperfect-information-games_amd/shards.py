"""Multi-GPU self-play shards (BASELINE.json configs[3] = C4).

One process per GPU, each with its own ``SelfPlayEngine`` (its own hands, memories and
learner; seeds 1234 + rank).  Hands never cross GPUs.  The one exchange is the optional
all-reduce of the average-policy (AR) gradients of both agents over RCCL:

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

from typing import Callable, Sequence

import torch


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
