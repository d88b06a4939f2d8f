"""C4's exchange on CPU (gloo, world size 2): shards.AvgPolicyAllReduce broadcasts rank 0's AR
nets, then, after each engine step's local SGD, all-reduces the accumulated gradient steps
so that every rank holds W0 + mean_r(W_r - W0).  The engine is replaced by rank-dependent
"SGD steps" on CPU tensors shaped like the two agents' packed AR nets (2 x 2,179 f32)."""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NP = 30 * 64 + 64 + 64 * 3 + 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _local_sgd(w, rank, step):
    """A rank's learner: a few SGD-like steps W -= lr * g with rank/step-dependent g."""
    g = np.random.RandomState(100 * rank + step)
    for _ in range(3):
        w -= 0.1 * g.standard_normal(w.shape).astype(np.float32)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, REPO)
    import torch
    import bench
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    _, r, _, dist = bench.init_dist(backend="gloo")
    rs = np.random.RandomState(7 + r)                    # different initial nets per rank
    nets = [torch.from_numpy(rs.uniform(-1, 1, NP).astype(np.float32)) for _ in range(2)]
    avg = pkg.shards.AvgPolicyAllReduce(nets, dist)
    w0 = [n.numpy().copy() for n in nets]                # after the broadcast
    trace = [w0]
    for step in range(3):
        before = [n.numpy().copy() for n in nets]
        for a, n in enumerate(nets):
            _local_sgd(n.numpy(), r, 10 * step + a)
        deltas = [n.numpy() - b for n, b in zip(nets, before)]
        avg()
        trace.append(([n.numpy().copy() for n in nets], before, deltas))
    q.put((r, trace, avg.calls))
    dist.destroy_process_group()


def test_two_shard_ar_allreduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (t, c)) for r, t, c in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (t0, c0), (t1, c1) = res[0], res[1]
    assert c0 == c1 == 3
    rs0 = np.random.RandomState(7)                       # rank 0's initial nets everywhere
    for a in range(2):
        expect = rs0.uniform(-1, 1, NP).astype(np.float32)
        assert np.array_equal(t0[0][a], expect) and np.array_equal(t1[0][a], expect)
    for k in range(1, 4):
        (n0, b0, d0), (n1, b1, d1) = t0[k], t1[k]
        for a in range(2):
            assert np.array_equal(b0[a], b1[a])          # common W0 before each exchange
            assert not np.array_equal(d0[a], d1[a])      # ... different local steps
            assert np.array_equal(n0[a], n1[a])          # identical nets after it
            np.testing.assert_allclose(n0[a], b0[a] + 0.5 * (d0[a] + d1[a]), rtol=0, atol=2e-6)
