"""C4's AR-gradient all-reduce on real engines (shards.AvgPolicyAllReduce over the device
weight views): two shards co-resident on one GPU, gloo between them (the one-GPU box has
no second device for RCCL).  After each engine step every shard holds W0 + mean_r(W_r - W0)
for both agents' AR nets; the BR nets stay per shard.  Two sizes: 4,096 lanes, and C4's own
shard (bench.py's C3 line per rank: 1,048,576 lanes in 16 pipelined slices, M_RL 200k,
M_SL 2M)."""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


SIZES = {"4k": dict(n_lanes=4096, rl_capacity=40_000, sl_capacity=40_000),
         "c4": dict(n_lanes=1_048_576, slices=16, slice_lag=2, rl_capacity=200_000,
                    sl_capacity=2_000_000)}


def _worker(rank, world, port, q, size):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        sys.path.insert(0, REPO)
        import torch
        torch.cuda.set_device(0)
        import bench
        import __graft_entry__
        pkg = __graft_entry__.load_package()
        _, r, _, dist = bench.init_dist(backend="gloo")
        eng = pkg.engine.SelfPlayEngine(seed=1234 + r, init_seed=r, **SIZES[size])
        AR, BR = pkg.engine.NET_AR, pkg.engine.NET_BR
        avg = pkg.shards.AvgPolicyAllReduce([eng.weights_tensor(a, AR) for a in (0, 1)], dist,
                                            sync=torch.cuda.synchronize)
        trace = {"w0": [eng.get_weights(a, AR) for a in (0, 1)], "steps": []}
        for _ in range(3):
            base = [eng.get_weights(a, AR) for a in (0, 1)]
            eng.step()
            torch.cuda.synchronize()
            local = [eng.get_weights(a, AR) for a in (0, 1)]
            avg()
            after = [eng.get_weights(a, AR) for a in (0, 1)]
            trace["steps"].append((base, local, after))
        trace["br"] = [eng.get_weights(a, BR) for a in (0, 1)]
        trace["ar_updates"] = eng.stats()["ar_updates"]
        q.put((r, trace))
        dist.destroy_process_group()
        eng.close()
    except Exception as ex:                      # surface the failure in the parent
        q.put((rank, repr(ex)))
        raise


@pytest.mark.gpu
@pytest.mark.parametrize("size", ["4k", "c4"])
def test_two_shards_share_the_average_policy(size):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, size)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert isinstance(res[r], dict), res[r]
    assert all(p.exitcode == 0 for p in procs)
    t0, t1 = res[0], res[1]
    for a in (0, 1):
        assert np.array_equal(t0["w0"][a], t1["w0"][a])          # rank 0's AR nets broadcast
        assert min(t0["ar_updates"][a], t1["ar_updates"][a]) > 0
        assert not np.array_equal(t0["br"][a], t1["br"][a])      # BR nets: per shard
    for (b0, l0, n0), (b1, l1, n1) in zip(t0["steps"], t1["steps"]):
        for a in (0, 1):
            assert np.array_equal(b0[a], b1[a])                  # common W0 before the step
            assert not np.array_equal(l0[a], l1[a])              # different local learning
            assert np.array_equal(n0[a], n1[a])                  # one AR net after the exchange
            expect = b0[a] + 0.5 * ((l0[a] - b0[a]) + (l1[a] - b1[a]))
            np.testing.assert_allclose(n0[a], expect, rtol=0, atol=1e-6)
