"""C4's per-slice exchange of the average-policy nets (include/nfsp.h nfsp_engine_set_exchange,
shards.AvgPolicyExchange): the rank path bench.py --gpus N runs equals the engine group that
emulates C4 on one GPU (nfsp_group_set_exchange, slice_lag 2).

* Two co-resident ranks (one GPU, gloo between them, the host transport): pipelined engines
  (slice_lag 2) exchanging after every slice's AR chain end every step with the same nets,
  counters and schedules as a 2-replica group stepping the same slices with the on-device
  exchange -- bit for bit (the bar the verdict set is 1e-6).
* The RCCL transport (libnfsp's own communicator, ncclAllReduce on the AR chain stream) at world
  size 1, the only size a one-GPU box runs: bit-identical to the host transport and to a
  1-replica group with the same exchange.
The reference trains one average-policy net per agent inside its hand loop (main.py:27-67,
agent/agent.py:153-154, 255-264); the exchange keeps the shards' copies one net."""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

# 8 slices of 8,192 lanes: the slice size of C4's shard (1,048,576 lanes in 128 slices, bench.CONFIGS["c4"])
CFG = dict(n_lanes=65_536, slices=8, slice_lag=2, rl_capacity=40_000, sl_capacity=60_000, target_every=40)
SEED, INIT = 777, 5
STEPS = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _state(pkg, eng):
    import torch
    torch.cuda.synchronize()
    w = {(a, n): eng.get_weights(a, n) for a in (0, 1) for n in (0, 1, 2)}
    st = eng.stats()
    return w, {k: st[k] for k in ("hands", "rollouts", "rl_total", "sl_total", "br_updates", "ar_updates",
                                  "iteration", "target_syncs", "actions", "epsilon")}


def _rank(rank, world, port, q, backend, transport, gain):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        sys.path.insert(0, REPO)
        import torch
        torch.cuda.set_device(0)
        import datetime
        import torch.distributed as dist
        import __graft_entry__
        pkg = __graft_entry__.load_package()
        if backend == "nccl":
            dist.init_process_group("nccl", timeout=datetime.timedelta(seconds=120),
                                    device_id=torch.device("cuda", 0))
        else:
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=120))
        eng = pkg.engine.SelfPlayEngine(seed=SEED + rank, init_seed=INIT + rank, **CFG)
        x = pkg.shards.AvgPolicyExchange(eng, dist, every=1, transport=transport, gain=gain)
        out = []
        for _ in range(STEPS):
            eng.step()
            out.append(_state(pkg, eng))
        out.append(x.calls)
        x.close()
        q.put((rank, out))
        dist.destroy_process_group()
        eng.close()
    except Exception as ex:                      # surface the failure in the parent
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


def _ranks(world, backend, transport, gain=1.0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, backend, transport, gain)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert isinstance(res[r], list), res[r]
    assert all(p.exitcode == 0 for p in procs)
    return res


def _group(pkg, R, gain=1.0):
    g = pkg.engine.EngineGroup(R, seed=SEED, init_seed=INIT, **CFG)
    g.set_exchange(pkg.native.XCHG_AR, every=1, scale=gain / R)
    g.average_ar()                       # the ranks' broadcast: replica 0's AR nets everywhere
    out = []
    for _ in range(STEPS):
        g.step()
        out.append([_state(pkg, e) for e in g.replicas])
    g.close()
    return out


def _compare(rank_res, group_res, R):
    worst = 0.0
    for k in range(STEPS):
        for r in range(R):
            (wr, sr), (wg, sg) = rank_res[r][k], group_res[k][r]
            assert sr == sg, (k, r, sr, sg)
            for key in wr:
                worst = max(worst, float(np.abs(wr[key] - wg[key]).max()))
                assert np.array_equal(wr[key], wg[key]), (k, r, key, float(np.abs(wr[key] - wg[key]).max()))
    return worst


@pytest.mark.parametrize("gain", [1.0, 2.0])
def test_two_ranks_exchange_per_slice_like_the_group(pkg, gain):
    """2 co-resident pipelined ranks, gloo, the exchange after every slice's AR chain (gain 1 =
    the mean of the deltas, 2 = bench.py's default gain) == a 2-replica group at slice_lag 2
    with the same exchange: every net, counter and schedule, after each of 2 steps."""
    res = _ranks(2, "gloo", "host", gain)
    assert res[0][-1] == res[1][-1] == STEPS * CFG["slices"]          # one exchange per slice
    grp = _group(pkg, 2, gain)
    assert _compare(res, grp, 2) == 0.0
    w = res[0][-2][0]
    assert np.array_equal(w[(0, 0)], res[1][-2][0][(0, 0)])           # one AR net on both ranks
    assert not np.array_equal(w[(0, 1)], res[1][-2][0][(0, 1)])       # BR nets per shard


def test_rccl_transport_at_world_one(pkg):
    """libnfsp's RCCL communicator (ncclAllReduce in place on the AR chain stream) at world 1:
    the same nets as the host transport and as a 1-replica group with the exchange."""
    rccl = _ranks(1, "nccl", "rccl")
    host = _ranks(1, "gloo", "host")
    assert rccl[0][-1] == STEPS * CFG["slices"]
    for k in range(STEPS):
        assert rccl[0][k][1] == host[0][k][1]
        for key in rccl[0][k][0]:
            assert np.array_equal(rccl[0][k][0][key], host[0][k][0][key]), (k, key)
    assert _compare(rccl, _group(pkg, 1), 1) == 0.0


def test_group_exchange_turned_on_again_starts_from_replica_0(pkg):
    """nfsp_group_set_exchange turning the AR exchange on again (after steps with it off, the
    replicas' AR nets apart) starts like the rank path does (rank 0's nets broadcast, then W0 =
    them): the first exchange copies replica 0's nets everywhere, not W0_old + the deltas
    accumulated since the exchange was off."""
    import torch
    g = pkg.engine.EngineGroup(2, seed=SEED, init_seed=INIT, **CFG)
    g.set_exchange(pkg.native.XCHG_AR, every=1, scale=1.0)
    g.step()
    g.set_exchange(pkg.native.XCHG_AR, every=0)
    g.step()
    torch.cuda.synchronize()
    w_r0 = [g.replicas[0].get_weights(a, 0) for a in (0, 1)]
    assert not np.array_equal(w_r0[0], g.replicas[1].get_weights(0, 0))    # apart while off
    g.set_exchange(pkg.native.XCHG_AR, every=1, scale=1.0)
    g.average_ar()                                   # the exchange by itself
    torch.cuda.synchronize()
    for e in g.replicas:
        for a in (0, 1):
            assert np.array_equal(e.get_weights(a, 0), w_r0[a])
    g.step()                                         # and it trains on from there
    torch.cuda.synchronize()
    assert np.array_equal(g.replicas[0].get_weights(0, 0), g.replicas[1].get_weights(0, 0))
    g.close()
