"""Engine groups (nfsp_group_*): R replicas stepped together, their SGD chains in shared
launches (one AR launch of 2R workgroups, BR rounds of every (replica, agent)'s k-th
target-sync segment).

Bar: replica r of a group is BIT-IDENTICAL to a standalone engine with seed + r and
init_seed + r stepped as often -- every net, the memories, the counters and schedules.
The standalone engine is itself pinned to the oracle (test_gpu_engine / test_gpu_learner),
so this carries that parity over to the grouped launches.  With the AR exchange on, the AR
nets equal shards.AvgPolicyAllReduce's W0 + sum_r (W_r - W0) / R, recomputed here in numpy
f32 in replica order from standalone engines stepped from the same common nets."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# small memories (M_RL wraps, M_SL replaces) and a short target-sync period, so one step has
# several BR rounds whose segments differ between replicas and agents
SMALL = dict(n_lanes=2048, rl_capacity=3000, sl_capacity=2000, target_every=7)


def nets(eng):
    return [eng.get_weights(a, n) for a in (0, 1) for n in (0, 1, 2)]


def mem(eng, a):
    m = eng.memories(a)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in m.items() if isinstance(v, torch.Tensor)}


STAT_KEYS = ("hands", "rl_total", "sl_total", "rl_size", "sl_size", "br_updates", "ar_updates",
             "iteration", "target_syncs", "actions", "reward", "epsilon", "temp", "lr_br",
             "exploitability")


@pytest.mark.parametrize("quirks,R", [(None, 3), (120, 2)])
def test_group_replicas_match_standalone_engines(pkg, quirks, R):
    kw = dict(SMALL)
    if quirks is not None:
        kw["quirks"] = quirks
    g = pkg.engine.EngineGroup(R, seed=777, init_seed=5, **kw)
    solo = [pkg.engine.SelfPlayEngine(seed=777 + r, init_seed=5 + r, **kw) for r in range(R)]
    for step in range(3):
        g.step()
        for e in solo:
            e.step()
        torch.cuda.synchronize()
        assert g.rounds() >= 2 or g.sched()["br_persist"]   # (one launch under NFSP_GROUP_BR_PERSIST)
        for r in range(R):
            a_st, b_st = g.replicas[r].stats(), solo[r].stats()
            for k in STAT_KEYS:
                assert a_st[k] == b_st[k], (step, r, k, a_st[k], b_st[k])
            for x, y in zip(nets(g.replicas[r]), nets(solo[r])):
                assert np.array_equal(x, y), (step, r)
    for r in range(R):
        for a in (0, 1):
            ma, mb = mem(g.replicas[r], a), mem(solo[r], a)
            for k in ma:
                assert np.array_equal(ma[k], mb[k]), (r, a, k)
    # replicas differ from each other (own seeds)
    assert not np.array_equal(nets(g.replicas[0])[0], nets(g.replicas[1])[0])


def test_group_loss_log_matches_standalone(pkg):
    g = pkg.engine.EngineGroup(2, seed=31, init_seed=2, **SMALL)
    solo = [pkg.engine.SelfPlayEngine(seed=31 + r, init_seed=2 + r, **SMALL) for r in range(2)]
    for e in g.replicas + solo:
        e.set_loss_log(True)
    for _ in range(2):
        g.step()
        for e in solo:
            e.step()
    for r in range(2):
        la, lb = g.replicas[r].losses(), solo[r].losses()
        for k in la:
            assert (np.isnan(la[k]) and np.isnan(lb[k])) or la[k] == lb[k], (r, k)


def test_group_ar_exchange(pkg):
    """avg_ar: replica 0's AR nets go everywhere first; after each step every replica holds
    W0 + sum_r (W_r - W0) / R (f32, replica order) of the replicas' own SGD results."""
    R = 3
    g = pkg.engine.EngineGroup(R, seed=99, init_seed=0, avg_ar=True, **SMALL)
    solo = [pkg.engine.SelfPlayEngine(seed=99 + r, init_seed=r, **SMALL) for r in range(R)]
    w0 = [solo[0].get_weights(a, 0) for a in (0, 1)]
    for e in solo:
        for a in (0, 1):
            e.set_weights(a, 0, w0[a])
    for step in range(2):
        g.step()
        for e in solo:
            e.step()
        torch.cuda.synchronize()
        for a in (0, 1):
            base = w0[a].astype(np.float32)
            s = np.zeros_like(base)
            for e in solo:
                s = (s + (e.get_weights(a, 0) - base)).astype(np.float32)
            exp = (base + s * np.float32(1.0 / R)).astype(np.float32)
            for r in range(R):
                assert np.array_equal(g.replicas[r].get_weights(a, 0), exp), (step, a, r)
            w0[a] = exp
            for e in solo:                          # the standalone side's own exchange
                e.set_weights(a, 0, exp)
        # BR nets stay per replica, and equal the standalone engines' (same AR nets acted)
        for r in range(R):
            for a in (0, 1):
                assert np.array_equal(g.replicas[r].get_weights(a, 1), solo[r].get_weights(a, 1))


def test_group_replica_refuses_its_own_update(pkg):
    g = pkg.engine.EngineGroup(2, **SMALL)
    with pytest.raises(pkg.native.NativeError):
        g.replicas[0].step()
    g.step()                                       # the group still steps
    assert g.stats()["hands"] == 2 * SMALL["n_lanes"]


@pytest.mark.parametrize("R", [80, 200])
def test_group_sharing_cus_matches_standalone_engines(pkg, R):
    """Past 64 replicas, 2 (R = 80) or 4 (R = 200) chain workgroups share a CU, each with a
    share of its LDS (chain_lds_shared).  The chain's results must not change: replicas at
    both ends of the group stay bit-identical to standalone engines over 2 steps."""
    kw = dict(n_lanes=256, rl_capacity=1500, sl_capacity=1000, target_every=7)
    g = pkg.engine.EngineGroup(R, seed=4242, init_seed=3, **kw)
    picks = (0, R // 2, R - 1)
    solo = {r: pkg.engine.SelfPlayEngine(seed=4242 + r, init_seed=3 + r, **kw) for r in picks}
    for step in range(2):
        g.step()
        for e in solo.values():
            e.step()
        torch.cuda.synchronize()
        for r in picks:
            gs, ss = g.replicas[r].stats(), solo[r].stats()
            for k in STAT_KEYS + ("rollouts",):      # incl. the counters past replica 64
                assert gs[k] == ss[k], (step, r, k)
            for x, y in zip(nets(g.replicas[r]), nets(solo[r])):
                assert np.array_equal(x, y), (step, r)
    st = g.stats()
    assert sum(st["br_updates"]) > 0
    assert st["hands"] == 2 * R * kw["n_lanes"] and st["rollouts"] == 2 * R
    g.close()


def test_sliced_group_matches_sliced_standalone_engines(pkg):
    """cfg.slices in a group: every replica advances its lanes slice by slice like a sliced
    standalone engine with its seed (the AR exchange after each whole step)."""
    kw = dict(n_lanes=1024, slices=4, rl_capacity=3000, sl_capacity=2000, target_every=11)
    R = 3
    g = pkg.engine.EngineGroup(R, seed=555, init_seed=1, **kw)
    solo = [pkg.engine.SelfPlayEngine(seed=555 + r, init_seed=1 + r, **kw) for r in range(R)]
    for step in range(3):
        g.step()
        for e in solo:
            e.step()
        for r in range(R):
            gs, ss = g.replicas[r].stats(), solo[r].stats()
            for k in STAT_KEYS + ("rollouts",):
                assert gs[k] == ss[k], (step, r, k)
            for x, y in zip(nets(g.replicas[r]), nets(solo[r])):
                assert np.array_equal(x, y), (step, r)
    assert g.stats()["rollouts"] == 3 * 4 * R
    assert min(g.stats()["br_updates"]) > 0


def test_group_replica_count_bounds(pkg):
    with pytest.raises(pkg.native.NativeError, match="replicas"):
        pkg.engine.EngineGroup(0, **SMALL)
    with pytest.raises(pkg.native.NativeError, match="replicas"):
        pkg.engine.EngineGroup(pkg.native.GROUP_MAX_REPLICAS + 1, **SMALL)


def test_group_trace_records_every_slice_plan(pkg):
    """nfsp_group_set_trace / nfsp_group_trace (tools/c4_slice_spread.py): one [R][agent][AR, BR]
    row of update counts per learner call (slice), summing over the step's slices to the
    replicas' update counters."""
    kw = dict(n_lanes=1024, slices=4, rl_capacity=3000, sl_capacity=2000, target_every=11)
    g = pkg.engine.EngineGroup(2, seed=77, init_seed=5, **kw)
    g.step()
    before = [r.stats() for r in g.replicas]
    g.set_trace(True)
    g.step()
    t = g.trace()
    g.set_trace(False)
    after = [r.stats() for r in g.replicas]
    assert t.shape == (4, 2, 2, 2)
    assert g.trace().shape[0] == 0                 # stopping clears it
    for r in range(2):
        for a in range(2):
            assert t[:, r, a, 1].sum() == after[r]["br_updates"][a] - before[r]["br_updates"][a]
            assert t[:, r, a, 0].sum() >= after[r]["ar_updates"][a] - before[r]["ar_updates"][a]
    g.close()


def test_pipelined_group_with_br_partitions_is_deterministic(pkg):
    """A sliced, pipelined group (slice_lag 2) runs its BR jobs in 2 partitions on their own
    streams, each partition going on into the next slice while the other finishes; every
    partition takes its replicas' BR results and snapshot itself before its next chains.  Two
    runs from the same seeds give the same nets bit for bit (a snapshot taken after the join,
    while a partition already ran the next slice's chains, moved C4's learning curve)."""
    kw = dict(n_lanes=65_536, slices=16, slice_lag=2, rl_capacity=200_000, sl_capacity=400_000)
    runs = []
    for _ in range(2):
        g = pkg.engine.EngineGroup(4, seed=4242, init_seed=3, **kw)
        g.set_exchange(pkg.native.XCHG_AR, every=1, scale=2.0 / 4)
        g.average_ar()
        for _ in range(3):
            g.step()
        assert min(g.stats()["br_updates"]) > 500
        runs.append([x.copy() for r in g.replicas for x in nets(r)])
        g.close()
    for x, y in zip(*runs):
        assert np.array_equal(x, y)


def test_group_sched_changes_no_sgd_step(pkg):
    """VERDICT r05 item 7 / ADVICE r05: the group's BR-round and slice schedule is a per-group
    setting (nfsp_group_set_sched), not process-static environment.  In ONE process, a
    4-replica pipelined group with the per-slice exchange runs under the default schedule (pieces
    of <= 40 paced, 2 BR partitions), then under whole segments on one stream, 16-update plain
    pieces on 4 partitions, and the serial slice loop: nets and counters bit for bit the same
    (a piece resumes from the weights in memory; the partitions run the same pieces)."""
    kw = dict(n_lanes=65_536, slices=16, slice_lag=2, rl_capacity=200_000, sl_capacity=400_000)
    variants = [dict(br_persist=0), dict(br_cap=0, br_pace=0, br_streams=1, br_persist=0),
                dict(br_cap=16, br_pace=0, br_streams=4, br_persist=0),
                dict(br_cap=40, br_pace=1, br_streams=3, br_persist=0), dict(serial=1), dict(br_persist=1)]
    runs = []
    for v in variants:
        g = pkg.engine.EngineGroup(4, seed=5151, init_seed=4, **kw)
        d = g.sched()
        if not any(k.startswith("NFSP_GROUP_") for k in os.environ):   # the defaults' environment
            assert d == dict(br_cap=-1, br_pace=1, br_streams=-1, serial=0, br_persist=0), d
        if v:
            g.set_sched(**v)
            assert all(g.sched()[k] == x for k, x in v.items())
        g.set_exchange(pkg.native.XCHG_AR, every=1, scale=2.0 / 4)
        g.average_ar()
        for _ in range(2):
            g.step()
        g.check()
        st = [r.stats() for r in g.replicas]
        assert min(min(s["br_updates"]) for s in st) > 300
        runs.append(([x.copy() for r in g.replicas for x in nets(r)], st, g.rounds()))
        g.close()
    base_nets, base_st, _ = runs[0]
    for v, (ns, st, _) in zip(variants[1:], runs[1:]):
        assert st == base_st, v
        for x, y in zip(base_nets, ns):
            assert np.array_equal(x, y), v
    # the schedules differ where they should: whole segments take fewer rounds than 16-pieces
    assert runs[1][2] < runs[2][2]
    with pytest.raises(Exception):
        g2 = pkg.engine.EngineGroup(2, seed=1, init_seed=0, **kw)
        try:
            g2.set_sched(br_streams=9)
        finally:
            g2.close()


@pytest.mark.parametrize("R", [1, 3])
def test_persistent_br_kernel_matches_standalone_engines(pkg, R):
    """sched br_persist: a learner call's BR work as ONE k_br_persist launch (chain workgroups
    taking 16-update pieces as 48 helper workgroups write the targets from a device work queue;
    DESIGN.md Appendix A.1b).  Short target-sync segments (7 updates) make many hand-offs per
    call.  Replicas stay bit-identical to standalone engines (which run the rounds' kernels)."""
    g = pkg.engine.EngineGroup(R, seed=2024, init_seed=7, **SMALL)
    g.set_sched(br_persist=1)
    solo = [pkg.engine.SelfPlayEngine(seed=2024 + r, init_seed=7 + r, **SMALL) for r in range(R)]
    for step in range(3):
        g.step()
        for e in solo:
            e.step()
        g.check()
        assert g.rounds() == 1                     # one launch per learner call
        for r in range(R):
            a_st, b_st = g.replicas[r].stats(), solo[r].stats()
            for k in STAT_KEYS:
                assert a_st[k] == b_st[k], (step, r, k, a_st[k], b_st[k])
            for x, y in zip(nets(g.replicas[r]), nets(solo[r])):
                assert np.array_equal(x, y), (step, r)
    assert min(g.replicas[0].stats()["target_syncs"]) >= 3
    g.close()


def test_persistent_br_kernel_c4_shape_matches_rounds(pkg):
    """C4's group shape (8 replicas, pipelined slices, the AR exchange after every slice) with
    the persistent BR kernel against the rounds: the same nets and counters bit for bit."""
    kw = dict(n_lanes=131_072, slices=32, slice_lag=2, rl_capacity=200_000, sl_capacity=400_000)
    runs = []
    for persist in (0, 1):
        g = pkg.engine.EngineGroup(8, seed=8080, init_seed=8, **kw)
        g.set_sched(br_persist=persist)
        g.set_exchange(pkg.native.XCHG_AR, every=1, scale=2.0 / 8)
        g.average_ar()
        for _ in range(2):
            g.step()
        g.check()
        st = [r.stats() for r in g.replicas]
        assert min(min(s["br_updates"]) for s in st) > 100
        runs.append(([x.copy() for r in g.replicas for x in nets(r)], st))
        g.close()
    assert runs[0][1] == runs[1][1]
    for x, y in zip(runs[0][0], runs[1][0]):
        assert np.array_equal(x, y)


def test_persistent_br_kernel_expired_wait_is_reported(pkg):
    """br_persist > 1 bounds every device wait at that many s_sleep rounds.  At 2 the chains'
    first waits expire before the helpers have written their targets: the kernel ends (it does
    not hang) and nfsp_group_check reports the expired hand-off."""
    g = pkg.engine.EngineGroup(2, seed=3, init_seed=1, **SMALL)
    g.set_sched(br_persist=2)
    g.step()
    try:
        g.check()
    except pkg.native.NativeError as ex:
        assert "bounded wait expired" in str(ex)
    else:
        pytest.skip("every hand-off was ready at its first poll (no wait expired)")
    finally:
        g.close()
