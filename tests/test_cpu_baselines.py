"""bench.py's CPU baselines beside the GPU line (BASELINE.md's CPU plan): workloads (a) env +
scheduler with random action vectors and (b) the agents' play without updates -- the CPU
counterparts of rollout_only_hands_per_s -- by both restatements, one process per core."""
import os
import sys

from conftest import REPO


def test_rollout_baselines_report_both_workloads_and_restatements():
    sys.path.insert(0, REPO)
    import bench
    r = bench.cpu_baseline_rollout(0.5, "c3", cores=2)
    assert r["cores"] == 2 and r["unit"] == "hands/s" and "rollout_only" in r["gpu_counterpart"]
    for wl in ("a", "b"):
        for kind in ("port", "numpy"):
            v = r[wl][kind]
            assert v["hands"] > 0 and v["value"] > 0 and v["per_core"] > 0, (wl, kind, v)
    # the env alone is faster than play with forwards, in either restatement
    assert r["a"]["port"]["value"] > r["b"]["port"]["value"]
    assert r["a"]["numpy"]["value"] > r["b"]["numpy"]["value"]


def test_cpu_port_workload_b_plays_like_c_without_updates():
    """Workload (b) is main.train with update_strategy skipped: the same hands, inserts and
    actions as (c) until the first update (game_step 128), and no updates ever."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import cpu_port
    stats = {}
    for wl in ("b", "c"):
        g = cpu_port.CpuGame(cpu_port.make_cfg(None, 0, True, "leduc", workload=wl))
        g.train(10, 0)              # 10 hands: < 128 RL inserts per agent
        stats[wl] = g.stats()
        g.train(400, 0)
        stats[wl + "_late"] = g.stats()
        g.close()
    for k in ("rl_inserts", "sl_inserts", "hands", "actions"):
        assert stats["b"][k] == stats["c"][k], k
    assert sum(stats["b_late"]["br_updates"]) == sum(stats["b_late"]["ar_updates"]) == 0
    assert sum(stats["c_late"]["br_updates"]) > 0
