"""The C++ restatement of main.train (oracle/nfsp_cpu.cpp, bench.py's cpu_baseline) against
the Python oracle (oracle/nfsp_oracle.py, pinned to the reference by the golden fixtures).

Both are run from the same seeds and must produce the same hands:
* identical deal, eta, eps and buffer draws, reproducing CPython `random` and numpy's
  legacy RandomState;
* identical action / insert / update counts, rewards and schedules (eps, lr, temp,
  iteration);
* the same memories record for record: observation bits, rewards and flags exact; the
  stored action vectors within 1e-5.

Weights and the proxy curve agree within 1e-5.  The tolerance covers the softmax (expf vs
numpy's SIMD exp, <= 2 ulp) and the gradient sums (row order vs BLAS); the ReLU forwards
match bit for bit.
"""
import numpy as np
import pytest

import cpu_port as cp
import nfsp_oracle as orc


def _bits(x):
    v = np.ravel(x)
    return int(sum(int(v[i] != 0) << i for i in range(orc.OBS_DIM)))


@pytest.fixture(scope="module", autouse=True)
def _lib():
    import os
    import subprocess
    if not os.path.exists(cp.LIB_PATH):
        subprocess.run(["make", "-s", "-C", cp.HERE], check=True)


@pytest.mark.parametrize("hands,quirks,game", [(3000, True, "leduc"), (1500, False, "leduc"),
                                               (1500, True, "kuhn")])
def test_cpu_port_matches_oracle(hands, quirks, game):
    cfg = dict(buffer=2000)
    env, p1, p2 = orc.make_main(cfg, init_seed=3, quirks=quirks)
    env.kuhn = game == "kuhn"
    curve = orc.train(env, p1, p2, hands)
    g = cp.CpuGame(cp.make_cfg(cfg, init_seed=3, quirks=quirks, game=game))
    ccurve = g.train(hands)
    st = g.stats()
    assert st["hands"] == hands and st["warnings"] == env.warnings
    np.testing.assert_allclose(ccurve, curve, atol=1e-5)
    for i, P in enumerate((p1, p2)):
        assert st["game_step"][i] == P.game_step
        assert st["rl_size"][i] == P._rl_memory.count and st["sl_size"][i] == P._sl_memory.count
        assert st["iteration"][i] == P.iteration and st["played"][i] == P.played
        assert st["actions"][i] == list(P.actions)
        assert st["reward"][i] == P.reward
        assert st["epsilon"][i] == P.epsilon and st["temp"][i] == P.temp
        assert st["lr_br"][i] == float(P.cur_lr_br)
        assert st["exploitability"][i] == pytest.approx(P.exploitability, abs=1e-6)
        for net, m in ((0, P.avg_strategy_model), (1, P.best_response_model), (2, P.target_br_model)):
            np.testing.assert_allclose(g.weights(i, net), m.flat(), atol=1e-5)
        s, a, r, s2, t = g.rl(i)
        items = list(P._rl_memory.items)
        assert [_bits(it[0]) for it in items] == list(s)
        assert [_bits(it[3]) for it in items] == list(s2)
        assert [float(it[2]) for it in items] == list(r)
        assert [bool(it[4]) for it in items] == [bool(x) for x in t]
        np.testing.assert_allclose(a, np.array([np.ravel(it[1]) for it in items]), atol=1e-5)
        ss, sa = g.sl(i)
        assert [_bits(it[0]) for it in P._sl_memory.items] == list(ss)
        np.testing.assert_allclose(sa, np.array([np.ravel(it[1]) for it in P._sl_memory.items]), atol=1e-5)


def test_cpu_port_bench_runs_replicas():
    c = cp.make_cfg(None, 0, True, "leduc", rl_capacity=5000, sl_capacity=5000)
    hands, el = cp.bench(c, 2, 0.3)
    assert hands > 0 and el >= 0.3
