"""The reference's own main.py, unchanged, through nfsp_amd.reference_main (CPU).

`reference_main.run` supplies the host-side modules main.py imports besides the drop-in
(tensorflow, matplotlib.pyplot, ConfigParser) and runs the file as __main__ in its own
directory.  Here, without a GPU, the leduc.newenv / agent.agent registrations are the CPU
oracle's classes (test infrastructure); the GPU suite runs the same launcher on the drop-in
(tests/test_gpu_dropin.py).  The run must be main.train's: the same curve, hand for hand,
as the oracle's restatement of main.train (nfsp_oracle.train, pinned to the reference's
event log) from the same seeds.
"""
import os
import random
import types

import numpy as np
import pytest

import nfsp_oracle as orc

REF_MAIN = "/root/reference/main.py"


def _oracle_modules():
    leduc = types.ModuleType("leduc")
    leduc.__path__ = []
    newenv = types.ModuleType("leduc.newenv")
    newenv.Env = orc.Env
    leduc.newenv = newenv
    agent = types.ModuleType("agent")
    agent.__path__ = []
    agentm = types.ModuleType("agent.agent")
    agentm.Agent = orc.Agent
    agent.agent = agentm
    return {"leduc": leduc, "leduc.newenv": newenv, "agent": agent, "agent.agent": agentm}


def test_stubs_cover_what_main_py_uses(pkg):
    rm = pkg.reference_main
    tf = rm.tensorflow_stub()
    with tf.Session() as sess:
        assert sess.run(tf.global_variables_initializer()) is None
    assert sess.closed
    tf.set_random_seed(1234)
    assert tf.seeds == [1234]
    mpl, plt = rm.matplotlib_stub()
    plt.plot([1.0, 2.0])
    plt.show()
    assert plt.curves == [[1.0, 2.0]] and plt.shown == 1 and mpl.pyplot is plt
    import time
    ts = rm.time_stub()
    assert ts.sleep(60) is None and ts.time is time.time and time.sleep is not ts.sleep
    # only code run with main_builtins gets the stub; sys.modules keeps the real module
    import sys
    g = {"__builtins__": rm.main_builtins(ts)}
    exec("import time\nimport os\ndef f():\n    import time as t\n    return t", g)
    assert g["time"] is ts and g["f"]() is ts and g["os"] is sys.modules["os"]
    assert sys.modules["time"] is time
    cp = rm.configparser_stub({("Common", "Episodes"): 7}).ConfigParser()
    cp.read_string("[Common]\nEpisodes: 400000\n[Agent]\nEta: 0.1\n")
    assert cp.get("Common", "Episodes") == "7" and cp.get("Agent", "Eta") == "0.1"


@pytest.mark.skipif(not os.path.isfile(REF_MAIN), reason="the reference checkout is not present")
def test_reference_main_py_runs_unchanged(pkg, capsys, tmp_path):
    before = open(REF_MAIN, "rb").read()
    episodes = 450
    random.seed(20261017)
    out = pkg.reference_main.run(REF_MAIN, episodes=episodes, modules=_oracle_modules(),
                                 plot_to=str(tmp_path / "curve"))
    assert open(REF_MAIN, "rb").read() == before              # nothing edited
    import sys
    import time
    assert out["globals"]["time"].sleep is not time.sleep     # main.py's own sleep is skipped ...
    assert sys.modules["time"] is time                        # ... and nobody else's
    printed = capsys.readouterr().out
    assert "NFSP by David Joos" in printed                    # main.py:151, its __main__ block ran
    assert out["tf_seeds"] == [1234]                          # main.py:133 with config.ini's Seed
    reports = [i for i in range(episodes) if i > 150 and i % 100 == 0]
    assert printed.count("Exploitability:") == len(reports)
    assert out["curves"] is not None and len(out["curves"]) == 1
    curve = out["curves"][0]
    assert len(curve) == len(reports)
    rows = (tmp_path / "curve.csv").read_text().strip().split("\n")[1:]   # main.py:122-123's plot
    assert [float(r.split(",")[1]) for r in rows] == curve

    # the oracle's main.train from the same state: main.main() is Env(), np.random.seed(Seed),
    # two Agents, train (main.py:127-146); the stdlib `random` main.py draws from is unseeded
    # by it, so both runs start from random.seed(20261017)
    random.seed(20261017)
    env = orc.Env()
    np.random.seed(1234)
    p1 = orc.Agent(None, env.observation_space, env.action_space, "Player0", env)
    p2 = orc.Agent(None, env.observation_space, env.action_space, "Player1", env)
    ref = orc.train(env, p1, p2, episodes)
    assert curve == ref


def test_cli_splits_its_own_options_from_main_py_args(pkg, monkeypatch):
    seen = {}

    def fake_run(main_py, episodes=None, argv=(), skip_sleep=True, plot_to=None, **kw):
        seen.update(main_py=main_py, episodes=episodes, argv=list(argv), skip_sleep=skip_sleep, plot_to=plot_to)
        return {"curves": [], "tf_seeds": [], "globals": {}}

    monkeypatch.setattr(pkg.reference_main, "run", fake_run)
    assert pkg.reference_main.main(["m.py", "--episodes", "10", "--plot-to", "c", "--", "--human"]) == 0
    assert seen == dict(main_py="m.py", episodes=10, argv=["--human"], skip_sleep=True, plot_to="c")
    pkg.reference_main.main(["m.py", "--sleep"])
    assert seen["argv"] == [] and seen["episodes"] is None and not seen["skip_sleep"]
