"""Observability: the scalar log and the engine scalars with the reference's tags."""
import json

import numpy as np
import pytest


def test_scalar_log_jsonl(pkg, tmp_path):
    obs = pkg.observability
    p = tmp_path / "log.jsonl"
    with obs.ScalarLog(str(p)) as log:
        log.write(0, **{"Player0rl/loss_mean": 0.5, "hands": 3})
        log.write(1, **{"Player0rl/loss_mean": np.float32(0.25)})
    rows = [json.loads(l) for l in p.read_text().splitlines()]
    assert [r["step"] for r in rows] == [0, 1]
    assert rows[1]["Player0rl/loss_mean"] == pytest.approx(0.25)
    assert all("wall_s" in r for r in rows)


@pytest.mark.gpu
def test_engine_scalars_tags(pkg):
    eng = pkg.engine.SelfPlayEngine(n_lanes=4096, rl_capacity=40_000, sl_capacity=40_000, seed=5)
    eng.set_loss_log(True)
    for _ in range(3):
        eng.step()
    sc = pkg.observability.engine_scalars(eng, exact=True)
    for a in (0, 1):
        for tag in ("rl", "sl"):
            v = sc[f"Player{a}{tag}/loss_mean"]
            assert np.isfinite(v) and v >= 0
        assert sc[f"Player{a}/folds"] + sc[f"Player{a}/calls"] + sc[f"Player{a}/raises"] > 0
    assert sc["hands"] == 3 * 4096
    assert sc["exploitability_exact_softmax"] >= 0


def test_save_curve_csv_and_png(pkg, tmp_path):
    """The curve artefact main.train plots at its end (main.py:122-123): CSV + PNG."""
    obs = pkg.observability
    obs.save_curve([1.5, 1.25, 1.0], str(tmp_path / "c.csv"), str(tmp_path / "c.png"))
    lines = (tmp_path / "c.csv").read_text().splitlines()
    assert lines[0] == "hands,exploitability proxy" and lines[1:] == ["0,1.5", "1,1.25", "2,1.0"]
    pytest.importorskip("matplotlib")
    assert (tmp_path / "c.png").read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"
    obs.save_curve([(128, 2.0), (256, 1.75)], str(tmp_path / "d.csv"))
    assert (tmp_path / "d.csv").read_text().splitlines()[1:] == ["128,2.0", "256,1.75"]
