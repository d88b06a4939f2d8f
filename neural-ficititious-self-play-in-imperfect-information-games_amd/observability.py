"""Observability: the reference's scalar outputs for the batched engine.

The reference reports through three channels, and each has an equivalent here:

* ``sampled_actions`` (agent/agent.py:196-204) prints per-agent action counts and rewards.
  The engine's counterpart is ``nfsp_engine_stats``' ``actions`` and ``reward`` fields (the
  drop-in ``Agent.sampled_actions`` keeps the reference's print).
* TensorBoard callbacks on every ``fit`` (agent/agent.py:84-88,243,264) log the epoch loss
  under ``./logs/<name>rl`` (BR) and ``./logs/<name>sl`` (AR).  The engine's loss log
  (``SelfPlayEngine.set_loss_log``) gives the same values; TensorBoard itself is not in the
  image, so they are written as JSON lines with the same tags.
* The exploitability proxy is printed and plotted (main.py:71-75,122-123).  It is logged
  here beside the exact exploitability (``nfsp_exploitability``).
"""
from __future__ import annotations

import json
import time


class ScalarLog:
    """One JSON object per line: ``{"step": k, "wall_s": t, <tag>: value, ...}``."""

    def __init__(self, path: str):
        self.f = open(path, "a", buffering=1)
        self.t0 = time.perf_counter()

    def write(self, step: int, **scalars):
        rec = {"step": int(step), "wall_s": round(time.perf_counter() - self.t0, 6)}
        for k, v in scalars.items():            # numpy scalars included
            rec[k] = v.item() if hasattr(v, "item") else v
        self.f.write(json.dumps(rec) + "\n")

    def close(self):
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def engine_scalars(eng, exact: bool = False) -> dict:
    """The scalars of one engine step, tagged like the reference's outputs."""
    st = eng.stats()
    out = {"hands": int(st["hands"]),
           "exploitability_proxy": float(sum(st["exploitability"]))}       # main.py:73
    for a in (0, 1):
        name = f"Player{a}"
        acts = st["actions"][a]
        out[f"{name}/folds"], out[f"{name}/calls"], out[f"{name}/raises"] = (int(x) for x in acts)
        out[f"{name}/reward"] = float(st["reward"][a])
        out[f"{name}/epsilon"] = float(st["epsilon"][a])
        out[f"{name}/lr_br"] = float(st["lr_br"][a])
        out[f"{name}/temp"] = float(st["temp"][a])
        out[f"{name}/iteration"] = int(st["iteration"][a])
        out[f"{name}/br_updates"] = int(st["br_updates"][a])
        out[f"{name}/ar_updates"] = int(st["ar_updates"][a])
        out[f"{name}/proxy"] = float(st["exploitability"][a])
    if getattr(eng, "loss_log", False):
        out.update(eng.losses())
    if exact:
        for m, tag in ((0, "softmax"), (1, "argmax")):
            out[f"exploitability_exact_{tag}"] = eng.exploitability(m)["exploitability"]
    return out


def save_curve(points, csv_path: str, png_path: str | None = None, ylabel: str = "exploitability proxy",
               xlabel: str = "hands") -> None:
    """The curve main.train plots at its end (main.py:122-123: plt.plot(plotter)), as a CSV
    artefact and, when matplotlib is importable, a PNG (Agg backend, no display).  `points`:
    a sequence of (x, y) pairs or plain y values (x = their index, as plt.plot(plotter))."""
    pts = [(i, p) if not isinstance(p, (tuple, list)) else tuple(p) for i, p in enumerate(points)]
    with open(csv_path, "w") as f:
        f.write(f"{xlabel},{ylabel}\n")
        for x, y in pts:
            f.write(f"{x},{float(y)!r}\n")
    if png_path is None:
        return
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        return
    fig, ax = plt.subplots(figsize=(6, 4))
    ax.plot([p[0] for p in pts], [p[1] for p in pts])
    ax.set_xlabel(xlabel)
    ax.set_ylabel(ylabel)
    fig.tight_layout()
    fig.savefig(png_path, dpi=100)
    plt.close(fig)
