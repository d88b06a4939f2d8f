"""MI355X-native NFSP-on-Leduc self-play engine (drop-in for the reference's
leduc.newenv / agent.agent / utils.* Python API, computed by libnfsp on the GPU).

Load with ``__graft_entry__.load_package()`` (the directory name is not an
identifier); it registers this package as ``nfsp_amd``.
"""
from . import native  # noqa: F401

__all__ = ["native", "install_dropin"]


def __getattr__(name):
    # heavy submodules (torch) load lazily so `native` can be probed without a GPU stack
    import importlib
    if name in ("leduc", "agent", "buffers", "selfplay", "engine", "observability", "pyrandom", "shards",
                "reference_main"):
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)


def install_dropin():
    """Register the reference's module names so main.py imports this engine unchanged:
    ``leduc.newenv`` -> .leduc, ``leduc.deck`` / ``leduc.cardmatrix`` -> .deck,
    ``agent.agent`` -> .agent, ``utils.replay_buffer`` / ``utils.ReservoirBuffer`` -> .buffers
    (see INTEGRATION.md)."""
    import importlib
    import sys
    import types
    pkg = sys.modules[__name__]
    le = importlib.import_module(".leduc", __name__)
    ag = importlib.import_module(".agent", __name__)
    bu = importlib.import_module(".buffers", __name__)
    dk = importlib.import_module(".deck", __name__)
    cm = types.ModuleType("cardmatrix")
    cm.Cardmatrix = dk.Cardmatrix
    for top, sub, mod in (("leduc", "newenv", le), ("leduc", "deck", dk), ("leduc", "cardmatrix", cm),
                          ("agent", "agent", ag),
                          ("utils", "replay_buffer", bu), ("utils", "ReservoirBuffer", bu)):
        parent = sys.modules.get(top) or types.ModuleType(top)
        parent.__path__ = []
        setattr(parent, sub, mod)
        sys.modules[top] = parent
        sys.modules[f"{top}.{sub}"] = mod
    return pkg
