"""Run the reference's own ``main.py``, unchanged, on the drop-in.

The reference's driver (``main.py``) imports ``tensorflow``, ``matplotlib.pyplot`` and the
py2 module ``ConfigParser`` at module level (main.py:1-11), reads ``./config.ini`` from the
working directory (main.py:17-18), opens a ``tf.Session`` only to hand it to
``agent.Agent`` and to run the variable initialiser (main.py:127-146), and ends ``train``
with ``plt.plot`` / ``plt.show()`` / ``time.sleep(60)`` (main.py:122-124).  With
``install_dropin()`` its ``leduc.newenv`` / ``agent.agent`` / ``utils.*`` imports resolve to
this engine; ``run`` adds the three host-side modules it still needs, as small stand-ins
that do what main.py asks of them and nothing else:

* ``tensorflow``: ``Session`` (a context manager whose ``run`` returns None),
  ``set_random_seed`` (recorded), ``global_variables_initializer`` (a marker).  The drop-in
  Agent keeps its nets on the GPU and ignores the session, as the reference's Keras models
  bind to the default one.
* ``matplotlib`` / ``matplotlib.pyplot``: ``plot`` keeps the curve (``run`` returns it);
  ``show`` opens no window; with ``plot_to``, the shown curve is written to
  ``plot_to``.csv / .png (``observability.save_curve``) once the file has run.
* ``ConfigParser``: Python 3's ``configparser.ConfigParser``, optionally with overrides
  (e.g. ``Common.Episodes`` for a short run).

Then the file runs as ``__main__`` (``runpy.run_path``) in its own directory, with
``sys.argv`` set, so its ``argparse`` block and ``main(args)`` run as written.  Nothing in
the file is edited.  The per-decision calls go through libnfsp (``leduc.Env``,
``agent.Agent``); the loop itself is main.py's Python, ~1.3k hands/s.

    python tools/run_reference_main.py /path/to/reference/main.py --episodes 2000 [-- main.py's args]

``modules`` (tests only) replaces what ``install_dropin`` registers, e.g. by the CPU
oracle's classes where there is no GPU.
"""
from __future__ import annotations

import argparse
import configparser
import contextlib
import importlib
import logging
import os
import runpy
import sys
import time
import types


class _Session:
    """main.py:129 ``with tf.Session() as sess`` and main.py:144 ``sess.run(...)``."""

    def __init__(self, *args, **kwargs):
        self.closed = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def run(self, fetches, *args, **kwargs):
        return None

    def close(self):
        self.closed = True


def tensorflow_stub() -> types.ModuleType:
    tf = types.ModuleType("tensorflow")
    tf.__nfsp_stub__ = True
    tf.seeds = []
    tf.Session = _Session
    tf.set_random_seed = tf.seeds.append
    tf.global_variables_initializer = lambda: "global_variables_initializer"
    return tf


def matplotlib_stub():
    mpl = types.ModuleType("matplotlib")
    plt = types.ModuleType("matplotlib.pyplot")
    mpl.__nfsp_stub__ = plt.__nfsp_stub__ = True
    plt.curves = []
    plt.shown = 0
    plt.plot = lambda y, *a, **k: plt.curves.append(list(y))

    def show(*a, **k):
        plt.shown += 1

    plt.show = show
    mpl.pyplot = plt
    return mpl, plt


def configparser_stub(overrides: dict | None = None) -> types.ModuleType:
    """``ConfigParser.ConfigParser`` (py2 name) whose ``get`` returns the override for a
    (section, option) pair when one is given."""
    ov = {(s.lower(), o.lower()): str(v) for (s, o), v in (overrides or {}).items()}

    class ConfigParser(configparser.ConfigParser):
        def get(self, section, option, *args, **kwargs):
            key = (section.lower(), option.lower())
            if key in ov:
                return ov[key]
            return super().get(section, option, *args, **kwargs)

    mod = types.ModuleType("ConfigParser")
    mod.ConfigParser = ConfigParser
    mod.RawConfigParser = configparser.RawConfigParser
    mod.SafeConfigParser = ConfigParser
    mod.Error = configparser.Error
    return mod


def time_stub() -> types.ModuleType:
    """``time`` for main.py's own code: everything is the real module's except ``sleep``, which
    returns at once (main.py:124 sleeps 60 s after plt.show()).  It is never put in sys.modules:
    only main.py's ``import time`` gets it (``main_builtins``), so a module imported for the first
    time during the run (the drop-in's, torch's) binds the real ``time``."""
    mod = types.ModuleType("time")
    mod.__dict__.update({k: v for k, v in vars(time).items() if not k.startswith("__")})
    mod.sleep = lambda seconds: None
    return mod


def main_builtins(time_mod: types.ModuleType) -> dict:
    """The builtins main.py's code runs with (its globals' ``__builtins__``): the real ones, but
    ``import time`` returns ``time_mod``.  Every other module keeps the real builtins and the
    real ``time`` (a stub in sys.modules would stick to whatever module was first
    imported during the run)."""
    import builtins
    real_import = builtins.__import__

    def _import(name, globals=None, locals=None, fromlist=(), level=0):
        if name == "time" and level == 0:
            return time_mod
        return real_import(name, globals, locals, fromlist, level)
    b = dict(vars(builtins))
    b["__import__"] = _import
    return b


@contextlib.contextmanager
def _patched(modules: dict, argv: list, cwd: str):
    saved_mods = {k: sys.modules.get(k) for k in modules}
    saved_argv, saved_cwd = sys.argv, os.getcwd()
    root = logging.getLogger()             # main.py:12 basicConfig(level=DEBUG) on the root logger
    saved_log = (root.level, list(root.handlers))
    try:
        sys.modules.update(modules)
        sys.argv = argv
        os.chdir(cwd)
        yield
    finally:
        root.setLevel(saved_log[0])
        root.handlers[:] = saved_log[1]
        os.chdir(saved_cwd)
        sys.argv = saved_argv
        for k, v in saved_mods.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


def run(main_py: str, episodes: int | None = None, argv=(), overrides: dict | None = None,
        skip_sleep: bool = True, plot_to: str | None = None, modules: dict | None = None) -> dict:
    """Run ``main_py`` (the reference's main.py) as ``__main__`` on the drop-in.

    episodes: overrides ``[Common] Episodes`` of its config.ini (main.py:27);
    overrides: further ``{(section, option): value}`` for its ConfigParser;
    skip_sleep: the ``time.sleep(60)`` after ``plt.show()`` (main.py:124) returns at once (the
      file's ``import time`` gets ``time_stub()``);
    plot_to: the curve ``plt.show()`` was asked to show goes to <plot_to>.csv / .png;
    modules: replaces the drop-in's module registrations (tests: the CPU oracle's classes).
    Returns ``{"globals": the module's globals, "curves": what it passed to plt.plot,
    "tf_seeds": its tf.set_random_seed calls}``."""
    main_py = os.path.abspath(main_py)
    if not os.path.isfile(main_py):
        raise FileNotFoundError(main_py)
    ov = dict(overrides or {})
    if episodes is not None:
        ov[("Common", "Episodes")] = int(episodes)
    if modules is None:
        pkg = importlib.import_module(__package__)
        pkg.install_dropin()
        mods = {}
    else:
        mods = dict(modules)
    tf = tensorflow_stub()
    mods["tensorflow"] = tf
    mpl, plt = matplotlib_stub()
    mods["matplotlib"], mods["matplotlib.pyplot"] = mpl, plt
    mods["ConfigParser"] = configparser_stub(ov)
    init = {"__builtins__": main_builtins(time_stub())} if skip_sleep else None
    with _patched(mods, [main_py, *argv], os.path.dirname(main_py)):
        g = runpy.run_path(main_py, init_globals=init, run_name="__main__")
    if plot_to and plt.shown and plt.curves:       # after the stand-ins are gone (real pyplot)
        from .observability import save_curve
        save_curve(plt.curves[-1], plot_to + ".csv", plot_to + ".png", xlabel="report")
    return {"globals": g, "curves": plt.curves, "tf_seeds": tf.seeds}


def main(argv=None):
    """CLI: ``<main.py> [--episodes N] [--sleep] [--plot-to PATH] [-- <main.py's own args>]``."""
    argv = list(sys.argv[1:] if argv is None else argv)
    own, rest = (argv[:argv.index("--")], argv[argv.index("--") + 1:]) if "--" in argv else (argv, [])
    ap = argparse.ArgumentParser(description="Run the reference's unchanged main.py on the MI355X drop-in.")
    ap.add_argument("main_py", help="path to the reference's main.py")
    ap.add_argument("--episodes", type=int, default=None, help="override [Common] Episodes")
    ap.add_argument("--sleep", action="store_true", help="keep main.py's time.sleep(60) at the end")
    ap.add_argument("--plot-to", default=None, help="plt.show() writes the curve to PATH.csv / PATH.png")
    a = ap.parse_args(own)
    out = run(a.main_py, episodes=a.episodes, argv=rest, skip_sleep=not a.sleep, plot_to=a.plot_to)
    if out["curves"]:
        print(f"exploitability-proxy curve: {len(out['curves'][-1])} points", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
