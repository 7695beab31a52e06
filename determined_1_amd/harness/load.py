"""Load the user's Trial class and build its controller (reference ``load/_load_implementation.py``
and ``load/_load_trial_controller.py:10-143``).

Two ways a trial process finds the user's Trial class:

  * ``entrypoint: "module:Class"`` in the experiment config (``load_trial_class``);
  * Native-API experiments (``det.experimental.create`` from a script or notebook) carry
    ``internal.native.command = [script, *argv]`` instead.  The trial process re-runs that script
    with ``runpy`` inside a ``RunpyGlobals`` context; there ``create()`` does not submit anything:
    it hands its ``trial_def`` to the loader and raises ``StopLoadingImplementation``, which skips
    the rest of the script (reference ``load/_load_implementation.py:69-196``).
"""
import contextlib
import importlib
import json
import logging
import os
import pathlib
import runpy
import sys
from typing import Any, Dict, Iterator, List, Optional, Type

from determined_1_amd import errors, trial, workload
from determined_1_amd.env import EnvContext, RendezvousInfo
from determined_1_amd.parallel.dist import DistributedConfig, RankInfo


def notebook_source(notebook_path: str) -> str:
    """The code cells of a Jupyter notebook as one Python script (reference
    ``load/_load_implementation.py:147``): IPython magics (``%...``) are commented out and shell
    escapes (``!...``) dropped, so the script runs under plain Python.  The one converter behind
    both the entrypoint loader (``notebook_to_py``) and the Native-API loader
    (``convert_notebook_to_python_script``)."""
    if not notebook_path.endswith(".ipynb"):
        raise errors.InvalidExperimentException(f"{notebook_path} is not a .ipynb notebook")
    nb = json.loads(pathlib.Path(notebook_path).read_text())
    if "cells" not in nb:
        raise errors.InvalidExperimentException(f"{notebook_path}: not a notebook (no cells)")
    out = []  # type: List[str]
    for cell in nb["cells"]:
        if cell.get("cell_type") != "code":
            continue
        src = cell.get("source", [])
        text = "".join(src) if isinstance(src, list) else str(src)
        for ln in text.splitlines():
            st = ln.lstrip()
            if st.startswith("!"):
                continue
            out.append(("# " + ln) if st.startswith("%") else ln)
        out.append("")
    return "\n".join(out)


def notebook_to_py(ipynb: pathlib.Path) -> pathlib.Path:
    """An entrypoint module shipped as ``<name>.ipynb``: write ``<name>.py`` next to it."""
    out = ipynb.with_suffix(".py")
    out.write_text(notebook_source(str(ipynb)))
    return out


def isolate_model_dir(d: str) -> None:
    """Put model directory ``d`` first on ``sys.path`` and evict cached modules named like one of its
    ``*.py`` files but loaded from elsewhere (two example directories that both ship a ``data.py``,
    loaded into one process, must each import their own)."""
    if d in sys.path:
        sys.path.remove(d)
    sys.path.insert(0, d)
    import sysconfig

    installed = tuple(os.path.abspath(p) for p in {sysconfig.get_paths()[k] for k in ("stdlib", "purelib", "platlib")})
    for f in os.listdir(d):
        if not f.endswith(".py"):
            continue
        m = sys.modules.get(f[:-3])
        mf = getattr(m, "__file__", None) if m is not None else None
        if not mf:
            continue
        mf = os.path.abspath(mf)
        # only user-code siblings from other model dirs, never installed or standard-library modules
        if os.path.dirname(mf) != d and not mf.startswith(installed):
            del sys.modules[f[:-3]]


def load_trial_class(entrypoint: str, model_dir: Optional[str] = None) -> Type[trial.Trial]:
    """``"module.sub:Class[.Inner]"`` -> the class.  The module is re-imported fresh (the reference
    pops it from ``sys.modules`` so a changed model definition is picked up)."""
    if ":" not in entrypoint:
        raise ValueError(f"entrypoint must look like 'module:TrialClass', got {entrypoint!r}")
    mod_name, qual = entrypoint.split(":", 1)
    if model_dir:
        isolate_model_dir(str(pathlib.Path(model_dir).resolve()))
    base = pathlib.Path(model_dir or ".")
    nb = base.joinpath(*mod_name.split(".")).with_suffix(".ipynb")
    if nb.exists() and not nb.with_suffix(".py").exists():
        notebook_to_py(nb)
    sys.modules.pop(mod_name, None)
    mod = importlib.import_module(mod_name)
    obj: Any = mod
    for part in qual.split("."):
        obj = getattr(obj, part)
    if not (isinstance(obj, type) and issubclass(obj, trial.Trial)):
        raise TypeError(f"{entrypoint} is not a Trial subclass")
    return obj


class RunpyGlobals:
    """Process-wide loader state while a Native-API command re-runs in a trial process: the env
    and distributed config for user code, and the Trial class ``create()`` hands back."""

    _instance = None  # type: Optional[RunpyGlobals]

    def __init__(self, env: Optional[EnvContext] = None, dist_config: Optional[DistributedConfig] = None) -> None:
        self.env = env
        self.dist_config = dist_config
        self.trial_cls = None  # type: Optional[Type[trial.Trial]]

    def __enter__(self) -> "RunpyGlobals":
        if RunpyGlobals._instance is not None:
            raise errors.InternalException("RunpyGlobals is already active (nested native loads)")
        RunpyGlobals._instance = self
        return self

    def __exit__(self, *_: Any) -> None:
        RunpyGlobals._instance = None

    @classmethod
    def is_initialized(cls) -> bool:
        return cls._instance is not None

    @classmethod
    def get_instance(cls) -> "RunpyGlobals":
        if cls._instance is None:
            raise errors.InternalException("RunpyGlobals is not active")
        return cls._instance

    @classmethod
    def set_runpy_trial_result(cls, trial_cls: Type[trial.Trial]) -> None:
        """Called by ``create()`` inside the loader: record the class and stop running the script."""
        inst = cls.get_instance()
        if inst.trial_cls is not None:
            raise errors.InvalidExperimentException("det.experimental.create() was called twice by one script")
        if not (isinstance(trial_cls, type) and issubclass(trial_cls, trial.Trial)):
            raise errors.InvalidExperimentException(f"{trial_cls!r} is not a Trial subclass")
        inst.trial_cls = trial_cls
        raise errors.StopLoadingImplementation()


def convert_notebook_to_python_script(notebook_path: str) -> str:
    """``x.ipynb`` -> ``x__det__.py`` (a Native-API notebook command), next to the notebook so
    relative imports and data paths keep working."""
    src = notebook_source(notebook_path)
    dst = notebook_path[: -len(".ipynb")] + "__det__.py"
    pathlib.Path(dst).write_text(src)
    return dst


@contextlib.contextmanager
def overwrite_sys_args(new_args: List[str]) -> Iterator[None]:
    old = sys.argv
    sys.argv = list(new_args)
    try:
        yield
    finally:
        sys.argv = old


def native_command(cfg: Dict[str, Any]) -> Optional[List[str]]:
    internal = cfg.get("internal") or {}
    native = internal.get("native") if isinstance(internal, dict) else None
    if not native:
        return None
    cmd = native.get("command") if isinstance(native, dict) else None
    if not cmd:
        raise errors.InvalidExperimentException("internal.native.command is empty")
    return [str(c) for c in cmd]


def load_native_implementation(env: Optional[EnvContext] = None,
                               dist_config: Optional[DistributedConfig] = None,
                               command: Optional[List[str]] = None) -> Type[trial.Trial]:
    """Re-run a Native-API script (or converted notebook) until it calls ``create()``."""
    cmd = list(command if command is not None else native_command(env.experiment_config if env else {}) or [])
    if not cmd:
        raise errors.InvalidExperimentException("no native command to load")
    logging.info("loading native implementation with command %s", cmd)
    if cmd[0].endswith(".ipynb"):
        cmd[0] = convert_notebook_to_python_script(cmd[0])
    script_dir = os.path.dirname(os.path.abspath(cmd[0]))
    if script_dir not in sys.path:
        sys.path.insert(0, script_dir)
    with RunpyGlobals(env, dist_config) as loader:
        with overwrite_sys_args(cmd):
            try:
                runpy.run_path(cmd[0], run_name="__main__")
            except errors.StopLoadingImplementation:
                pass  # create() handed the class over; the rest of the script is the submitter's
    if loader.trial_cls is None:
        raise errors.InvalidExperimentException(
            f"{cmd[0]} finished without calling det.experimental.create(trial_def=...)")
    return loader.trial_cls


def load_trial_for_config(cfg: Dict[str, Any], env: Optional[EnvContext] = None,
                          dist_config: Optional[DistributedConfig] = None) -> Type[trial.Trial]:
    if native_command(cfg) is not None:
        return load_native_implementation(env, dist_config, native_command(cfg))
    return load_trial_class(cfg["entrypoint"])


def prepare_controller(env: EnvContext, workloads: workload.Stream, load_path: Optional[pathlib.Path],
                       rendezvous: RendezvousInfo, dist_config: DistributedConfig,
                       rank_info: Optional[RankInfo] = None) -> trial.TrialController:
    """pre_execute_hook -> context -> Trial(context) -> controller.from_trial (reference
    ``load_controller_from_trial``)."""
    from determined_1_amd.harness import timeline

    trial_class = load_trial_for_config(env.experiment_config, env, dist_config)
    timeline.mark("user code imported")
    controller_cls = trial_class.trial_controller_class
    assert controller_cls is not None, f"{trial_class.__name__} has no trial_controller_class"
    controller_cls.pre_execute_hook(env, dist_config)
    timeline.mark("pre_execute_hook (device init)")
    rank = rank_info or RankInfo.from_env()
    context = trial_class.trial_context_class(env, dist_config, rank)
    logging.info("constructing %s (rank %d/%d)", trial_class.__name__, rank.rank, rank.size)
    trial_inst = trial_class(context)
    timeline.mark("trial constructed")
    ctrl = controller_cls.from_trial(trial_inst, context, env, workloads, load_path, rendezvous, dist_config)
    timeline.mark("controller ready")
    return ctrl
