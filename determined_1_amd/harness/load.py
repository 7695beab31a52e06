"""Load the user's Trial class and build its controller (reference ``load/_load_implementation.py``
and ``load/_load_trial_controller.py:10-143``)."""
import importlib
import logging
import os
import pathlib
import sys
from typing import Any, Optional, Type

from determined_1_amd import trial, workload
from determined_1_amd.env import EnvContext, RendezvousInfo
from determined_1_amd.parallel.dist import DistributedConfig, RankInfo


def notebook_to_py(ipynb: pathlib.Path) -> pathlib.Path:
    """Convert a Jupyter notebook's code cells into ``<name>.py`` next to it (reference
    ``load/_load_implementation.py:147``); magics and shell escapes are commented out."""
    import json

    nb = json.loads(ipynb.read_text())
    lines = []
    for cell in nb.get("cells", []):
        if cell.get("cell_type") != "code":
            continue
        src = cell.get("source", [])
        text = "".join(src) if isinstance(src, list) else str(src)
        for ln in text.splitlines():
            lines.append(("# " + ln) if ln.lstrip().startswith(("%", "!")) else ln)
        lines.append("")
    out = ipynb.with_suffix(".py")
    out.write_text("\n".join(lines))
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


def prepare_controller(env: EnvContext, workloads: workload.Stream, load_path: Optional[pathlib.Path],
                       rendezvous: RendezvousInfo, dist_config: DistributedConfig,
                       rank_info: Optional[RankInfo] = None) -> trial.TrialController:
    """pre_execute_hook -> context -> Trial(context) -> controller.from_trial (reference
    ``load_controller_from_trial``)."""
    from determined_1_amd.harness import timeline

    trial_class = load_trial_class(env.experiment_config["entrypoint"])
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
