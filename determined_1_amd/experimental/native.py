"""Native API (reference ``experimental/_native.py:254-340``):

    det.experimental.create(MyTrial, config, local=True, test=True)   # one batch, in-process
    det.experimental.create(MyTrial, config, local=True)              # full single-trial run, in-process
    det.experimental.create(MyTrial, config, context_dir=".", master_url="host:8080")  # cluster

The trial class is resolved to ``module:QualName`` relative to ``context_dir`` for cluster
submission, exactly like an ``entrypoint`` in a config file.
"""
import inspect
import logging
import os
import pathlib
import tempfile
import uuid
from typing import Any, Dict, Iterator, Optional, Type

from determined_1_amd import trial, workload
from determined_1_amd.config import merge_with_defaults
from determined_1_amd.config.length import BATCHES, Length, UnitContext
from determined_1_amd.experimental._local import make_controller, test_one_batch


def _entrypoint_for(trial_def: Type[trial.Trial], context_dir: str) -> str:
    mod = inspect.getmodule(trial_def)
    assert mod is not None and getattr(mod, "__file__", None), "trial class must live in a module file"
    rel = os.path.relpath(os.path.abspath(mod.__file__), os.path.abspath(context_dir))
    if rel.startswith(".."):
        raise ValueError(f"{mod.__file__} is not inside context_dir {context_dir}")
    modname = rel[:-3].replace(os.sep, ".") if rel.endswith(".py") else rel.replace(os.sep, ".")
    if modname.endswith(".__init__"):
        modname = modname[: -len(".__init__")]
    return f"{modname}:{trial_def.__qualname__}"


def local_training_workloads(cfg: Dict[str, Any], ckpt_root: pathlib.Path) -> Iterator:
    """Single-trial schedule without a master: train max_length in scheduling_unit steps, validate
    every min_validation_period (and at the end), checkpoint at the end."""
    cfg = merge_with_defaults(cfg)
    gbs = int(cfg["hyperparameters"].get("global_batch_size", 1))
    rpe = int(cfg.get("records_per_epoch", 0) or 0)
    uctx = UnitContext(BATCHES, gbs, rpe)
    total = Length.parse(cfg["searcher"]["max_length"]).to_nearest_batch(uctx)
    val_every = Length.parse(cfg.get("min_validation_period", {"batches": 0})).to_nearest_batch(uctx)
    unit = int(cfg.get("scheduling_unit", 100))
    done, step, since_val = 0, 1, 0
    while done < total:
        n = min(unit, total - done, (val_every - since_val) if val_every else unit)
        yield workload.train_workload(step, num_batches=n, total_batches_processed=done), [], workload.ignore_response
        done += n
        since_val += n
        if val_every and since_val >= val_every:
            yield workload.validation_workload(step, total_batches_processed=done), [], workload.ignore_response
            since_val = 0
        step += 1
    yield workload.validation_workload(step, total_batches_processed=done), [], workload.ignore_response
    path = ckpt_root.joinpath(str(uuid.uuid4()))
    yield workload.checkpoint_workload(step, total_batches_processed=done), [path], workload.ignore_response
    yield workload.terminate_workload(step, total_batches_processed=done), [], workload.ignore_response


def create(trial_def: Type[trial.Trial], config: Optional[Dict[str, Any]] = None, local: bool = False,
           test: bool = False, context_dir: str = "", master_url: Optional[str] = None,
           checkpoint_dir: Optional[str] = None) -> Any:
    config = dict(config or {})
    if local and test:
        return test_one_batch(trial_def, config)
    if local:
        root = pathlib.Path(checkpoint_dir or tempfile.mkdtemp(prefix="det-local-ckpt-"))
        ctrl = make_controller(trial_def, config, local_training_workloads(config, root))
        ctrl.run()
        logging.info("local training finished; checkpoints in %s", root)
        return ctrl
    from determined_1_amd.experimental.client import Determined

    if not context_dir:
        raise ValueError("cluster mode needs context_dir (the directory shipped as the model definition)")
    config.setdefault("entrypoint", _entrypoint_for(trial_def, context_dir))
    if test:
        from determined_1_amd.cli.cli import make_test_config

        config = make_test_config(config)
    exp = Determined(master_url).create_experiment(config, context_dir)
    logging.info("created experiment %d", exp.id)
    return exp
