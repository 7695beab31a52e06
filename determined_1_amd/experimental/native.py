"""Native API (reference ``experimental/_native.py:254-340``):

    det.experimental.create(MyTrial, config, local=True, test=True)   # one batch, in-process
    det.experimental.create(MyTrial, config, local=True)              # full single-trial run, in-process
    det.experimental.create(MyTrial, config, context_dir=".", master_url="host:8080")  # cluster

Cluster mode works like the reference's (``experimental/_native.py:21-68,114-165``): the submitting
script records itself as ``internal.native.command = [script relative to context_dir, *argv]`` (a
notebook passes ``command=["nb.ipynb"]``), and every trial process re-runs that command under the
harness loader (``harness/load.py`` ``RunpyGlobals``).  There ``create()`` hands ``trial_def`` back and
raises ``StopLoadingImplementation`` instead of submitting again, so a script with a top-level
``create()`` call and no ``__main__`` guard yields exactly one experiment.
"""
import logging
import os
import pathlib
import sys
import tempfile
import uuid
from typing import Any, Dict, Iterator, List, Optional, Type

from determined_1_amd import errors, trial, workload
from determined_1_amd.config import merge_with_defaults
from determined_1_amd.config.length import BATCHES, Length, UnitContext
from determined_1_amd.experimental._local import make_controller, test_one_batch


def _set_command_default(context_dir: str, command: Optional[List[str]]) -> List[str]:
    """``[script relative to context_dir, *sys.argv[1:]]`` unless the caller gave a command."""
    if command:
        cmd = [str(c) for c in command]
        if not cmd[0].endswith((".py", ".ipynb")):
            raise errors.InvalidExperimentException(f"command must start with a .py or .ipynb file, got {cmd}")
        return cmd
    import __main__

    main_file = getattr(__main__, "__file__", None)
    if not main_file:  # a notebook / REPL: there is no script to re-run
        raise errors.InvalidExperimentException(
            "Must specify the location of the notebook file relative to the context directory "
            "(command=[\"notebook.ipynb\"]) when not running a script.")
    try:
        rel = pathlib.Path(main_file).resolve().relative_to(pathlib.Path(context_dir).resolve())
    except ValueError:
        raise errors.InvalidExperimentException(
            f"the submitting script {main_file} is not inside context_dir {context_dir}") from None
    if rel.suffix not in (".py", ".ipynb"):
        raise errors.InvalidExperimentException(f"command must start with a .py or .ipynb file, got {rel}")
    return [str(rel), *sys.argv[1:]]


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
           test: bool = False, context_dir: str = "", command: Optional[List[str]] = None,
           master_url: Optional[str] = None, checkpoint_dir: Optional[str] = None, follow: bool = False) -> Any:
    """Create an experiment from ``trial_def`` (reference ``experimental/_native.py:254-340``).

    Inside a trial process (the harness re-running this script) it returns nothing: it hands the
    class to the loader and stops the script.  ``follow`` waits for the cluster experiment to end,
    printing trial logs, like the reference's ``create_experiment_and_follow_logs``.
    """
    from determined_1_amd.harness.load import RunpyGlobals

    if RunpyGlobals.is_initialized():
        RunpyGlobals.set_runpy_trial_result(trial_def)  # raises StopLoadingImplementation
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
        raise errors.InvalidExperimentException("Cannot specify the context directory to be empty.")
    internal = dict(config.get("internal") or {})
    internal["native"] = {"command": _set_command_default(context_dir, command)}
    config["internal"] = internal
    if test:
        from determined_1_amd.cli.cli import make_test_config

        config = make_test_config(config)
    d = Determined(master_url)
    exp = d.create_experiment(config, context_dir)
    logging.info("created experiment %d (native command %s)", exp.id, internal["native"]["command"])
    if follow or test:
        from determined_1_amd.cli.cli import _follow

        state = _follow(d._client, exp.id)
        if test and state != "COMPLETED":
            raise errors.InvalidExperimentException(f"test experiment {exp.id} ended in state {state}")
    return exp
