"""Local (no-master) execution: synthetic env, controller construction, synthetic workloads.

Reference: ``harness/determined/experimental/_native.py:88-254`` (test mode workloads: 1 train step
of ``scheduling_unit`` batches, validation, checkpoint, terminate) and
``harness/determined/_execution.py:63-160`` (local execution env/managers).  Also the unit-test
harness of the reference (``harness/tests/experiment/utils.py:101-160``) builds controllers the
same way, so tests, local mode, ``bench.py`` and the cluster entrypoint share this code path.
"""
import copy
import json
import os
import pathlib
import tempfile
import uuid
from typing import Any, Dict, Iterator, List, Optional, Tuple, Type

from determined_1_amd import constants, trial, workload
from determined_1_amd.config import merge_with_defaults
from determined_1_amd.env import EnvContext, RendezvousInfo
from determined_1_amd.parallel.dist import DistributedConfig, RankInfo


def _local_defaults(config: Dict[str, Any]) -> Dict[str, Any]:
    cfg = merge_with_defaults(copy.deepcopy(config))
    for k, v in constants.DEFAULT_EXP_CFG.items():
        if isinstance(v, dict):
            for kk, vv in v.items():
                cfg.setdefault(k, {}).setdefault(kk, vv)
        else:
            cfg.setdefault(k, v)
    cfg["searcher"].setdefault("name", "single")
    cfg["searcher"].setdefault("max_length", {"batches": 100})
    cfg["searcher"].setdefault("metric", "validation_loss")
    return cfg


def sample_hparams(hparams_cfg: Dict[str, Any]) -> Dict[str, Any]:
    """Const values, or a deterministic pick (min / first category) for searchable params."""
    out = {}
    for name, hp in (hparams_cfg or {}).items():
        if not isinstance(hp, dict) or "type" not in hp:
            out[name] = hp
            continue
        t = hp["type"]
        if t == "const":
            out[name] = hp["val"]
        elif t == "int":
            out[name] = int(hp["minval"])
        elif t == "double":
            out[name] = float(hp["minval"])
        elif t == "log":
            out[name] = float(hp.get("base", 10.0)) ** float(hp["minval"])
        elif t == "categorical":
            out[name] = hp["vals"][0]
    return out


def make_local_env(
    config: Dict[str, Any],
    hparams: Optional[Dict[str, Any]] = None,
    managed_training: bool = True,
    initial_workload: Optional[workload.Workload] = None,
    use_gpu: Optional[bool] = None,
    trial_seed: int = 0,
    rank_info: Optional[RankInfo] = None,
    test_mode: bool = False,
) -> Tuple[EnvContext, DistributedConfig, RankInfo]:
    import torch

    cfg = _local_defaults(config)
    if hparams is None:
        hparams = sample_hparams(cfg.get("hyperparameters", {}))
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    rank = rank_info or RankInfo.from_env()
    gpus = [str(rank.local_rank)] if use_gpu else []
    env = EnvContext(
        master_addr="",
        master_port=0,
        use_tls=False,
        master_cert_file=None,
        master_cert_name=None,
        container_id="local",
        experiment_config=cfg,
        hparams=hparams,
        initial_workload=initial_workload or workload.train_workload(1, 1, 1, cfg.get("scheduling_unit", 100)),
        latest_checkpoint=None,
        use_gpu=use_gpu,
        container_gpus=gpus,
        slot_ids=[rank.local_rank] if use_gpu else [],
        debug=bool(cfg.get("debug", False)),
        workload_manager_type="TRIAL_WORKLOAD_MANAGER",
        det_rendezvous_ports="",
        det_trial_unique_port_offset=0,
        det_trial_runner_network_interface=constants.AUTO_DETECT_TRIAL_RUNNER_NETWORK_INTERFACE,
        det_trial_id="1",
        det_experiment_id="1",
        det_cluster_id="local",
        trial_seed=trial_seed,
        managed_training=managed_training,
        test_mode=test_mode,
    )
    dist_cfg = DistributedConfig.from_configs(cfg, world_size=rank.size, num_agents=rank.cross_size)
    if rank.size <= 1 and os.environ.get("DET_FORCE_DISTRIBUTED", "0") != "1":
        dist_cfg.use = False
    return env, dist_cfg, rank


def make_controller(
    trial_class: Type[trial.Trial],
    config: Dict[str, Any],
    workloads: workload.Stream,
    hparams: Optional[Dict[str, Any]] = None,
    load_path: Optional[pathlib.Path] = None,
    trial_seed: int = 0,
    initial_workload: Optional[workload.Workload] = None,
    use_gpu: Optional[bool] = None,
    rank_info: Optional[RankInfo] = None,
) -> trial.TrialController:
    """Build env + context + user trial + controller, exactly as a cluster trial process does."""
    env, dist_cfg, rank = make_local_env(config, hparams, initial_workload=initial_workload, use_gpu=use_gpu,
                                         trial_seed=trial_seed, rank_info=rank_info)
    controller_cls = trial_class.trial_controller_class
    assert controller_cls is not None, f"{trial_class.__name__} has no trial_controller_class"
    controller_cls.pre_execute_hook(env, dist_cfg)
    context = trial_class.trial_context_class(env, dist_cfg, rank)
    trial_inst = trial_class(context)
    rendezvous = RendezvousInfo([f"127.0.0.1:{constants.LOCAL_RENDEZVOUS_PORT}"] * max(1, rank.cross_size),
                                [f"127.0.0.1:{constants.LOCAL_RENDEZVOUS_PORT + 1}"] * max(1, rank.cross_size),
                                rank.cross_rank)
    return controller_cls.from_trial(trial_inst, context, env, workloads, load_path, rendezvous, dist_cfg)


def make_test_workloads(checkpoint_dir: pathlib.Path, scheduling_unit: int = 1) -> workload.Stream:
    """Test-mode stream (reference _native.py:88-111): train, validate, checkpoint, terminate."""
    interceptor = workload.WorkloadResponseInterceptor()
    yield from interceptor.send(workload.train_workload(1, num_batches=scheduling_unit), [])
    yield from interceptor.send(workload.validation_workload(1, total_batches_processed=scheduling_unit), [])
    yield from interceptor.send(workload.checkpoint_workload(1, total_batches_processed=scheduling_unit),
                                [checkpoint_dir])
    yield workload.terminate_workload(1, total_batches_processed=scheduling_unit), [], workload.ignore_response


def test_one_batch(trial_class: Type[trial.Trial], config: Optional[Dict[str, Any]] = None,
                   hparams: Optional[Dict[str, Any]] = None) -> trial.TrialController:
    """Run the test-mode sequence on one batch locally (reference ``_native.py:189``)."""
    cfg = dict(config or {})
    cfg["scheduling_unit"] = 1
    with tempfile.TemporaryDirectory() as td:
        ckpt = pathlib.Path(td).joinpath(str(uuid.uuid4()))
        ctrl = make_controller(trial_class, cfg, make_test_workloads(ckpt, 1), hparams=hparams)
        ctrl.run()
    return ctrl


def run_local_test(config: Dict[str, Any], model_dir: str) -> trial.TrialController:
    """``det experiment create --local --test``: load the trial from ``model_dir`` and run the
    test-mode workload sequence in this process."""
    from determined_1_amd.harness.load import load_trial_class

    cls = load_trial_class(config["entrypoint"], model_dir)
    return test_one_batch(cls, config)


def dump_env(env: EnvContext) -> Dict[str, str]:
    """Inverse of ``EnvContext.from_environ`` (used by the agent/launcher to spawn ranks)."""
    return {
        "DET_MASTER_ADDR": env.master_addr,
        "DET_MASTER_PORT": str(env.master_port),
        "DET_CONTAINER_ID": env.container_id,
        "DET_EXPERIMENT_ID": env.det_experiment_id,
        "DET_TRIAL_ID": env.det_trial_id,
        "DET_TRIAL_SEED": str(env.trial_seed),
        "DET_EXPERIMENT_CONFIG": json.dumps(dict(env.experiment_config)),
        "DET_HPARAMS": json.dumps(env.hparams),
        "DET_INITIAL_WORKLOAD": json.dumps(env.initial_workload.__json__()),
        "DET_LATEST_CHECKPOINT": "",
        "DET_WORKLOAD_MANAGER_TYPE": env.workload_manager_type,
        "DET_RENDEZVOUS_PORTS": env.det_rendezvous_ports,
        "DET_TRIAL_RUNNER_NETWORK_INTERFACE": env.det_trial_runner_network_interface,
        "DET_USE_GPU": "true" if env.use_gpu else "false",
        "DET_SLOT_IDS": json.dumps(env.slot_ids),
        "DET_AGENT_ID": os.environ.get("DET_AGENT_ID", "local"),
    }


def list_of_workloads(items: List[Tuple[workload.Workload, List[Any]]]) -> Iterator:
    for w, args in items:
        yield w, args, workload.ignore_response


def load_model_def(model_dir: str, name: str = "model_def") -> Any:
    """Import ``<model_dir>/<name>.py`` as a uniquely named module (so several example directories,
    each with its own ``model_def.py``, can be loaded in one process) with ``model_dir`` on
    ``sys.path`` for its sibling imports.  Used by bench.py and the benchmark scripts to run the
    examples' Trial classes -- the same user code an experiment's checkpoint ``code/`` holds."""
    import hashlib
    import importlib.util
    import os
    import sys

    path = os.path.join(os.path.abspath(model_dir), name + ".py")
    modname = "det_model_def_" + hashlib.sha1(path.encode()).hexdigest()[:12]
    if modname in sys.modules:
        return sys.modules[modname]
    from determined_1_amd.harness.load import isolate_model_dir

    isolate_model_dir(os.path.dirname(path))
    spec = importlib.util.spec_from_file_location(modname, path)
    assert spec is not None and spec.loader is not None, path
    mod = importlib.util.module_from_spec(spec)
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod
