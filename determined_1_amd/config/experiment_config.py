"""Experiment config schema: defaults, merge and validation.

Defaults follow ``master/pkg/model/defaults.go:33-128``; searcher-union defaults are applied for
the method named in ``searcher.name`` only (the Go union fills the selected arm).  Validation
follows the ``Validate()`` methods of ``experiment_config.go:50-118``, ``searcher_config.go``,
``hyperparameters_config.go`` and ``storage_config.go``.  Unknown top-level keys are rejected
(the master decodes with ``DisallowUnknownFields``).
"""
import copy
import time
from typing import Any, Dict, List, Optional, cast

from determined_1_amd.config.length import EPOCHS, Length

MAX_ALLOWED_TRIALS = 2000
ADAPTIVE_MODES = ("aggressive", "standard", "conservative")

TOP_LEVEL_KEYS = {
    "description", "labels", "data", "checkpoint_storage", "tensorboard_storage",
    "perform_initial_validation", "min_checkpoint_period", "min_validation_period",
    "checkpoint_policy", "hyperparameters", "searcher", "resources", "optimizations",
    "records_per_epoch", "scheduling_unit", "bind_mounts", "environment", "reproducibility",
    "max_restarts", "security", "debug", "internal", "entrypoint", "data_layer",
    # accepted for compatibility with older configs
    "batches_per_step",
}

_SEARCHER_DEFAULTS = {
    "single": {},
    "random": {},
    "grid": {},
    "sync_halving": {"divisor": 4, "train_stragglers": True},
    "adaptive": {"divisor": 4, "train_stragglers": True, "mode": "standard", "max_rungs": 5},
    "adaptive_simple": {"divisor": 4, "mode": "standard", "max_rungs": 5},
    "async_halving": {"divisor": 4, "max_concurrent_trials": 0},
    "adaptive_asha": {"divisor": 4, "mode": "standard", "max_rungs": 5, "max_concurrent_trials": 0},
    "pbt": {},
}

_LENGTH_FIELDS = ("max_length", "budget", "length_per_round")
# replaced wholesale on merge: free-form dicts and Length unions ({"batches": n} vs {"epochs": n})
_ATOMIC_KEYS = ("hyperparameters", "data", "min_validation_period", "min_checkpoint_period") + _LENGTH_FIELDS


def default_experiment_config(experiment_seed: Optional[int] = None) -> Dict[str, Any]:
    return {
        "description": "Experiment",
        "checkpoint_storage": {
            "type": "shared_fs",
            "host_path": "/tmp",
            "save_experiment_best": 0,
            "save_trial_best": 1,
            "save_trial_latest": 1,
        },
        "checkpoint_policy": "best",
        "data_layer": {"type": "shared_fs"},
        "hyperparameters": {},
        "searcher": {"smaller_is_better": True},
        "resources": {"slots_per_trial": 1, "weight": 1, "native_parallel": False, "agent_label": "",
                      "resource_pool": ""},
        "optimizations": {
            "aggregation_frequency": 1,
            "average_aggregated_gradients": True,
            "average_training_metrics": False,
            "gradient_compression": False,
            "mixed_precision": "O0",
            "tensor_fusion_threshold": 64,
            "tensor_fusion_cycle_time": 5,
            "auto_tune_tensor_fusion": False,
            "grad_reduction": "fp32_accum",
            "rccl": {},
            "hip_graph": False,
            "hip_graph_batches": 1,
        },
        "perform_initial_validation": False,
        "min_checkpoint_period": {"batches": 0},
        "min_validation_period": {"batches": 0},
        "records_per_epoch": 0,
        "scheduling_unit": 100,
        "environment": {"image": {"cpu": "determined-mi355x:cpu", "gpu": "determined-mi355x:rocm"}},
        "reproducibility": {
            "experiment_seed": int(time.time()) & 0xFFFFFFFF if experiment_seed is None else int(experiment_seed)
        },
        "max_restarts": 5,
        "debug": False,
        "internal": None,
        "entrypoint": "",
    }


def _deep_merge(base: Dict[str, Any], over: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(base)
    for k, v in over.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict) and k not in _ATOMIC_KEYS:
            # tagged unions: a different "type"/"name" replaces the arm wholesale
            tag = "type" if "type" in v or "type" in out[k] else ("name" if "name" in v else None)
            if tag and tag in v and out[k].get(tag) not in (None, v[tag]):
                keep = {kk: vv for kk, vv in out[k].items()
                        if kk.startswith("save_") or kk in ("smaller_is_better",)}
                out[k] = {**keep, **copy.deepcopy(v)}
            else:
                out[k] = _deep_merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def merge_with_defaults(user: Dict[str, Any], defaults: Optional[Dict[str, Any]] = None,
                        template: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    """defaults -> template -> user (reference merge order, core_experiment.go:355-416)."""
    cfg = copy.deepcopy(defaults if defaults is not None else default_experiment_config())
    if template:
        cfg = _deep_merge(cfg, template)
    cfg = _deep_merge(cfg, user)
    s = cfg.setdefault("searcher", {})
    name = s.get("name")
    if name in _SEARCHER_DEFAULTS:
        for k, v in _SEARCHER_DEFAULTS[name].items():
            s.setdefault(k, v)
    s.setdefault("smaller_is_better", True)
    return cfg


def _length_err(v: Any, what: str, errs: List[str]) -> Optional[Length]:
    try:
        return Length.parse(v)
    except (ValueError, TypeError):
        errs.append(f"{what}: invalid length {v!r}")
        return None


def _validate_hparams(hps: Dict[str, Any], errs: List[str], grid: bool) -> int:
    n = 1
    missing = []
    for name, hp in hps.items():
        if not isinstance(hp, dict) or "type" not in hp:
            continue  # bare values are treated as const
        t = hp["type"]
        if t == "const":
            if "val" not in hp:
                errs.append(f"hyperparameters.{name}: const needs val")
        elif t in ("int", "double", "log"):
            if not hp.get("maxval", 0) > hp.get("minval", 0):
                errs.append(f"hyperparameters.{name}: minval is greater than maxval")
            if t == "log" and not hp.get("base", 0) > 0:
                errs.append(f"hyperparameters.{name}: base must be >= 0")
            cnt = hp.get("count")
            if cnt is not None and cnt <= 0:
                errs.append(f"hyperparameters.{name}: count must be >= 0")
            if grid:
                if cnt is None:
                    missing.append(name)
                elif t == "int" and cnt > hp["maxval"] - hp["minval"]:
                    n *= hp["maxval"] - hp["minval"]
                else:
                    n *= cnt
        elif t == "categorical":
            vals = hp.get("vals", [])
            if not vals:
                errs.append(f"hyperparameters.{name}: must have at least one category")
            n *= max(1, len(vals))
        else:
            errs.append(f"hyperparameters.{name}: unknown type {t!r}")
    if grid and missing:
        errs.append("these hyperparameters must specify counts for grid search: " + ", ".join(missing))
    return n


def _is_number(v: Any) -> bool:
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def _validate_global_batch_size(hps: Dict[str, Any], errs: List[str]) -> None:
    """reference master/pkg/model/hyperparameters_config.go:20-44."""
    if "global_batch_size" not in hps:
        errs.append("global_batch_size hyperparameter must be specified")
        return
    b = hps["global_batch_size"]
    if isinstance(b, dict) and b.get("type") == "categorical":
        vals = b.get("vals", [])
    elif isinstance(b, dict) and b.get("type") == "const":
        vals = [b.get("val")]
    elif isinstance(b, dict):
        vals = []  # ranged types are numeric by construction
    else:
        vals = [b]
    if not all(_is_number(v) for v in vals):
        errs.append("global_batch_size hyperparameter must be a numeric value")


def validate_experiment_config(cfg: Dict[str, Any], require_entrypoint: bool = True) -> List[str]:
    errs = []  # type: List[str]
    unknown = set(cfg) - TOP_LEVEL_KEYS
    if unknown:
        errs.append(f"unknown config keys: {sorted(unknown)}")
    native = bool(cfg.get("internal") and cfg["internal"].get("native"))
    if require_entrypoint and not native and not cfg.get("entrypoint"):
        errs.append("Must specify an entrypoint that references the trial class.")
    s = cfg.get("searcher", {})
    name = s.get("name")
    if name not in _SEARCHER_DEFAULTS:
        errs.append(f"searcher.name: unknown searcher {name!r}")
    if not s.get("metric"):
        errs.append("searcher.metric must be set")
    units = set()
    for f in _LENGTH_FIELDS:
        if f in s:
            ln = _length_err(s[f], f"searcher.{f}", errs)
            if ln is not None:
                units.add(ln.unit)
                if ln.units <= 0:
                    errs.append(f"{f} must be > 0")
    if name in ("random", "async_halving", "adaptive_simple", "adaptive_asha"):
        if not s.get("max_trials", 0) > 0:
            errs.append("max_trials must be > 0")
    if name in ("sync_halving", "async_halving", "adaptive", "adaptive_simple", "adaptive_asha"):
        if not float(s.get("divisor", 0)) > 1.0:
            errs.append("divisor must be > 1.0")
    if name in ("sync_halving", "async_halving") and not s.get("num_rungs", 0) > 0:
        errs.append("num_rungs must be > 0")
    if name in ("adaptive", "adaptive_simple", "adaptive_asha"):
        if s.get("mode") not in ADAPTIVE_MODES:
            errs.append(f"mode must be one of {ADAPTIVE_MODES}")
        if not s.get("max_rungs", 0) > 0:
            errs.append("max_rungs must be > 0")
    if name in ("async_halving", "adaptive_asha") and s.get("max_concurrent_trials", 0) < 0:
        errs.append("max_concurrent_trials must be >= 0")
    if name in ("adaptive", "sync_halving") and "budget" in s and "max_length" in s:
        try:
            b, m = Length.parse(s["budget"]), Length.parse(s["max_length"])
            if b.unit != m.unit:
                errs.append("max_length and budget must be specified in terms of the same unit")
            elif name == "adaptive" and not b.units > m.units:
                errs.append("budget must be greater than max_length")
        except ValueError:
            pass
    if name == "adaptive_simple" and s.get("max_trials", 0) > MAX_ALLOWED_TRIALS:
        errs.append(f"max_trials must be <= {MAX_ALLOWED_TRIALS}")
    if name == "pbt":
        if not s.get("population_size", 0) > 0:
            errs.append("population_size must be > 0")
        if not s.get("num_rounds", 0) > 0:
            errs.append("num_rounds must be > 0")
        rf = s.get("replace_function", {})
        tf = rf.get("truncate_fraction", 0.0)
        if not 0.0 <= tf <= 0.5:
            errs.append("truncate_fraction must be in [0, 0.5]")
        ef = s.get("explore_function", {})
        if not 0.0 <= ef.get("resample_probability", 0.0) <= 1.0:
            errs.append("resample_probability must be in [0, 1]")
        if not 0.0 <= ef.get("perturb_factor", 0.0) <= 1.0:
            errs.append("perturb_factor must be in [0, 1]")
    for f in ("min_validation_period", "min_checkpoint_period"):
        if f in cfg:
            ln = _length_err(cfg[f], f, errs)
            if ln is not None:
                units.add(ln.unit)
    if EPOCHS in units and not cfg.get("records_per_epoch", 0) > 0:
        errs.append("Must specify records_per_epoch when any configuration is in terms of epochs")
    hps = cfg.get("hyperparameters", {}) or {}
    _validate_global_batch_size(hps, errs)
    n_grid = _validate_hparams(hps, errs, grid=(name == "grid"))
    if name == "grid" and n_grid > MAX_ALLOWED_TRIALS:
        errs.append(f"number of trials for grid search must be <= {MAX_ALLOWED_TRIALS}")
    if cfg.get("max_restarts", 0) < 0:
        errs.append("max_restarts must be >= 0")
    cs = cfg.get("checkpoint_storage", {}) or {}
    for k in ("save_experiment_best", "save_trial_best", "save_trial_latest"):
        if cs.get(k, 0) < 0:
            errs.append(f"{k} must be >= 0")
    if cfg.get("checkpoint_policy", "best") not in ("best", "all", "none"):
        errs.append("checkpoint_policy must be one of best, all, none")
    if (cfg.get("resources", {}) or {}).get("slots_per_trial", 1) < 0:
        errs.append("slots_per_trial must be >= 0")
    if (cfg.get("optimizations", {}) or {}).get("aggregation_frequency", 1) < 1:
        errs.append("aggregation_frequency must be >= 1")
    if cfg.get("scheduling_unit", 100) <= 0:
        errs.append("scheduling_unit must be > 0")
    if cs.get("type") not in (None, "shared_fs", "s3", "gcs", "hdfs"):
        errs.append(f"checkpoint_storage.type: unknown {cs.get('type')!r}")
    if cfg.get("checkpoint_policy", "best") not in ("best", "all", "none"):
        errs.append("checkpoint_policy must be one of best, all, none")
    res = cfg.get("resources", {})
    if res.get("slots_per_trial", 1) < 0:
        errs.append("slots_per_trial must be >= 0")
    opt = cfg.get("optimizations", {})
    if opt.get("aggregation_frequency", 1) < 1:
        errs.append("aggregation_frequency must be >= 1")
    hgb = opt.get("hip_graph_batches", 1)
    if not isinstance(hgb, int) or isinstance(hgb, bool) or hgb < 1:
        errs.append("optimizations.hip_graph_batches must be an integer >= 1")
    if opt.get("grad_reduction", "fp32_accum") not in ("fp32_accum", "allreduce", "auto"):
        errs.append("optimizations.grad_reduction must be fp32_accum, allreduce or auto")
    if not isinstance(opt.get("rccl", {}) or {}, dict):
        errs.append("optimizations.rccl must be a mapping")
    if opt.get("mixed_precision", "O0") not in ("O0", "O1", "O2", "O3"):
        errs.append("mixed_precision must be one of O0, O1, O2, O3")
    if cfg.get("scheduling_unit", 100) <= 0:
        errs.append("scheduling_unit must be > 0")
    return errs


class ExperimentConfig(dict):
    """Dict view of the (already defaulted) experiment config with typed accessors
    (reference ``harness/determined/_experiment_config.py``)."""

    def debug_enabled(self) -> bool:
        return bool(self.get("debug", False))

    def dtrain_optional_args(self) -> List[str]:
        return cast(List[str], (self.get("data") or {}).get("__det_dtrain_args", []))

    # reference name, kept for user code that calls it
    horovod_optional_args = dtrain_optional_args

    def scheduling_unit(self) -> int:
        return int(self.get("scheduling_unit", 100))

    def native_enabled(self) -> bool:
        return bool(self.get("internal")) and "native" in self["internal"]

    def native_parallel_enabled(self) -> bool:
        return bool(self.get("resources", {}).get("native_parallel", False))

    def mixed_precision_enabled(self) -> bool:
        return self.get("optimizations", {}).get("mixed_precision", "O0") != "O0"

    def averaging_training_metrics_enabled(self) -> bool:
        return bool(self.get("optimizations", {}).get("average_training_metrics", False))

    def slots_per_trial(self) -> int:
        return int(self.get("resources", {}).get("slots_per_trial", 1))

    def experiment_seed(self) -> int:
        return int(self.get("reproducibility", {}).get("experiment_seed", 0))

    def get_data_layer_type(self) -> str:
        return cast(str, self.get("data_layer", {}).get("type", "shared_fs"))

    def get_records_per_epoch(self) -> Optional[int]:
        r = self.get("records_per_epoch")
        return int(r) if r else None

    def get_min_validation_period(self) -> Dict[str, Any]:
        return cast(Dict[str, Any], self.get("min_validation_period", {}))

    def get_min_checkpoint_period(self) -> Dict[str, Any]:
        return cast(Dict[str, Any], self.get("min_checkpoint_period", {}))

    def get_optimizations(self) -> Dict[str, Any]:
        return cast(Dict[str, Any], self.get("optimizations", {}))

    def profiling_enabled(self) -> bool:
        return bool((self.get("data") or {}).get("__det_profile", False))
