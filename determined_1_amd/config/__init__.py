"""Experiment configuration: schema defaults, validation, ``Length`` arithmetic.

Mirrors the reference master's config model (``master/pkg/model/experiment_config.go:22-47``,
``defaults.go:33-128``, ``searcher_config.go``, ``hyperparameters_config.go:65-146``,
``length.go:13-196``) so that YAML written for the reference is accepted unchanged.  The C++
master (``native/src/config.cc``) applies the same defaults; this module is what the harness,
CLI ``--test`` mode and local/native mode use.
"""
from determined_1_amd.config.experiment_config import (
    ExperimentConfig,
    default_experiment_config,
    merge_with_defaults,
    validate_experiment_config,
)
from determined_1_amd.config.length import Length, UnitContext

__all__ = [
    "ExperimentConfig",
    "Length",
    "UnitContext",
    "default_experiment_config",
    "merge_with_defaults",
    "validate_experiment_config",
]
