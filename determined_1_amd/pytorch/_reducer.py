"""Validation-metric reducers (reference ``harness/determined/pytorch/_reducer.py``).

AVG across processes is weighted by each process's batch count, so a rank that saw a partial
last shard does not skew the mean.
"""
import enum
from typing import List, Optional

import numpy as np


class Reducer(enum.Enum):
    AVG = 1
    SUM = 2
    MAX = 3
    MIN = 4


def _reduce_metrics(reducer: Reducer, metrics: np.ndarray, num_batches: Optional[List[int]] = None) -> float:
    if reducer == Reducer.AVG:
        if num_batches:
            if len(metrics) != len(num_batches):
                raise ValueError("metrics and num_batches lengths differ")
        return np.average(metrics, weights=num_batches, axis=0)
    if reducer == Reducer.SUM:
        return np.sum(metrics, axis=0)
    if reducer == Reducer.MAX:
        return np.max(metrics, axis=0)
    if reducer == Reducer.MIN:
        return np.min(metrics, axis=0)
    raise NotImplementedError(reducer)
