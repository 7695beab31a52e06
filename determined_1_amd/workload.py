"""The master<->harness workload protocol (SURVEY §2.6 C-ws / C-done).

A trial process consumes a *stream* of ``(Workload, args, respond)`` triples.  Each layer of the
harness (socket manager -> workload manager -> [rank fan-out] -> trial controller) is a generator
that wraps the stream of the layer above it and may intercept ``respond``.  The protocol is
strictly synchronous: exactly one response per workload, in order.

Reference behaviour: ``harness/determined/workload.py:9-236`` (Kind enum values, JSON shape,
``Skipped`` for non-chief ranks, the response interceptor used by tests).
"""
import enum
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple, Union


class Workload:
    class Kind(enum.Enum):
        RUN_STEP = 1
        COMPUTE_VALIDATION_METRICS = 2
        CHECKPOINT_MODEL = 3
        TERMINATE = 4

    __slots__ = ("kind", "experiment_id", "trial_id", "step_id", "num_batches", "total_batches_processed")

    def __init__(self, kind: "Workload.Kind", e_id: int, t_id: int, s_id: int, num_batches: int,
                 total_batches_processed: int) -> None:
        self.kind = kind
        self.experiment_id = e_id
        self.trial_id = t_id
        self.step_id = s_id
        self.num_batches = num_batches
        self.total_batches_processed = total_batches_processed

    def _key(self) -> Tuple:
        return (self.kind, self.experiment_id, self.trial_id, self.step_id, self.num_batches,
                self.total_batches_processed)

    def __eq__(self, other: object) -> bool:
        return isinstance(other, Workload) and self._key() == other._key()

    def __hash__(self) -> int:
        return hash(self._key()[:4])

    def __repr__(self) -> str:
        nb = f" ({self.num_batches} Batches)" if self.kind == Workload.Kind.RUN_STEP else ""
        return f"<{self.kind.name}{nb}: ({self.experiment_id},{self.trial_id},{self.step_id})>"

    def __json__(self) -> Dict[str, Any]:
        return {
            "kind": self.kind.name,
            "experiment_id": self.experiment_id,
            "trial_id": self.trial_id,
            "step_id": self.step_id,
            "num_batches": self.num_batches,
            "total_batches_processed": self.total_batches_processed,
        }

    @staticmethod
    def from_json(d: Dict[str, Any]) -> "Workload":
        kind = d["kind"]
        if kind not in Workload.Kind.__members__:
            raise ValueError(f"unknown workload kind {kind!r}")
        return Workload(Workload.Kind[kind], int(d["experiment_id"]), int(d["trial_id"]), int(d["step_id"]),
                        int(d["num_batches"]), int(d["total_batches_processed"]))


Metrics = Dict[str, Any]


class Skipped:
    """Response of a rank/layer that does not report for this workload (non-chief ranks)."""

    def __repr__(self) -> str:
        return "Skipped()"

    def __eq__(self, other: object) -> bool:
        return isinstance(other, Skipped)

    def __hash__(self) -> int:
        return 0


Response = Union[Metrics, Skipped]
ResponseFunc = Callable[[Response], None]
Args = List[Any]
Stream = Iterator[Tuple[Workload, Args, ResponseFunc]]


class Source:
    """A harness layer that produces a workload stream."""

    def __iter__(self) -> Stream:  # pragma: no cover - interface
        raise NotImplementedError


class WorkloadResponseInterceptor:
    """Wrap a stream to capture the response of each workload (test utility and local mode)."""

    def __init__(self) -> None:
        self._response = None  # type: Optional[Response]

    def send(self, w: Workload, args: Args) -> Stream:
        self._response = None

        def _respond(r: Response) -> None:
            self._response = r

        yield w, args, _respond

    def result(self) -> Response:
        if self._response is None:
            raise AssertionError("workload was not responded to")
        return self._response


def ignore_response(_: Response) -> None:
    pass


def train_workload(step_id: int, exp_id: int = 1, trial_id: int = 1, num_batches: int = 1,
                   total_batches_processed: int = 0) -> Workload:
    return Workload(Workload.Kind.RUN_STEP, exp_id, trial_id, step_id, num_batches, total_batches_processed)


def validation_workload(step_id: int = 1, exp_id: int = 1, trial_id: int = 1,
                        total_batches_processed: int = 0) -> Workload:
    return Workload(Workload.Kind.COMPUTE_VALIDATION_METRICS, exp_id, trial_id, step_id, 0, total_batches_processed)


def checkpoint_workload(step_id: int = 1, exp_id: int = 1, trial_id: int = 1,
                        total_batches_processed: int = 0) -> Workload:
    return Workload(Workload.Kind.CHECKPOINT_MODEL, exp_id, trial_id, step_id, 0, total_batches_processed)


def terminate_workload(step_id: int = 1, exp_id: int = 1, trial_id: int = 1,
                       total_batches_processed: int = 0) -> Workload:
    return Workload(Workload.Kind.TERMINATE, exp_id, trial_id, step_id, 0, total_batches_processed)


def stream_from_list(items: List[Tuple[Workload, Args, ResponseFunc]]) -> Stream:
    yield from items
