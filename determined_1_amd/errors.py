"""Exception types of the harness (reference: harness/determined/errors.py:4-63)."""


class InternalException(Exception):
    """An unexpected internal error of the framework itself."""


class InvalidExperimentException(Exception):
    """The experiment configuration or trial definition is invalid."""


class InvalidConfigurationException(InvalidExperimentException):
    def __init__(self, errors):
        self.errors = list(errors) if not isinstance(errors, str) else [errors]
        super().__init__("invalid experiment configuration:\n  " + "\n  ".join(map(str, self.errors)))


class InvalidHP(Exception):
    """Raised by user code to signal that the sampled hyperparameters are invalid
    (the trial exits with ``exited_reason: INVALID_HP``)."""


class SkipWorkloadException(Exception):
    pass


class WorkerError(Exception):
    """A training rank failed; raised on the chief."""


class CheckpointNotFoundException(Exception):
    pass


class StopLoadingImplementation(Exception):
    """Raised by ``init()`` to stop executing a native-API user script once its trial is captured."""


class TrialStopped(Exception):
    pass


class StorageError(Exception):
    pass
