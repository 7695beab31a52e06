"""The RPC table of the ``determined.api.v1.Determined`` service: for every method its HTTP binding
on det-master's ``/api/v1`` surface (native/src/api_v1.cc), as the ``google.api.http`` annotations
of the reference's ``api.proto`` bind them (reference ``proto/src/determined/api/v1/api.proto``).

Each entry: (method, verb, path template, body, server_streaming).  ``{a.b}`` path variables read
the request field ``a.b``; ``body`` is ``"*"`` (the whole request minus path variables), a field
name (that field only), or None (the remaining fields go to the query string)."""
from typing import List, NamedTuple, Optional

SERVICE = "determined.api.v1.Determined"


class Route(NamedTuple):
    method: str
    verb: str
    path: str
    body: Optional[str]
    stream: bool = False


def _tasks() -> List[Route]:
    out = []
    for kind, one in (("notebooks", "Notebook"), ("shells", "Shell"), ("commands", "Command"),
                      ("tensorboards", "Tensorboard")):
        key = f"{one.lower()}_id"
        out += [Route(f"Get{one}s", "GET", f"/api/v1/{kind}", None),
                Route(f"Get{one}", "GET", f"/api/v1/{kind}/{{{key}}}", None),
                Route(f"Kill{one}", "POST", f"/api/v1/{kind}/{{{key}}}/kill", None),
                Route(f"Launch{one}", "POST", f"/api/v1/{kind}", "*")]
    return out


ROUTES: List[Route] = [
    # authentication and users
    Route("Login", "POST", "/api/v1/auth/login", "*"),
    Route("CurrentUser", "GET", "/api/v1/auth/user", None),
    Route("Logout", "POST", "/api/v1/auth/logout", None),
    Route("GetUsers", "GET", "/api/v1/users", None),
    Route("GetUser", "GET", "/api/v1/users/{username}", None),
    Route("PostUser", "POST", "/api/v1/users", "*"),
    Route("SetUserPassword", "POST", "/api/v1/users/{username}/password", "password"),
    # master
    Route("GetTelemetry", "GET", "/api/v1/master/telemetry", None),
    Route("GetMaster", "GET", "/api/v1/master", None),
    Route("GetMasterConfig", "GET", "/api/v1/master/config", None),
    Route("MasterLogs", "GET", "/api/v1/master/logs", None, True),
    # agents and slots
    Route("GetAgents", "GET", "/api/v1/agents", None),
    Route("GetAgent", "GET", "/api/v1/agents/{agent_id}", None),
    Route("GetSlots", "GET", "/api/v1/agents/{agent_id}/slots", None),
    Route("GetSlot", "GET", "/api/v1/agents/{agent_id}/slots/{slot_id}", None),
    Route("EnableAgent", "POST", "/api/v1/agents/{agent_id}/enable", None),
    Route("DisableAgent", "POST", "/api/v1/agents/{agent_id}/disable", None),
    Route("EnableSlot", "POST", "/api/v1/agents/{agent_id}/slots/{slot_id}/enable", None),
    Route("DisableSlot", "POST", "/api/v1/agents/{agent_id}/slots/{slot_id}/disable", None),
    # experiments
    Route("CreateExperiment", "POST", "/api/v1/experiments", "*"),
    Route("GetExperiment", "GET", "/api/v1/experiments/{experiment_id}", None),
    Route("GetExperiments", "GET", "/api/v1/experiments", None),
    Route("GetExperimentLabels", "GET", "/api/v1/experiment/labels", None),
    Route("GetExperimentValidationHistory", "GET", "/api/v1/experiments/{experiment_id}/validation-history", None),
    Route("ActivateExperiment", "POST", "/api/v1/experiments/{id}/activate", None),
    Route("PauseExperiment", "POST", "/api/v1/experiments/{id}/pause", None),
    Route("CancelExperiment", "POST", "/api/v1/experiments/{id}/cancel", None),
    Route("KillExperiment", "POST", "/api/v1/experiments/{id}/kill", None),
    Route("ArchiveExperiment", "POST", "/api/v1/experiments/{id}/archive", None),
    Route("UnarchiveExperiment", "POST", "/api/v1/experiments/{id}/unarchive", None),
    Route("PatchExperiment", "PATCH", "/api/v1/experiments/{experiment.id}", "experiment"),
    Route("GetExperimentCheckpoints", "GET", "/api/v1/experiments/{id}/checkpoints", None),
    Route("PreviewHPSearch", "POST", "/api/v1/preview-hp-search", "*"),
    Route("GetExperimentTrials", "GET", "/api/v1/experiments/{experiment_id}/trials", None),
    # trials
    Route("GetTrial", "GET", "/api/v1/trials/{trial_id}", None),
    Route("TrialLogs", "GET", "/api/v1/trials/{trial_id}/logs", None, True),
    Route("TrialLogsFields", "GET", "/api/v1/trials/{trial_id}/logs/fields", None, True),
    Route("KillTrial", "POST", "/api/v1/trials/{id}/kill", None),
    Route("GetTrialCheckpoints", "GET", "/api/v1/trials/{id}/checkpoints", None),
    # templates
    Route("GetTemplates", "GET", "/api/v1/templates", None),
    Route("GetTemplate", "GET", "/api/v1/templates/{template_name}", None),
    Route("PutTemplate", "PUT", "/api/v1/templates/{template.name}", "template"),
    Route("DeleteTemplate", "DELETE", "/api/v1/templates/{template_name}", None),
    # notebooks, shells, commands, TensorBoards
    *_tasks(),
    Route("NotebookLogs", "GET", "/api/v1/notebooks/{notebook_id}/logs", None, True),
    # model registry and checkpoints
    Route("GetModel", "GET", "/api/v1/models/{model_name}", None),
    Route("PostModel", "POST", "/api/v1/models/{model.name}", "model"),
    Route("PatchModel", "PATCH", "/api/v1/models/{model.name}", "*"),
    Route("GetModels", "GET", "/api/v1/models", None),
    Route("GetModelVersion", "GET", "/api/v1/models/{model_name}/versions/{model_version}", None),
    Route("GetModelVersions", "GET", "/api/v1/models/{model_name}/versions", None),
    Route("PostModelVersion", "POST", "/api/v1/models/{model_name}/versions", "*"),
    Route("GetCheckpoint", "GET", "/api/v1/checkpoints/{checkpoint_uuid}", None),
    Route("PostCheckpointMetadata", "POST", "/api/v1/checkpoints/{checkpoint.uuid}/metadata", "*"),
    # metric streams
    Route("MetricNames", "GET", "/api/v1/experiments/{experiment_id}/metrics-stream/metric-names", None, True),
    Route("MetricBatches", "GET", "/api/v1/experiments/{experiment_id}/metrics-stream/batches", None, True),
    Route("TrialsSnapshot", "GET", "/api/v1/experiments/{experiment_id}/metrics-stream/trials-snapshot", None, True),
    Route("TrialsSample", "GET", "/api/v1/experiments/{experiment_id}/metrics-stream/trials-sample", None, True),
]

BY_NAME = {r.method: r for r in ROUTES}
