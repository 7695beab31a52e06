"""Python SDK (reference ``common/determined_common/experimental/``).

    d = Determined("127.0.0.1:8080")
    ckpt = d.get_experiment(3).top_checkpoint()
    model = ckpt.load(map_location="cpu")          # rebuilt from <ckpt>/code + state_dict.pth

``Checkpoint.download()`` materialises ``<dir>/<uuid>`` and writes ``metadata.json``
(``{determined_version, framework, format, experiment_id, trial_id, hparams, experiment_config,
metadata}``, reference ``_checkpoint.py:170-184``).
"""
import json
import pathlib
import shutil
import tempfile
from typing import Any, Dict, List, Optional

from determined_1_amd import __version__, storage
from determined_1_amd.api import MasterClient


class Checkpoint:
    def __init__(self, client: MasterClient, record: Dict[str, Any]) -> None:
        self._client = client
        self.record = record
        self.uuid = record["uuid"]
        self.trial_id = record.get("trial_id")
        self.experiment_id = record.get("experiment_id")
        self.step_id = record.get("step_id")
        self.resources = record.get("resources") or {}
        self.framework = record.get("framework")
        self.format = record.get("format")
        self.validation_metrics = record.get("validation_metrics")
        self.experiment_config = record.get("experiment_config")
        self.hparams = record.get("hparams")

    def _full(self) -> None:
        if self.experiment_config is None:
            full = self._client.get(f"/checkpoints/{self.uuid}")
            self.experiment_config = full.get("experiment_config")
            self.hparams = full.get("hparams")
            self.validation_metrics = full.get("validation_metrics")

    def download(self, path: Optional[str] = None) -> str:
        self._full()
        dst = pathlib.Path(path or tempfile.mkdtemp(prefix="det-ckpt-")).joinpath(self.uuid) \
            if path is None else pathlib.Path(path)
        if not dst.joinpath("metadata.json").exists():
            mgr = storage.build((self.experiment_config or {}).get("checkpoint_storage", {}))
            with mgr.restore_path(storage.StorageMetadata(self.uuid, self.resources)) as src:
                shutil.copytree(str(src), str(dst), dirs_exist_ok=True)
            meta = {
                "determined_version": __version__,
                "framework": self.framework,
                "format": self.format,
                "experiment_id": self.experiment_id,
                "trial_id": self.trial_id,
                "hparams": self.hparams,
                "experiment_config": self.experiment_config,
                "metadata": self.record.get("metadata") or {},
            }
            dst.joinpath("metadata.json").write_text(json.dumps(meta, indent=2))
        return str(dst)

    def load(self, path: Optional[str] = None, map_location: Any = None) -> Any:
        return load_checkpoint(self.download(path), map_location=map_location)

    def __repr__(self) -> str:
        return f"Checkpoint(uuid={self.uuid}, trial_id={self.trial_id}, step_id={self.step_id})"


def load_checkpoint(ckpt_dir: str, map_location: Any = None) -> Any:
    """Re-instantiate the trial from ``<ckpt>/code`` and load ``models_state_dict`` into it
    (reference ``experimental/checkpoint/_torch.py:10``).  Returns the first wrapped model."""
    import torch

    from determined_1_amd.experimental._local import make_controller
    from determined_1_amd.harness.load import load_trial_class

    ckpt = pathlib.Path(ckpt_dir)
    meta = json.loads(ckpt.joinpath("metadata.json").read_text())
    trial_class = load_trial_class(meta["experiment_config"]["entrypoint"], str(ckpt.joinpath("code")))
    ctrl = make_controller(trial_class, meta["experiment_config"], iter([]), hparams=meta["hparams"],
                           use_gpu=map_location not in ("cpu", torch.device("cpu")) and torch.cuda.is_available())
    from determined_1_amd.pytorch._trial import CHECKPOINT_FILE, _pickle_module

    state = torch.load(str(ckpt.joinpath(CHECKPOINT_FILE)), map_location=map_location, weights_only=False,
                       pickle_module=_pickle_module)
    models = ctrl.context.models
    for m, sd in zip(models, state["models_state_dict"]):
        m.load_state_dict(sd)
    return models[0] if len(models) == 1 else models


class TrialReference:
    def __init__(self, client: MasterClient, trial_id: int) -> None:
        self._client = client
        self.id = trial_id

    def describe(self) -> Dict[str, Any]:
        return self._client.get(f"/trials/{self.id}")

    def select_checkpoint(self, latest: bool = False, best: bool = False, uuid: Optional[str] = None,
                          sort_by: Optional[str] = None, smaller_is_better: bool = True) -> Checkpoint:
        t = self.describe()
        ckpts = [c for c in t["checkpoints"] if c.get("state") == "COMPLETED"]
        if uuid:
            ckpts = [c for c in ckpts if c["uuid"] == uuid]
        elif latest:
            ckpts.sort(key=lambda c: c["step_id"], reverse=True)
        else:
            vals = {v["step_id"]: v for v in t["validations"] if v.get("state") == "COMPLETED"}
            exp = self._client.experiment(t["experiment_id"])
            metric = sort_by or exp["config"]["searcher"]["metric"]
            sib = smaller_is_better if sort_by else exp["config"]["searcher"].get("smaller_is_better", True)

            def key(c: Dict[str, Any]) -> float:
                v = vals.get(c["step_id"], {}).get("metrics", {}).get("validation_metrics", {}).get(metric)
                if v is None:
                    return float("inf")
                return v if sib else -v

            ckpts.sort(key=key)
        if not ckpts:
            raise LookupError(f"no checkpoint for trial {self.id}")
        rec = dict(ckpts[0])
        rec.setdefault("experiment_id", t["experiment_id"])
        return Checkpoint(self._client, rec)

    def top_checkpoint(self) -> Checkpoint:
        return self.select_checkpoint(best=True)


class ExperimentReference:
    def __init__(self, client: MasterClient, exp_id: int) -> None:
        self._client = client
        self.id = exp_id

    def describe(self) -> Dict[str, Any]:
        return self._client.experiment(self.id)

    def activate(self) -> None:
        self._client.set_state(self.id, "ACTIVE")

    def pause(self) -> None:
        self._client.set_state(self.id, "PAUSED")

    def cancel(self) -> None:
        self._client.set_state(self.id, "STOPPING_CANCELED")

    def kill(self) -> None:
        self._client.post(f"/experiments/{self.id}/kill")

    def wait(self, timeout: float = 86400) -> str:
        return self._client.wait_for_experiment(self.id, timeout=timeout)

    def trials(self) -> List[TrialReference]:
        return [TrialReference(self._client, t["id"]) for t in self.describe()["trials"]]

    def top_n_checkpoints(self, limit: int) -> List[Checkpoint]:
        return [Checkpoint(self._client, c) for c in self._client.get(f"/experiments/{self.id}/checkpoints")[:limit]]

    def top_checkpoint(self) -> Checkpoint:
        cs = self.top_n_checkpoints(1)
        if not cs:
            raise LookupError(f"no checkpoints for experiment {self.id}")
        return cs[0]


class Determined:
    def __init__(self, master: Optional[str] = None) -> None:
        self._client = MasterClient(master)

    def create_experiment(self, config: Dict[str, Any], model_dir: str, activate: bool = True) -> ExperimentReference:
        from determined_1_amd.api import read_context

        r = self._client.create_experiment(config, read_context(pathlib.Path(model_dir)), activate=activate)
        return ExperimentReference(self._client, r["id"])

    def get_experiment(self, exp_id: int) -> ExperimentReference:
        return ExperimentReference(self._client, exp_id)

    def get_trial(self, trial_id: int) -> TrialReference:
        return TrialReference(self._client, trial_id)

    def get_checkpoint(self, uuid: str) -> Checkpoint:
        return Checkpoint(self._client, self._client.get(f"/checkpoints/{uuid}"))

    def get_models(self) -> List[Dict[str, Any]]:
        return self._client.get("/models")

    def create_model(self, name: str, description: str = "") -> Dict[str, Any]:
        return self._client.post(f"/models/{name}", {"description": description})

    def register_model_version(self, name: str, checkpoint_uuid: str) -> Dict[str, Any]:
        return self._client.post(f"/models/{name}/versions", {"checkpoint_uuid": checkpoint_uuid})
