"""Trial-process environment: the typed view of the ``DET_*`` env-var contract (SURVEY C-env).

Reference: ``harness/determined/_env_context.py:9-109`` (batch-size math and its warnings),
``harness/determined/_rendezvous_info.py``, ``harness/determined/exec/harness.py:43-60`` (the
required keys).
"""
import json
import logging
import os
from typing import Any, Dict, List, Optional, Tuple

from determined_1_amd import constants, workload
from determined_1_amd.config import ExperimentConfig

REQUIRED_ENV_KEYS = [
    "DET_MASTER_ADDR",
    "DET_MASTER_PORT",
    "DET_CONTAINER_ID",
    "DET_EXPERIMENT_ID",
    "DET_TRIAL_ID",
    "DET_TRIAL_SEED",
    "DET_EXPERIMENT_CONFIG",
    "DET_HPARAMS",
    "DET_INITIAL_WORKLOAD",
    "DET_LATEST_CHECKPOINT",
    "DET_WORKLOAD_MANAGER_TYPE",
    "DET_RENDEZVOUS_PORTS",
    "DET_TRIAL_RUNNER_NETWORK_INTERFACE",
    "DET_USE_GPU",
    "DET_SLOT_IDS",
    "DET_AGENT_ID",
]


class EnvContext:
    def __init__(
        self,
        master_addr: str,
        master_port: int,
        use_tls: bool,
        master_cert_file: Optional[str],
        master_cert_name: Optional[str],
        container_id: str,
        experiment_config: Dict[str, Any],
        hparams: Dict[str, Any],
        initial_workload: workload.Workload,
        latest_checkpoint: Optional[Dict[str, Any]],
        use_gpu: bool,
        container_gpus: List[str],
        slot_ids: List[int],
        debug: bool,
        workload_manager_type: str,
        det_rendezvous_ports: str,
        det_trial_unique_port_offset: int,
        det_trial_runner_network_interface: str,
        det_trial_id: str,
        det_experiment_id: str,
        det_cluster_id: str,
        trial_seed: int,
        managed_training: bool = True,
        test_mode: bool = False,
        on_cluster: bool = False,
    ) -> None:
        self.master_addr = master_addr
        self.master_port = master_port
        self.use_tls = use_tls
        self.master_cert_file = master_cert_file
        self.master_cert_name = master_cert_name
        self.container_id = container_id
        self.experiment_config = ExperimentConfig(experiment_config)
        self.hparams = hparams
        self.initial_workload = initial_workload
        self.latest_checkpoint = latest_checkpoint
        self.use_gpu = use_gpu
        self.container_gpus = container_gpus
        self.slot_ids = slot_ids
        self.debug = debug
        self.workload_manager_type = workload_manager_type
        self.det_rendezvous_ports = det_rendezvous_ports
        self.det_trial_unique_port_offset = det_trial_unique_port_offset
        self.det_trial_runner_network_interface = det_trial_runner_network_interface
        self.det_trial_id = det_trial_id
        self.det_experiment_id = det_experiment_id
        self.det_cluster_id = det_cluster_id
        self.trial_seed = trial_seed
        self.managed_training = managed_training
        self.test_mode = test_mode
        self.on_cluster = on_cluster
        self._per_slot_batch_size, self._global_batch_size = self._calculate_batch_sizes()

    def first_step(self) -> int:
        return self.initial_workload.step_id

    def rendezvous_ports(self) -> Tuple[int, int]:
        try:
            ports = [int(x) for x in self.det_rendezvous_ports.split(",") if x]
        except ValueError:
            ports = []
        if len(ports) != 2:
            base = constants.LOCAL_RENDEZVOUS_PORT + self.det_trial_unique_port_offset
            ports = [base, base + constants.MAX_SLOTS_PER_AGENT]
        return ports[0], ports[1]

    def _calculate_batch_sizes(self) -> Tuple[int, int]:
        if "global_batch_size" not in self.hparams:
            raise AssertionError(
                "Please specify `global_batch_size` under `hyperparameters` in experiment config."
            )
        if "batch_size" in self.hparams:
            logging.warning("Use `global_batch_size` not `batch_size` under `hyperparameters` in experiment config.")
        gbs = self.hparams["global_batch_size"]
        if not isinstance(gbs, int):
            raise AssertionError("`global_batch_size` hparam must be an int.")
        if self.experiment_config.native_parallel_enabled():
            return gbs, gbs
        slots = max(1, self.experiment_config.slots_per_trial())
        if gbs < slots:
            raise AssertionError(
                "Please set the `global_batch_size` hyperparameter to be greater or equal to the "
                f"number of slots. Current batch_size: {gbs}, slots_per_trial: {slots}."
            )
        per = gbs // slots
        eff = per * slots
        if eff != gbs:
            logging.warning(f"`global_batch_size` changed from {gbs} to {eff} to divide equally across {slots} slots.")
        return per, eff

    @property
    def per_slot_batch_size(self) -> int:
        return self._per_slot_batch_size

    @property
    def global_batch_size(self) -> int:
        return self._global_batch_size

    # ------------------------------------------------------------------------------------------
    @staticmethod
    def from_environ(environ: Optional[Dict[str, str]] = None) -> "EnvContext":
        """Build from the container env (the C-env contract written by the agent/master)."""
        env = dict(os.environ if environ is None else environ)
        missing = [k for k in REQUIRED_ENV_KEYS if k not in env]
        if missing:
            raise KeyError(f"missing required environment variables: {missing}")
        latest_ckpt = None
        path = env.get("DET_LATEST_CHECKPOINT", "")
        if path and os.path.exists(path):
            with open(path) as f:
                latest_ckpt = json.load(f)
        gpus = [g for g in env.get("DET_CONTAINER_GPUS", "").split(",") if g]
        slot_ids = json.loads(env.get("DET_SLOT_IDS", "[]"))
        use_gpu = env.get("DET_USE_GPU", "false").lower() == "true"
        if use_gpu and not gpus:
            gpus = [str(s) for s in slot_ids]
        return EnvContext(
            master_addr=env["DET_MASTER_ADDR"],
            master_port=int(env["DET_MASTER_PORT"]),
            use_tls=env.get("DET_USE_TLS", "false").lower() == "true",
            master_cert_file=env.get("DET_MASTER_CERT_FILE"),
            master_cert_name=env.get("DET_MASTER_CERT_NAME"),
            container_id=env["DET_CONTAINER_ID"],
            experiment_config=json.loads(env["DET_EXPERIMENT_CONFIG"]),
            hparams=json.loads(env["DET_HPARAMS"]),
            initial_workload=workload.Workload.from_json(json.loads(env["DET_INITIAL_WORKLOAD"])),
            latest_checkpoint=latest_ckpt,
            use_gpu=use_gpu,
            container_gpus=gpus,
            slot_ids=slot_ids,
            debug=json.loads(env["DET_EXPERIMENT_CONFIG"]).get("debug", False),
            workload_manager_type=env["DET_WORKLOAD_MANAGER_TYPE"],
            det_rendezvous_ports=env["DET_RENDEZVOUS_PORTS"],
            det_trial_unique_port_offset=int(env.get("DET_TRIAL_UNIQUE_PORT_OFFSET", "0")),
            det_trial_runner_network_interface=env["DET_TRIAL_RUNNER_NETWORK_INTERFACE"],
            det_trial_id=env["DET_TRIAL_ID"],
            det_experiment_id=env["DET_EXPERIMENT_ID"],
            det_cluster_id=env.get("DET_CLUSTER_ID", ""),
            trial_seed=int(env["DET_TRIAL_SEED"]),
            on_cluster=True,
        )


class RendezvousInfo:
    """Addresses of every container of the trial plus this container's rank
    (reference ``_rendezvous_info.py``; master pushes ``RENDEZVOUS_INFO``, trial.go:813-908)."""

    def __init__(self, addrs: List[str], addrs2: List[str], rank: int) -> None:
        self.addrs = addrs
        self.addrs2 = addrs2
        self.rank = rank

    def get_rank(self) -> int:
        return self.rank

    def get_size(self) -> int:
        return len(self.addrs)

    def get_addrs(self) -> List[str]:
        return self.addrs

    def get_ip_addresses(self) -> List[str]:
        return [a.split(":")[0] for a in self.addrs]

    def get_master_address(self) -> Tuple[str, int]:
        host, port = self.addrs[0].rsplit(":", 1)
        return host, int(port)
