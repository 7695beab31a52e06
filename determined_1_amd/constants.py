"""Well-known ports, paths and local-mode defaults (reference: harness/determined/constants.py)."""
from pathlib import Path

# Rendezvous port base; offset by the trial's min slot id (master/pkg/tasks/ports.go:13-40).
LOCAL_RENDEZVOUS_PORT = 1734
MAX_SLOTS_PER_AGENT = 16

# torch.distributed TCPStore / RCCL bootstrap port base for one trial (replaces horovod's
# sshd 12350 / gloo 12355 ports).
DIST_STORE_PORT = 12355
# Control channel (metric gather, workload fan-out) port base.
INTER_TRAIN_PROCESS_COMM_PORT_1 = 12360
INTER_TRAIN_PROCESS_COMM_PORT_2 = INTER_TRAIN_PROCESS_COMM_PORT_1 + MAX_SLOTS_PER_AGENT

TRAIN_PROCESS_ENVIRONMENT_VARIABLE_PATH = Path("/tmp/det_train_process_env.json")

DEFAULT_SEARCHER_CFG = {"name": "single", "max_length": {"batches": 100}}
DEFAULT_RESOURCES_CFG = {"slots_per_trial": 1, "native_parallel": False}
DEFAULT_SCHEDULING_UNIT = 100
DEFAULT_OPTIMIZATIONS = {
    "aggregation_frequency": 1,
    "average_aggregated_gradients": True,
    "average_training_metrics": False,
    "gradient_compression": False,
    "mixed_precision": "O0",
    "tensor_fusion_threshold": 64,
    "tensor_fusion_cycle_time": 5,
    "auto_tune_tensor_fusion": False,
}
DEFAULT_EXP_CFG = {
    "searcher": DEFAULT_SEARCHER_CFG,
    "scheduling_unit": DEFAULT_SCHEDULING_UNIT,
    "resources": DEFAULT_RESOURCES_CFG,
    "optimizations": DEFAULT_OPTIMIZATIONS,
}

AUTO_DETECT_TRIAL_RUNNER_NETWORK_INTERFACE = "DET_AUTO_DETECT_NETWORK_INTERFACE"
DIST_STARTUP_TIMEOUT_SECONDS = 1200

CONTAINER_STDOUT = "/run/determined/train/logs/stdout.log"
CONTAINER_STDERR = "/run/determined/train/logs/stderr.log"

# In-container mount point of shared_fs checkpoint storage (common/determined_common/constants.py:33).
SHARED_FS_CONTAINER_PATH = "/determined_shared_fs"

# Context packaging limit (common/determined_common/constants.py:5-18).
MAX_CONTEXT_SIZE = 95 * 1024 * 1024

# tensor-fusion autotune CSV (reference HOROVOD_AUTOTUNE_LOG_FILEPATH)
FUSION_AUTOTUNE_LOG_FILEPATH = "/tmp/autotune_log.csv"
