"""Trial-process layers: the same layering as the reference harness,

    SocketManager (master WebSocket)  ->  WorkloadManager (checks, storage, tensorboard)
        ->  SubprocessLauncher (one worker process per GPU; multi-slot trials)
            ->  WorkerReceiver  ->  TrialController (PyTorchTrial loop)

Single-slot trials skip the launcher and run the controller in the harness process.
"""
from determined_1_amd.harness.load import load_trial_class, prepare_controller
from determined_1_amd.harness.socket_manager import SocketManager
from determined_1_amd.harness.workload_manager import WorkloadManager, build_workload_manager

__all__ = ["SocketManager", "WorkloadManager", "build_workload_manager", "load_trial_class", "prepare_controller"]
