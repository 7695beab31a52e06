"""Trial-process entrypoint started by the agent (reference ``exec/harness.py:150-227``).

    python -m determined_1_amd.exec.harness          (env: the C-env contract)

1. parse/validate the ``DET_*`` environment into an ``EnvContext``;
2. build + validate checkpoint storage (write/read/delete probe);
3. connect the master socket and wait for rendezvous;
4. restore the latest checkpoint (if any);
5. run the pipeline: SocketManager -> WorkloadManager -> (SubprocessLauncher | controller).
``InvalidHP`` raised by user code becomes ``exited_reason: INVALID_HP``; other exceptions exit
non-zero so the master restarts the trial from its last checkpoint.
"""
import contextlib
import faulthandler
import json
import logging
import os
import pathlib
import sys
import traceback
from typing import Iterator, Optional

from determined_1_amd import errors, storage
from determined_1_amd.env import EnvContext
from determined_1_amd.harness.load import prepare_controller
from determined_1_amd.harness import timeline
from determined_1_amd.harness.socket_manager import SocketManager
from determined_1_amd.harness.workload_manager import build_workload_manager
from determined_1_amd.parallel.dist import DistributedConfig, RankInfo


@contextlib.contextmanager
def maybe_load_checkpoint(storage_mgr: storage.StorageManager, latest: Optional[dict]) -> Iterator[Optional[pathlib.Path]]:
    if not latest or not latest.get("uuid"):
        yield None
        return
    md = storage.StorageMetadata.from_json(latest)
    with storage_mgr.restore_path(md) as path:
        yield pathlib.Path(path)


def local_slot_count(env: EnvContext) -> int:
    if env.use_gpu:
        return max(1, len(env.container_gpus) or len(env.slot_ids))
    # CPU slots (artificial agents): one gloo process per slot
    return max(1, len(env.slot_ids))


def _warm_gpu() -> None:
    """HIP runtime + device init (~0.3-0.5 s on an MI355X) on a side thread, overlapped with the
    storage probe, the master rendezvous and the user-code import; the model's first ``.cuda()``
    then finds the runtime up.  torch serialises its lazy init, so a concurrent caller just waits."""
    try:
        import torch

        torch.cuda.init()
        torch.empty(1, device="cuda")  # primary context + caching allocator
    except Exception as e:  # the trial's own device use reports real problems
        logging.debug("early GPU init failed: %s", e)


def main() -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s [harness] %(levelname)s %(message)s")
    faulthandler.enable()  # a crashing trial process leaves its Python stack in the trial log
    if os.environ.get("DET_ZYGOTE_PID"):
        logging.info("trial process forked from warm zygote %s", os.environ["DET_ZYGOTE_PID"])
    timeline.mark("imports done")
    env = EnvContext.from_environ()
    # the shipped MIOpen find-db + kernel cache (ops/miopen_db): trial containers start with the
    # conv kernels already compiled instead of JIT-compiling them per container
    from determined_1_amd.ops import miopen_db

    miopen_db.configure(os.environ)
    slots_per_trial = int((env.experiment_config.get("resources") or {}).get("slots_per_trial", 1) or 1)
    if env.use_gpu and slots_per_trial == 1 and os.environ.get("DET_EARLY_GPU_INIT", "1") == "1":
        # single-process trial: this process is the one that uses the GPU (a multi-slot launcher
        # parent never touches it)
        import threading

        threading.Thread(target=_warm_gpu, name="det-gpu-init", daemon=True).start()
    if env.debug:
        faulthandler.dump_traceback_later(30, repeat=True)
    cfg = env.experiment_config
    storage_mgr = storage.build(cfg.get("checkpoint_storage", {}))
    storage.validate_manager(storage_mgr)
    timeline.mark("storage validated")
    socket_mgr = SocketManager(env)
    rendezvous = socket_mgr.rendezvous_info
    timeline.mark("rendezvous")
    metric_writer = None
    tb_mgr = None
    try:
        from determined_1_amd import tensorboard

        tb_mgr = tensorboard.build(env, cfg.get("checkpoint_storage", {}))
        metric_writer = tensorboard.MetricWriter(tb_mgr.base_dir) if rendezvous.get_rank() == 0 else None
    except ImportError:
        pass
    wm = build_workload_manager(env, iter(socket_mgr), rendezvous, storage_mgr, tb_mgr, metric_writer)
    local_size = local_slot_count(env)
    world = local_size * max(1, rendezvous.get_size())
    native_parallel = bool(cfg.get("resources", {}).get("native_parallel", False))
    try:
        with maybe_load_checkpoint(storage_mgr, env.latest_checkpoint) as load_path:
            if world > 1 and not native_parallel:
                from determined_1_amd.harness.launcher import SubprocessLauncher

                SubprocessLauncher(env, iter(wm), rendezvous, local_size, load_path).run()
            else:
                dist_cfg = DistributedConfig.from_configs(cfg, world_size=1, num_agents=1)
                dist_cfg.use = False
                ctrl = prepare_controller(env, iter(wm), load_path, rendezvous, dist_cfg, RankInfo())
                ctrl.run()
    except errors.InvalidHP as e:
        logging.warning("trial reported invalid hyperparameters: %s", e)
        socket_mgr.respond_current({"metrics": None, "exited_reason": "INVALID_HP"})
    except Exception:
        traceback.print_exc()
        socket_mgr.close()
        return 1
    socket_mgr.close()
    timeline.mark("exit")
    return 0


def _fast_exit(rc: int) -> None:
    """Leave without interpreter/HIP-runtime teardown once all work is durable: every checkpoint
    and TensorBoard event file was written and flushed inside its workload, and the master socket
    is closed.  Teardown of a torch+HIP process takes a noticeable fraction of a short HP-search
    trial and the master counts it, since a trial ends when its container exits."""
    logging.shutdown()
    try:
        sys.stdout.flush()
        sys.stderr.flush()
    finally:
        os._exit(rc)


if __name__ == "__main__":
    code = main()
    if code == 0 and os.environ.get("DET_FAST_EXIT", "1") == "1":
        _fast_exit(code)
    sys.exit(code)
