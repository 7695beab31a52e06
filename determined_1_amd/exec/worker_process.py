"""One training process per slot, started by ``SubprocessLauncher`` (reference
``exec/worker_process.py:19-60``).  Joins the torch.distributed world (RCCL on GPUs, gloo on CPU)
through the controller's pre_execute_hook, then runs the trial controller on the broadcast
workload stream."""
import logging
import os
import pathlib
import sys
import traceback

from determined_1_amd.env import EnvContext, RendezvousInfo
from determined_1_amd.harness.launcher import WorkerReceiver
from determined_1_amd.harness.load import prepare_controller
from determined_1_amd.parallel.dist import DistributedConfig, RankInfo


def main() -> int:
    rank = RankInfo.from_env()
    logging.basicConfig(level=logging.INFO if rank.rank == 0 else logging.WARNING,
                        format=f"%(asctime)s [rank={rank.rank}] %(levelname)s %(message)s")
    env = EnvContext.from_environ()
    receiver = WorkerReceiver(rank.local_rank)
    try:
        rdv = RendezvousInfo(os.environ["DET_RENDEZVOUS_ADDRS"].split(","),
                             os.environ.get("DET_RENDEZVOUS_ADDRS2", "").split(","),
                             int(os.environ["DET_RENDEZVOUS_RANK"]))
        dist_cfg = DistributedConfig.from_configs(env.experiment_config, world_size=rank.size,
                                                  num_agents=rank.cross_size)
        dist_cfg.use = rank.size > 1
        lp = os.environ.get("DET_LOAD_PATH") or None
        ctrl = prepare_controller(env, iter(receiver), pathlib.Path(lp) if lp else None, rdv, dist_cfg, rank)
        ctrl.run()
    except Exception:
        tb = traceback.format_exc()
        sys.stderr.write(tb)
        receiver.send_error(tb)
        return 1
    finally:
        from determined_1_amd.parallel import dist as pdist

        pdist.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
