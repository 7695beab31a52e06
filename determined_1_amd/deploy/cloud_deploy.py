"""``det deploy aws|gcp up|down|list`` (reference ``deploy/determined_deploy/{aws,gcp}``, which
drive CloudFormation / Terraform): bring up a master VM whose startup script runs ``det-master``
with the cloud provisioner configured, so agent VMs are then launched on demand by the master
itself (``deploy/cloud_provider.py``); tear everything of a cluster id down again.

Instances are found by tag (``determined-cluster=<cluster-id>``; agents additionally carry their
pool tag), over the same REST clients as the provisioner (EC2 Query API with SigV4, Compute v1).
"""
import argparse
import json
import sys
from typing import Any, Dict, List

from determined_1_amd.deploy.cloud_provider import AWSProvider, GCPProvider, STATE


# Credentials the deploying user passed for THIS client; they must never be rendered into the master
# VM's user-data / startup-script (readable through instance metadata and DescribeInstanceAttribute).
# The master VM authenticates with its instance profile (AWS) or service account (GCP) instead.
SECRET_KEYS = ("access_key", "secret_key", "session_token", "token")


def _strip_secrets(cfg: Dict[str, Any]) -> Dict[str, Any]:
    return {k: v for k, v in cfg.items() if k not in SECRET_KEYS}


def master_script(args: argparse.Namespace, provider_cfg: Dict[str, Any]) -> str:
    provider_cfg = _strip_secrets(provider_cfg)
    prov = {"provider": args.provider, "max_instances": args.max_agents, "slots_per_instance": args.slots_per_agent,
            "max_idle_agent_period_ms": args.max_idle_agent_period_ms, args.provider: provider_cfg}
    cfg = {"port": args.master_port, "store_dir": args.store_dir, "provisioner": prov,
           "checkpoint_storage": json.loads(args.checkpoint_storage)}
    return ("#!/bin/bash\n" + (args.startup_script + "\n" if args.startup_script else "") +
            f"cat > /tmp/det-master.json <<'DETEOF'\n{json.dumps(cfg)}\nDETEOF\n"
            f"exec {args.master_command} --config-file /tmp/det-master.json\n")


class AWSDeployment(AWSProvider):
    def __init__(self, args: argparse.Namespace) -> None:
        cfg = json.loads(args.provider_config)
        cfg.setdefault("tag_key", "determined-cluster")
        cfg["tag_value"] = args.cluster_id
        super().__init__(cfg, "master", "", 0)
        self.args = args

    def up(self) -> List[str]:
        agent_cfg = _strip_secrets(self.cfg)
        agent_cfg.pop("tag_value", None)
        agent_cfg["tag_key"] = "determined-resource-pool"
        agent_cfg["cluster_id"] = self.args.cluster_id
        self.user_data = master_script(self.args, agent_cfg)
        return self.launch(1)

    def down(self) -> List[str]:
        ids = [i["id"] for i in self.list() if i["state"] != "Stopped"]
        for pool in self.args.pools.split(","):  # agent VMs carry "<cluster-id>-<pool>"
            agents = AWSProvider(dict(self.cfg, tag_key="determined-resource-pool", tag_value=None,
                                      cluster_id=self.args.cluster_id), pool, "", 0)
            ids += [i["id"] for i in agents.list() if i["state"] != "Stopped"]
        return self.terminate(ids)


class GCPDeployment(GCPProvider):
    def __init__(self, args: argparse.Namespace) -> None:
        cfg = json.loads(args.provider_config)
        cfg["label_value"] = args.cluster_id
        super().__init__(cfg, "master", "", 0)
        self.args = args

    def up(self) -> List[str]:
        agent_cfg = _strip_secrets(self.cfg)
        agent_cfg.pop("label_value", None)
        agent_cfg["cluster_id"] = self.args.cluster_id
        self.script = master_script(self.args, agent_cfg)
        return self.launch(1)

    def down(self) -> List[str]:
        ids = [i["id"] for i in self.list()]
        for pool in self.args.pools.split(","):
            agents = GCPProvider(dict(self.cfg, label_value=None, cluster_id=self.args.cluster_id), pool, "", 0)
            ids += [i["id"] for i in agents.list()]
        return self.terminate(ids)


def main(argv: List[str]) -> int:
    ap = argparse.ArgumentParser(prog="det deploy")
    ap.add_argument("provider", choices=["aws", "gcp"])
    ap.add_argument("action", choices=["up", "down", "list"])
    ap.add_argument("--cluster-id", required=True)
    ap.add_argument("--provider-config", default="{}",
                    help="JSON: aws {region, image_id, instance_type, endpoint_url, ...} / gcp {project, zone, image, ...}")
    ap.add_argument("--master-port", type=int, default=8080)
    ap.add_argument("--master-command", default="det-master")
    ap.add_argument("--store-dir", default="/var/lib/determined/store")
    ap.add_argument("--max-agents", type=int, default=8)
    ap.add_argument("--slots-per-agent", type=int, default=8)
    ap.add_argument("--max-idle-agent-period-ms", type=int, default=300000)
    ap.add_argument("--checkpoint-storage", default='{"type": "shared_fs", "host_path": "/mnt/checkpoints"}')
    ap.add_argument("--startup-script", default="")
    ap.add_argument("--pools", default="default", help="resource pools whose agent VMs `down` terminates")
    args = ap.parse_args(argv)
    dep = AWSDeployment(args) if args.provider == "aws" else GCPDeployment(args)
    if args.action == "up":
        print(json.dumps({"master_instances": dep.up(), "master_port": args.master_port}))
    elif args.action == "down":
        print(json.dumps({"terminated": dep.down()}))
    else:
        print(json.dumps({"master_instances": dep.list()}))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
