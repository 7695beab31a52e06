"""Cloud instance providers for the master's provisioner (reference
``master/internal/provisioner/{aws,gcp}.go``): launch / list / terminate agent VMs whose startup
script runs ``det-agent`` against this master, tagged so the provisioner only ever sees its own
pool's instances.

Speaks the clouds' REST APIs directly (no boto3 / google-api-client on this image):
  * AWS  -- EC2 Query API (``RunInstances``, ``DescribeInstances``, ``TerminateInstances``,
            Signature V4 with ``storage.rest_clients.sigv4_headers``), user-data startup script;
  * GCP  -- Compute Engine v1 (``instances.insert/list/delete``) with an OAuth bearer token,
            ``startup-script`` metadata.
Both take ``endpoint_url`` overrides (tests use in-process fakes).

The C++ provisioner (native/src/provisioner.cc, ``CommandProvider``) runs this module once as a
coprocess and exchanges one JSON object per line:

    -> {"op": "list"}                 <- {"instances": [{"id", "state": Starting|Running|Stopped}]}
    -> {"op": "launch", "n": 2}       <- {"launched": ["i-..", ...]}
    -> {"op": "terminate", "ids": []} <- {"terminated": [...]}
    (errors: {"error": "..."})

    python -m determined_1_amd.deploy.cloud_provider --config '<provisioner JSON>' --pool default \\
        --master-host H --master-port P
"""
import argparse
import base64
import json
import os
import sys
import time
import urllib.parse
import uuid
import xml.etree.ElementTree as ET
from typing import Any, Dict, List, Optional

import requests

from determined_1_amd.storage.rest_clients import sigv4_headers, _sha256

STATE = {"pending": "Starting", "running": "Running", "provisioning": "Starting", "staging": "Starting",
         "shutting-down": "Stopped", "terminated": "Stopped", "stopping": "Stopped", "stopped": "Stopped",
         "suspending": "Stopped", "suspended": "Stopped"}


def startup_script(cfg: Dict[str, Any], pool: str, master_host: str, master_port: int, id_cmd: str) -> str:
    agent = cfg.get("agent_command", "det-agent")
    extra = " ".join(cfg.get("agent_args", []))
    pre = cfg.get("startup_script", "")
    return ("#!/bin/bash\n" + (pre + "\n" if pre else "") +
            f'AGENT_ID="${{DET_INSTANCE_ID:-$({id_cmd})}}"\n'
            f"exec {agent} --master-host {master_host} --master-port {master_port} --agent-id \"$AGENT_ID\" "
            f"--resource-pool {pool} {extra}\n")


class AWSProvider:
    VERSION = "2016-11-15"

    def __init__(self, cfg: Dict[str, Any], pool: str, master_host: str, master_port: int) -> None:
        self.cfg = cfg
        self.pool = pool
        self.region = cfg.get("region") or os.environ.get("AWS_DEFAULT_REGION", "us-east-1")
        self.endpoint = (cfg.get("endpoint_url") or f"https://ec2.{self.region}.amazonaws.com").rstrip("/") + "/"
        self.ak = cfg.get("access_key") or os.environ.get("AWS_ACCESS_KEY_ID", "")
        self.sk = cfg.get("secret_key") or os.environ.get("AWS_SECRET_ACCESS_KEY", "")
        self.token = cfg.get("session_token") or os.environ.get("AWS_SESSION_TOKEN")
        # no static keys (the deployed master VM): the instance profile's rotating credentials from the
        # instance metadata service, refreshed ahead of their expiry
        self._imds = None if self.ak else (cfg.get("instance_metadata_url") or "http://169.254.169.254").rstrip("/")
        self._creds_expire = 0.0
        self.tag_key = cfg.get("tag_key", "determined-resource-pool")
        self.tag_value = cfg.get("tag_value") or f"{cfg.get('cluster_id', 'det')}-{pool}"
        self.user_data = startup_script(cfg, pool, master_host, master_port,
                                        "curl -s http://169.254.169.254/latest/meta-data/instance-id")

    def _refresh_instance_credentials(self) -> None:
        """IMDSv2: session token, then the role's temporary credentials (AccessKeyId/SecretAccessKey/Token)."""
        import time

        if self._imds is None or time.time() < self._creds_expire:
            return
        t = requests.put(f"{self._imds}/latest/api/token", headers={"X-aws-ec2-metadata-token-ttl-seconds": "300"},
                         timeout=5)
        h = {"X-aws-ec2-metadata-token": t.text} if t.status_code == 200 else {}
        base = f"{self._imds}/latest/meta-data/iam/security-credentials/"
        role = requests.get(base, headers=h, timeout=5).text.strip().splitlines()[0]
        c = requests.get(base + role, headers=h, timeout=5).json()
        self.ak, self.sk, self.token = c["AccessKeyId"], c["SecretAccessKey"], c.get("Token") or None
        self._creds_expire = time.time() + 600  # re-read well inside the credentials' hour-long lifetime

    def _call(self, params: Dict[str, str]) -> ET.Element:
        self._refresh_instance_credentials()
        params = dict(params, Version=self.VERSION)
        body = urllib.parse.urlencode(sorted(params.items())).encode()
        h = sigv4_headers("POST", self.endpoint, self.region, self.ak, self.sk, _sha256(body), self.token,
                          service="ec2", extra={"content-type": "application/x-www-form-urlencoded; charset=utf-8"})
        r = requests.post(self.endpoint, data=body, headers=h, timeout=60)
        if r.status_code != 200:
            raise IOError(f"EC2 {params.get('Action')}: {r.status_code} {r.text[:400]}")
        root = ET.fromstring(r.content)
        for el in root.iter():  # drop the namespace for simple lookups
            if "}" in el.tag:
                el.tag = el.tag.split("}", 1)[1]
        return root

    def list(self) -> List[Dict[str, str]]:
        root = self._call({"Action": "DescribeInstances", "Filter.1.Name": f"tag:{self.tag_key}",
                           "Filter.1.Value.1": self.tag_value})
        out = []
        for inst in root.iter("instancesSet"):
            for item in inst.findall("item"):
                state = item.findtext("instanceState/name", "pending")
                out.append({"id": item.findtext("instanceId"), "state": STATE.get(state, "Starting")})
        return out

    def launch(self, n: int) -> List[str]:
        c = self.cfg
        p = {"Action": "RunInstances", "ImageId": c["image_id"], "InstanceType": c.get("instance_type", "m5.large"),
             "MinCount": str(n), "MaxCount": str(n), "UserData": base64.b64encode(self.user_data.encode()).decode(),
             "ClientToken": uuid.uuid4().hex,
             "TagSpecification.1.ResourceType": "instance",
             "TagSpecification.1.Tag.1.Key": self.tag_key, "TagSpecification.1.Tag.1.Value": self.tag_value,
             "TagSpecification.1.Tag.2.Key": "Name", "TagSpecification.1.Tag.2.Value": f"det-agent-{self.pool}"}
        if c.get("key_name"):
            p["KeyName"] = c["key_name"]
        if c.get("subnet_id"):
            p["SubnetId"] = c["subnet_id"]
        for i, sg in enumerate(c.get("security_group_ids", []), 1):
            p[f"SecurityGroupId.{i}"] = sg
        if c.get("iam_instance_profile_arn"):
            p["IamInstanceProfile.Arn"] = c["iam_instance_profile_arn"]
        if c.get("root_volume_size"):
            p["BlockDeviceMapping.1.DeviceName"] = c.get("root_device_name", "/dev/sda1")
            p["BlockDeviceMapping.1.Ebs.VolumeSize"] = str(c["root_volume_size"])
        if c.get("spot"):
            p["InstanceMarketOptions.MarketType"] = "spot"
        root = self._call(p)
        return [it.findtext("instanceId") for it in root.iter("item") if it.findtext("instanceId")]

    def terminate(self, ids: List[str]) -> List[str]:
        if not ids:
            return []
        p = {"Action": "TerminateInstances"}
        for i, x in enumerate(ids, 1):
            p[f"InstanceId.{i}"] = x
        self._call(p)
        return ids


class GCPProvider:
    def __init__(self, cfg: Dict[str, Any], pool: str, master_host: str, master_port: int) -> None:
        self.cfg = cfg
        self.pool = pool
        self.base = (cfg.get("endpoint_url") or "https://compute.googleapis.com").rstrip("/")
        self.project, self.zone = cfg["project"], cfg["zone"]
        self.label = cfg.get("label_value") or f"{cfg.get('cluster_id', 'det')}-{pool}".lower()
        self._token = cfg.get("token") or os.environ.get("GOOGLE_OAUTH_ACCESS_TOKEN")
        self.script = startup_script(cfg, pool, master_host, master_port, "hostname")

    def _auth(self) -> Dict[str, str]:
        if not self._token:
            r = requests.get("http://metadata.google.internal/computeMetadata/v1/instance/service-accounts/default/token",
                             headers={"Metadata-Flavor": "Google"}, timeout=5)
            self._token = r.json()["access_token"]
        return {"Authorization": f"Bearer {self._token}"}

    def _url(self, suffix: str = "") -> str:
        return f"{self.base}/compute/v1/projects/{self.project}/zones/{self.zone}/instances{suffix}"

    def list(self) -> List[Dict[str, str]]:
        out, token = [], None
        while True:
            params = {"filter": f"labels.determined-pool={self.label}"}
            if token:
                params["pageToken"] = token
            r = requests.get(self._url(), params=params, headers=self._auth(), timeout=60)
            if r.status_code != 200:
                raise IOError(f"GCE list: {r.status_code} {r.text[:300]}")
            j = r.json()
            for it in j.get("items", []):
                out.append({"id": it["name"], "state": STATE.get(it.get("status", "PROVISIONING").lower(), "Starting")})
            token = j.get("nextPageToken")
            if not token:
                return out

    def launch(self, n: int) -> List[str]:
        c = self.cfg
        names = []
        for _ in range(n):
            name = f"det-{self.pool}-{uuid.uuid4().hex[:10]}".lower()
            body = {
                "name": name,
                "machineType": f"zones/{self.zone}/machineTypes/{c.get('machine_type', 'n1-standard-8')}",
                "labels": {"determined-pool": self.label},
                "disks": [{"boot": True, "autoDelete": True, "initializeParams": {
                    "sourceImage": c["image"], "diskSizeGb": str(c.get("boot_disk_size", 200))}}],
                "networkInterfaces": [{"network": c.get("network", "global/networks/default"),
                                       "accessConfigs": [{"type": "ONE_TO_ONE_NAT"}]}],
                "metadata": {"items": [{"key": "startup-script", "value": self.script}]},
                "scheduling": {"preemptible": bool(c.get("preemptible", False)),
                               "onHostMaintenance": "TERMINATE"},
            }
            if c.get("service_account_email"):
                body["serviceAccounts"] = [{"email": c["service_account_email"],
                                            "scopes": ["https://www.googleapis.com/auth/cloud-platform"]}]
            r = requests.post(self._url(), json=body, headers=self._auth(), timeout=60)
            if r.status_code not in (200, 201):
                raise IOError(f"GCE insert: {r.status_code} {r.text[:300]}")
            names.append(name)
        return names

    def terminate(self, ids: List[str]) -> List[str]:
        for name in ids:
            r = requests.delete(self._url("/" + name), headers=self._auth(), timeout=60)
            if r.status_code not in (200, 204, 404):
                raise IOError(f"GCE delete {name}: {r.status_code}")
        return ids


PROVIDERS = {"aws": AWSProvider, "gcp": GCPProvider}


def build(cfg: Dict[str, Any], pool: str, master_host: str, master_port: int) -> Any:
    kind = cfg.get("provider", "aws")
    sub = dict(cfg.get(kind, {}))
    sub.setdefault("cluster_id", cfg.get("cluster_id", "det"))
    return PROVIDERS[kind](sub, pool, master_host, master_port)


def serve(provider: Any, inp=sys.stdin, out=sys.stdout) -> None:
    for line in inp:
        line = line.strip()
        if not line:
            continue
        try:
            req = json.loads(line)
            op = req.get("op")
            if op == "list":
                resp: Dict[str, Any] = {"instances": provider.list()}
            elif op == "launch":
                resp = {"launched": provider.launch(int(req.get("n", 0)))}
            elif op == "terminate":
                resp = {"terminated": provider.terminate(list(req.get("ids", [])))}
            else:
                resp = {"error": f"unknown op {op!r}"}
        except Exception as e:  # report and keep serving: the master retries on its next tick
            resp = {"error": f"{type(e).__name__}: {e}"}
        out.write(json.dumps(resp) + "\n")
        out.flush()


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True, help="provisioner config JSON")
    ap.add_argument("--pool", default="default")
    ap.add_argument("--master-host", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=8080)
    ap.add_argument("--once", choices=["list", "launch", "terminate"])
    ap.add_argument("args", nargs="*")
    a = ap.parse_args(argv)
    prov = build(json.loads(a.config), a.pool, a.master_host, a.master_port)
    if a.once == "list":
        print(json.dumps(prov.list()))
    elif a.once == "launch":
        print(json.dumps(prov.launch(int(a.args[0]))))
    elif a.once == "terminate":
        print(json.dumps(prov.terminate(a.args)))
    else:
        serve(prov)
    return 0


if __name__ == "__main__":
    sys.exit(main())
