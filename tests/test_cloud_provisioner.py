"""Cloud provisioning (deploy/cloud_provider.py + the master's CommandProvider; SURVEY M15,
reference master/internal/provisioner/{aws,gcp}.go, provisioner_test.go).

* a fake EC2 Query endpoint that checks each request's SigV4 signature, keeps instances tagged by
  resource pool and "boots" an instance by running its user-data script (which starts a real
  det-agent with the instance id as agent id);
* e2e: a master with ``provider: aws`` and no agents scales up when a trial is pending, the trial
  runs on the provisioned agent, and the idle instance is terminated afterwards;
* a fake Compute Engine endpoint for the GCP provider's insert/list/delete with bearer auth."""
import base64
import json
import os
import pathlib
import re
import signal
import subprocess
import sys
import threading
import time
import urllib.parse
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from determined_1_amd.api import MasterClient, read_context
from determined_1_amd.deploy import LocalCluster
from determined_1_amd.deploy.cloud_provider import GCPProvider, build
from determined_1_amd.deploy.local import native_binary
from determined_1_amd.storage.rest_clients import sigv4_headers, _sha256

AK, SK = "AKIDTEST", "secret/test"
NOOP = pathlib.Path(__file__).resolve().parent / "fixtures" / "no_op"
REPO = str(pathlib.Path(__file__).resolve().parent.parent)


class FakeEC2:
    def __init__(self, workdir):
        self.instances = {}  # id -> {"state", "tags", "proc"}
        self.calls = []
        self.imds_reads = 0
        self.workdir = workdir
        ec2 = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def do_POST(self):
                n = int(self.headers.get("Content-Length", "0"))
                body = self.rfile.read(n)
                auth = self.headers.get("Authorization", "")
                m = re.search(r"Credential=([^/]+)/\d{8}/([^/]+)/ec2/aws4_request", auth)
                import datetime

                now = datetime.datetime.strptime(self.headers["x-amz-date"], "%Y%m%dT%H%M%SZ").replace(
                    tzinfo=datetime.timezone.utc)
                want = sigv4_headers("POST", f"http://{self.headers['Host']}{self.path}", m.group(2) if m else "x",
                                     AK, SK, _sha256(body), self.headers.get("x-amz-security-token"),
                                     service="ec2", now=now,
                                     extra={"content-type": self.headers["Content-Type"]})
                if not m or want["Authorization"] != auth:
                    return self._send(403, "<Response><Errors><Error><Code>AuthFailure</Code></Error></Errors></Response>")
                q = dict(urllib.parse.parse_qsl(body.decode()))
                ec2.calls.append(q["Action"])
                self._send(200, getattr(ec2, q["Action"])(q))

            # instance metadata service (IMDSv2) of the fake "VM": the instance profile's credentials
            def do_PUT(self):
                self._send(200, "imds-session") if self.path == "/latest/api/token" else self._send(404, "")

            def do_GET(self):
                if self.headers.get("X-aws-ec2-metadata-token") != "imds-session":
                    return self._send(401, "")
                base = "/latest/meta-data/iam/security-credentials/"
                if self.path == base:
                    return self._send(200, "det-master-role")
                if self.path == base + "det-master-role":
                    ec2.imds_reads += 1
                    return self._send(200, json.dumps({"AccessKeyId": AK, "SecretAccessKey": SK,
                                                       "Token": "session-tok"}))
                self._send(404, "")

            def _send(self, code, text):
                b = text.encode()
                self.send_response(code)
                self.send_header("Content-Type", "text/xml")
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.srv.daemon_threads = True
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    @property
    def url(self):
        return f"http://127.0.0.1:{self.srv.server_address[1]}"

    NS = 'xmlns="http://ec2.amazonaws.com/doc/2016-11-15/"'

    def RunInstances(self, q):
        n = int(q["MaxCount"])
        tags = {q[k]: q[k.replace(".Key", ".Value")] for k in q if re.match(r"TagSpecification\.1\.Tag\.\d+\.Key", k)}
        script = base64.b64decode(q["UserData"]).decode()
        items = ""
        for _ in range(n):
            iid = "i-" + uuid.uuid4().hex[:17]
            path = os.path.join(self.workdir, iid + ".sh")
            pathlib.Path(path).write_text(script)
            log = open(os.path.join(self.workdir, iid + ".log"), "wb")
            proc = subprocess.Popen(["bash", path], env=dict(os.environ, DET_INSTANCE_ID=iid), stdout=log,
                                    stderr=subprocess.STDOUT, start_new_session=True)
            self.instances[iid] = {"state": "running", "tags": tags, "proc": proc, "script": script}
            items += f"<item><instanceId>{iid}</instanceId><instanceState><name>pending</name></instanceState></item>"
        return f"<RunInstancesResponse {self.NS}><instancesSet>{items}</instancesSet></RunInstancesResponse>"

    def DescribeInstances(self, q):
        key = q["Filter.1.Name"][len("tag:"):]
        val = q["Filter.1.Value.1"]
        items = "".join(f"<item><instanceId>{i}</instanceId><instanceState><name>{d['state']}</name></instanceState></item>"
                        for i, d in self.instances.items() if d["tags"].get(key) == val)
        return (f"<DescribeInstancesResponse {self.NS}><reservationSet><item><instancesSet>{items}</instancesSet>"
                f"</item></reservationSet></DescribeInstancesResponse>")

    def TerminateInstances(self, q):
        for k, iid in q.items():
            if k.startswith("InstanceId.") and iid in self.instances:
                d = self.instances[iid]
                d["state"] = "terminated"
                try:
                    os.killpg(d["proc"].pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        return f"<TerminateInstancesResponse {self.NS}/>"

    def close(self):
        self.srv.shutdown()
        for d in self.instances.values():
            if d["proc"].poll() is None:
                try:
                    os.killpg(d["proc"].pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass


def test_aws_provisioner_scales_up_runs_trial_and_scales_down(tmp_path):
    ec2 = FakeEC2(str(tmp_path))
    cfg = {"provisioner": {"provider": "aws", "max_instances": 2, "slots_per_instance": 1,
                           "max_idle_agent_period_ms": 1500,
                           "aws": {"endpoint_url": ec2.url, "region": "us-west-2", "access_key": AK, "secret_key": SK,
                                   "image_id": "ami-mi355x", "instance_type": "mi355x.48xlarge",
                                   "agent_command": native_binary("det-agent"),
                                   "agent_args": ["--artificial-slots", "1", "--python", sys.executable, "--work-dir",
                                                  str(tmp_path / "agentwork"), "--framework-root", REPO]}}}
    conf = tmp_path / "master.json"
    conf.write_text(json.dumps(cfg))
    try:
        with LocalCluster(agents=0, log_dir=str(tmp_path), tick_ms=50, master_args=["--config-file", str(conf)]) as c:
            cl = MasterClient(c.address)
            eid = cl.create_experiment({"description": "prov", "entrypoint": "model_def:NoOpTrial",
                                        "hyperparameters": {"global_batch_size": 4, "metrics_base": 0.9},
                                        "searcher": {"name": "single", "metric": "validation_error",
                                                     "max_length": {"batches": 10}},
                                        "scheduling_unit": 5}, read_context(NOOP))["id"]
            assert cl.wait_for_experiment(eid, timeout=180) == "COMPLETED", open(tmp_path / "master.log").read()[-3000:]
            assert "RunInstances" in ec2.calls
            launched = list(ec2.instances)
            assert len(launched) == 1
            inst = ec2.instances[launched[0]]
            assert inst["tags"]["determined-resource-pool"].endswith("-default")
            assert "--agent-id" in inst["script"]
            deadline = time.time() + 30  # idle instance is terminated after max_idle_agent_period
            while time.time() < deadline and inst["state"] != "terminated":
                time.sleep(0.2)
            assert inst["state"] == "terminated" and "TerminateInstances" in ec2.calls
    finally:
        ec2.close()


def test_gcp_provider_against_fake_compute(tmp_path):
    TOKEN = "ya29.gce"
    state = {"instances": {}}

    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a):
            pass

        def _send(self, code, obj):
            b = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(b)))
            self.end_headers()
            self.wfile.write(b)

        def _ok(self):
            if self.headers.get("Authorization") != f"Bearer {TOKEN}":
                self._send(401, {"error": "auth"})
                return False
            return "/compute/v1/projects/p1/zones/z1/instances" in self.path

        def do_POST(self):
            if not self._ok():
                return
            body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
            state["instances"][body["name"]] = dict(body, status="PROVISIONING")
            self._send(200, {"kind": "compute#operation", "status": "RUNNING"})

        def do_GET(self):
            if not self._ok():
                return
            q = dict(urllib.parse.parse_qsl(urllib.parse.urlsplit(self.path).query))
            want = q["filter"].split("=", 1)[1]
            items = [{"name": n, "status": d["status"]} for n, d in state["instances"].items()
                     if d["labels"]["determined-pool"] == want]
            self._send(200, {"items": items})

        def do_DELETE(self):
            if not self._ok():
                return
            state["instances"].pop(self.path.rsplit("/", 1)[1], None)
            self._send(200, {"kind": "compute#operation"})

    srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        prov = build({"provider": "gcp", "cluster_id": "c1",
                      "gcp": {"endpoint_url": f"http://127.0.0.1:{srv.server_address[1]}", "project": "p1",
                              "zone": "z1", "image": "projects/p/global/images/rocm", "token": TOKEN}},
                     "default", "10.0.0.2", 8080)
        assert isinstance(prov, GCPProvider)
        names = prov.launch(2)
        assert len(names) == 2 and all(n.startswith("det-default-") for n in names)
        inst = state["instances"][names[0]]
        script = inst["metadata"]["items"][0]["value"]
        assert "--master-host 10.0.0.2 --master-port 8080" in script and "$(hostname)" in script
        assert {i["id"] for i in prov.list()} == set(names)
        assert all(i["state"] == "Starting" for i in prov.list())
        prov.terminate([names[0]])
        assert [i["id"] for i in prov.list()] == [names[1]]
    finally:
        srv.shutdown()


def test_det_deploy_aws_up_runs_experiment_and_down(tmp_path):
    """`det deploy aws up`: the master VM's user-data starts det-master with the AWS provisioner;
    the master then provisions its own agent VM for a pending trial; `down` terminates both."""
    from determined_1_amd.deploy.local import free_port

    ec2 = FakeEC2(str(tmp_path))
    port = free_port()
    prov_cfg = {"endpoint_url": ec2.url, "region": "us-west-2", "access_key": AK, "secret_key": SK,
                "instance_metadata_url": ec2.url,
                "image_id": "ami-mi355x", "agent_command": native_binary("det-agent"),
                "agent_args": ["--artificial-slots", "1", "--python", sys.executable, "--work-dir",
                               str(tmp_path / "agentwork"), "--framework-root", REPO]}
    base = [sys.executable, "-m", "determined_1_amd.cli", "deploy", "aws"]
    common = ["--cluster-id", "c1", "--provider-config", json.dumps(prov_cfg)]
    try:
        r = subprocess.run(base + ["up"] + common + [
            "--master-command", f"{native_binary('det-master')} --host 127.0.0.1 --python {sys.executable}",
            "--master-port", str(port), "--store-dir", str(tmp_path / "store"), "--slots-per-agent", "1",
            "--max-agents", "1", "--max-idle-agent-period-ms", "1500",
            "--checkpoint-storage", json.dumps({"type": "shared_fs", "host_path": str(tmp_path / "ckpt")})],
            capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        masters = json.loads(r.stdout)["master_instances"]
        assert len(masters) == 1 and ec2.instances[masters[0]]["tags"]["determined-cluster"] == "c1"
        cl = MasterClient(f"127.0.0.1:{port}")
        deadline = time.time() + 30
        while time.time() < deadline:
            try:
                cl.get("/info")
                break
            except Exception:
                time.sleep(0.2)
        eid = cl.create_experiment({"description": "deploy", "entrypoint": "model_def:NoOpTrial",
                                    "hyperparameters": {"global_batch_size": 4, "metrics_base": 0.9},
                                    "searcher": {"name": "single", "metric": "validation_error",
                                                 "max_length": {"batches": 5}}, "scheduling_unit": 5},
                                   read_context(NOOP))["id"]
        assert cl.wait_for_experiment(eid, timeout=180) == "COMPLETED"
        agents = [i for i, d in ec2.instances.items() if d["tags"].get("determined-resource-pool") == "c1-default"]
        assert len(agents) == 1
        assert ec2.imds_reads >= 1  # the master signed with its instance-profile credentials
        r = subprocess.run(base + ["down"] + common, capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        assert set(json.loads(r.stdout)["terminated"]) >= set(masters)
        assert all(d["state"] == "terminated" for d in ec2.instances.values())
    finally:
        ec2.close()


def test_deploy_master_script_never_embeds_credentials():
    """--provider-config credentials stay with the deploying client; the master VM's
    user-data (readable via instance metadata) carries none of them."""
    import argparse

    from determined_1_amd.deploy import cloud_deploy

    args = argparse.Namespace(provider="aws", max_agents=2, slots_per_agent=8, max_idle_agent_period_ms=1000,
                              master_port=8080, store_dir="/var/det", checkpoint_storage='{"type": "shared_fs"}',
                              startup_script="", master_command="det-master", cluster_id="c1")
    cfg = {"region": "us-east-1", "access_key": "AKIDSECRET1", "secret_key": "SKSECRET2",
           "session_token": "STSECRET3", "image_id": "ami-1"}
    script = cloud_deploy.master_script(args, cfg)
    for secret in ("AKIDSECRET1", "SKSECRET2", "STSECRET3"):
        assert secret not in script
    assert "ami-1" in script and "us-east-1" in script
