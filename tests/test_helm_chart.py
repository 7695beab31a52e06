"""Helm chart (deploy/helm/determined-mi355x; reference helm/charts/determined): the templates
render to valid Kubernetes objects, and the master config the chart ships boots a real det-master
whose Kubernetes resource manager finds the cluster's AMD GPUs (fake API server standing in for
the kubectl-proxy sidecar)."""
import json
import pathlib
import re
import subprocess
import time

import requests
import yaml

from determined_1_amd.deploy.local import free_port, native_binary
from tests.fake_kube import FakeKube

CHART = pathlib.Path(__file__).resolve().parent.parent / "deploy" / "helm" / "determined-mi355x"


def render(release="det", namespace="ml"):
    values = yaml.safe_load((CHART / "values.yaml").read_text())

    def lookup(path):
        v = values
        for k in path.split("."):
            v = v[k]
        return str(v)

    out = {}
    for f in sorted((CHART / "templates").glob("*.yaml")):
        text = f.read_text()
        text = re.sub(r"\{\{\s*\.Values\.([\w.]+)\s*\}\}", lambda m: lookup(m.group(1)), text)
        text = text.replace("{{ .Release.Name }}", release).replace("{{ .Release.Namespace }}", namespace)
        assert "{{" not in text, f"unrendered template in {f.name}"
        out[f.name] = [d for d in yaml.safe_load_all(text) if d]
    return out


def test_chart_renders_valid_objects():
    docs = render()
    kinds = sorted(d["kind"] for ds in docs.values() for d in ds)
    assert kinds == sorted(["ConfigMap", "ServiceAccount", "Role", "RoleBinding", "ClusterRole", "ClusterRoleBinding",
                            "PersistentVolumeClaim", "Deployment", "Service"])
    dep = next(d for d in docs["master-deployment.yaml"] if d["kind"] == "Deployment")
    names = [c["name"] for c in dep["spec"]["template"]["spec"]["containers"]]
    assert names == ["determined-master", "kubectl-proxy"]
    role = next(d for d in docs["master-permissions.yaml"] if d["kind"] == "Role")
    assert {"pods", "pods/log", "configmaps"} <= set(role["rules"][0]["resources"])


def test_chart_master_config_boots_master_with_kubernetes_rm(tmp_path):
    cm = render()["master-config.yaml"][0]
    cfg = json.loads(cm["data"]["master.json"])
    assert cfg["resource_manager"]["type"] == "kubernetes"
    assert cfg["resource_manager"]["slot_resource"] == "amd.com/gpu"
    with FakeKube(nodes=1, gpus_per_node=8) as kube:
        port = free_port()
        cfg.update(port=port, store_dir=str(tmp_path / "store"))
        cfg["resource_manager"]["api_server"] = kube.address
        cfg["resource_manager"]["master_service_host"] = "127.0.0.1"
        cfg["checkpoint_storage"]["host_path"] = str(tmp_path / "ckpt")
        (tmp_path / "master.json").write_text(json.dumps(cfg))
        log = open(tmp_path / "master.log", "wb")
        p = subprocess.Popen([native_binary("det-master"), "--config-file", str(tmp_path / "master.json"),
                              "--host", "127.0.0.1"], stdout=log, stderr=subprocess.STDOUT)
        try:
            deadline = time.time() + 30
            agents = []
            while time.time() < deadline:
                try:
                    agents = requests.get(f"http://127.0.0.1:{port}/agents", timeout=2).json()
                    if agents:
                        break
                except requests.RequestException:
                    pass
                time.sleep(0.2)
            assert [a["id"] for a in agents] == ["k8s-node-0-0"], (tmp_path / "master.log").read_text()[-2000:]
            assert len(agents[0]["slots"]) == 8
            assert requests.get(f"http://127.0.0.1:{port}/det/", timeout=5).status_code == 200
        finally:
            p.terminate()
            p.wait(timeout=20)
