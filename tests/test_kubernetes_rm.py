"""Kubernetes resource manager (native/src/kubernetes.cc; reference
master/internal/resourcemanagers/kubernetes_resource_manager.go + master/internal/kubernetes/)
against tests/fake_kube.py: node capacity -> virtual agents, trials and commands as pods
(ConfigMap spec + pod_entrypoint), pod phases -> container states, pod logs -> trial logs,
max_slots_per_pod splitting a multi-slot trial into one pod per rank, kill -> pod deletion."""
import os
import pathlib
import time

import pytest

from determined_1_amd.api import MasterClient, read_context
from determined_1_amd.deploy import LocalCluster
from tests.fake_kube import FakeKube

REPO = str(pathlib.Path(__file__).resolve().parent.parent)
NOOP = pathlib.Path(__file__).resolve().parent / "fixtures" / "no_op"


def _cfg(searcher, **extra):
    cfg = {"description": "k8s", "entrypoint": "model_def:NoOpTrial",
           "hyperparameters": {"global_batch_size": 4, "metrics_base": 0.9},
           "searcher": dict(searcher, metric="validation_error"), "scheduling_unit": 5, "max_restarts": 0}
    cfg.update(extra)
    return cfg


def _cluster(tmp_path, kube, slot_type="cpu", per_pod=8, cpu_slots=1):
    args = ["--kubernetes-api", kube.address, "--kubernetes-namespace", "det", "--kubernetes-slot-type", slot_type,
            "--kubernetes-max-slots-per-pod", str(per_pod), "--kubernetes-cpu-slots-per-node", str(cpu_slots),
            "--kubernetes-master-host", "127.0.0.1"]
    return LocalCluster(agents=0, store_dir=str(tmp_path / "store"), checkpoint_dir=str(tmp_path / "ckpt"),
                        log_dir=str(tmp_path), tick_ms=50, master_args=args)


def test_virtual_agents_from_node_capacity(tmp_path):
    with FakeKube(nodes=2, gpus_per_node=8) as kube, _cluster(tmp_path, kube, slot_type="gpu", per_pod=4) as c:
        agents = MasterClient(c.address).get("/agents")
        # 2 nodes x 8 GPUs, max 4 per pod -> 4 virtual agents of 4 slots
        assert sorted(a["id"] for a in agents) == ["k8s-node-0-0", "k8s-node-0-1", "k8s-node-1-0", "k8s-node-1-1"]
        assert all(len(a["slots"]) == 4 for a in agents)


def test_trial_runs_as_pod_with_logs_and_checkpoints(tmp_path):
    with FakeKube(nodes=1, extra_env={"PYTHONPATH": REPO}) as kube, _cluster(tmp_path, kube, cpu_slots=2) as c:
        cl = MasterClient(c.address)
        eid = cl.create_experiment(_cfg({"name": "single", "max_length": {"batches": 10}}), read_context(NOOP))["id"]
        assert cl.wait_for_experiment(eid, timeout=180) == "COMPLETED", open(tmp_path / "master.log").read()[-3000:]
        t = cl.experiment(eid)["trials"][0]
        assert t["state"] == "COMPLETED" and t["total_batches_processed"] == 10
        pod = kube.created[0]
        assert pod["metadata"]["name"].startswith(f"exp-{eid}-trial-{t['id']}-rank-0-")
        assert pod["spec"]["restartPolicy"] == "Never"
        assert pod["spec"]["nodeSelector"] == {"kubernetes.io/hostname": "node-0"}
        cmd = pod["spec"]["containers"][0]["command"]
        assert cmd[:3] == ["python3", "-m", "determined_1_amd.exec.pod_entrypoint"]
        env = {e["name"]: e["value"] for e in pod["spec"]["containers"][0]["env"]}
        assert env["DET_USE_GPU"] == "false" and env["DET_EXPERIMENT_ID"] == str(eid)
        logs = [l["message"] for l in cl.trial_logs(t["id"])]
        assert any("running" in m and "harness" in m for m in logs), logs[:10]  # pod_entrypoint line
        assert any("saved checkpoint" in m for m in logs)
        deadline = time.time() + 20  # finished pods and their ConfigMaps are cleaned up
        while time.time() < deadline and (kube.pods or kube.configmaps):
            time.sleep(0.1)
        assert not kube.pods and not kube.configmaps


def test_multi_slot_trial_splits_into_pods(tmp_path):
    with FakeKube(nodes=2, extra_env={"PYTHONPATH": REPO}) as kube, _cluster(tmp_path, kube, per_pod=1, cpu_slots=1) as c:
        cl = MasterClient(c.address)
        cfg = _cfg({"name": "single", "max_length": {"batches": 10}}, resources={"slots_per_trial": 2})
        eid = cl.create_experiment(cfg, read_context(NOOP))["id"]
        assert cl.wait_for_experiment(eid, timeout=240) == "COMPLETED", open(tmp_path / "master.log").read()[-3000:]
        names = sorted(p["metadata"]["name"] for p in kube.created)
        assert len(names) == 2 and "-rank-0-" in names[0] and "-rank-1-" in names[1]
        assert {p["spec"]["nodeSelector"]["kubernetes.io/hostname"] for p in kube.created} == {"node-0", "node-1"}


def test_kill_deletes_pod(tmp_path):
    with FakeKube(nodes=1, extra_env={"PYTHONPATH": REPO}) as kube, _cluster(tmp_path, kube) as c:
        cl = MasterClient(c.address)
        cfg = _cfg({"name": "single", "max_length": {"batches": 100000}},
                   hyperparameters={"global_batch_size": 4, "metrics_base": 0.9, "sleep": 0.05})
        eid = cl.create_experiment(cfg, read_context(NOOP))["id"]
        deadline = time.time() + 60
        while time.time() < deadline and not any(p["status"].get("phase") == "Running" for p in kube.pods.values()):
            time.sleep(0.1)
        assert kube.pods, "pod never started"
        cl.post(f"/experiments/{eid}/kill")
        assert cl.wait_for_experiment(eid, timeout=60) == "CANCELED"
        assert kube.deleted
        deadline = time.time() + 20
        while time.time() < deadline and kube.pods:
            time.sleep(0.1)
        assert not kube.pods


def test_gpu_pod_requests_amd_gpus(tmp_path):
    with FakeKube(nodes=1, gpus_per_node=8) as kube, _cluster(tmp_path, kube, slot_type="gpu", per_pod=8) as c:
        cl = MasterClient(c.address)
        cfg = _cfg({"name": "single", "max_length": {"batches": 10}}, resources={"slots_per_trial": 4})
        eid = cl.create_experiment(cfg, read_context(NOOP))["id"]
        deadline = time.time() + 60
        while time.time() < deadline and not kube.created:
            time.sleep(0.1)
        assert kube.created
        c0 = kube.created[0]["spec"]["containers"][0]
        assert c0["resources"]["limits"] == {"amd.com/gpu": "4"} and c0["resources"]["requests"] == {"amd.com/gpu": "4"}
        env = {e["name"]: e["value"] for e in c0["env"]}
        assert env["DET_USE_GPU"] == "true" and env["DET_SLOT_IDS"] == "[0,1,2,3]"
        cl.post(f"/experiments/{eid}/kill")
        cl.wait_for_experiment(eid, timeout=60)


def test_pod_runs_as_the_owners_agent_user_group(tmp_path):
    """Agent user groups on the Kubernetes RM: the pod's container securityContext carries the
    experiment owner's linked uid/gid (the default account of security.default_agent_user_group
    here, as the experiment is created without a session)."""
    cfgfile = tmp_path / "master.yaml"
    cfgfile.write_text("security:\n  default_agent_user_group: {uid: 1234, gid: 5678, user: u, group: g}\n")
    with FakeKube(nodes=1) as kube:
        args = ["--kubernetes-api", kube.address, "--kubernetes-namespace", "det", "--kubernetes-slot-type", "cpu",
                "--kubernetes-max-slots-per-pod", "8", "--kubernetes-cpu-slots-per-node", "1",
                "--kubernetes-master-host", "127.0.0.1", "--config-file", str(cfgfile)]
        with LocalCluster(agents=0, store_dir=str(tmp_path / "store"), checkpoint_dir=str(tmp_path / "ckpt"),
                          log_dir=str(tmp_path), tick_ms=50, master_args=args) as c:
            cl = MasterClient(c.address)
            eid = cl.create_experiment(_cfg({"name": "single", "max_length": {"batches": 10}}), read_context(NOOP))["id"]
            deadline = time.time() + 60
            while time.time() < deadline and not kube.created:
                time.sleep(0.1)
            assert kube.created
            sc = kube.created[0]["spec"]["containers"][0]["securityContext"]
            assert sc == {"runAsUser": 1234, "runAsGroup": 5678}
            cl.post(f"/experiments/{eid}/kill")
            cl.wait_for_experiment(eid, timeout=60)
