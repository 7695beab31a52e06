"""Agent user groups (reference master/internal/user/service.go:22-45,272-290,
master/pkg/model/agent_user_group.go, master/pkg/tasks/task.go:60-100, cli/determined_cli/user.py:
165-234): an admin links a user to a host account with ``det user link-with-agent-user``; that
user's tasks -- trials and commands -- run on the agents as uid:gid, with passwd/group entries for
the account in the task's work dir; users without a link run as the master's
``security.default_agent_user_group`` (else as the agent's own account).  Needs root (setuid)."""
import json
import os
import pathlib
import subprocess
import sys
import time

import pytest

from determined_1_amd.api import MasterClient, read_context
from determined_1_amd.deploy import LocalCluster

pytestmark = pytest.mark.skipif(os.geteuid() != 0, reason="switching the task's uid needs a root det-agent")
NOOP = pathlib.Path(__file__).resolve().parent / "fixtures" / "no_op"
PROBE = ("import os, json; print('IDS ' + json.dumps({'uid': os.getuid(), 'gid': os.getgid(), "
         "'user': os.environ.get('USER'), 'passwd': open(os.environ['DET_TASK_ETC'] + '/passwd').read() "
         "if os.environ.get('DET_TASK_ETC') else None}), flush=True)")


def _cmd_ids(client, timeout=60):
    cid = client.post("/commands", {"config": {"entrypoint": [sys.executable, "-c", PROBE], "resources": {"slots": 0},
                                               "description": "whoami"}, "context": []})["id"]
    deadline = time.time() + timeout
    while time.time() < deadline:
        if client.get(f"/commands/{cid}")["state"] == "TERMINATED":
            break
        time.sleep(0.2)
    logs = client.get(f"/commands/{cid}/logs") if True else []
    lines = [l.get("message", l.get("log", "")) for l in logs]
    hit = [l for l in lines if l.startswith("IDS ")]
    assert hit, lines[-20:]
    return json.loads(hit[-1][4:])


def test_linked_and_default_agent_users(tmp_path):
    cfg = tmp_path / "master.yaml"
    cfg.write_text("security:\n  authentication: true\n  default_agent_user_group:\n"
                   "    uid: 4322\n    gid: 4322\n    user: det-default\n    group: det-default\n")
    # tasks import the framework and write checkpoints as their own account: a world-readable copy
    # of the package (this checkout and pytest's tmp dirs are private to root), as an installed
    # package would be, and a world-writable checkpoint dir
    import shutil
    import tempfile

    base = pathlib.Path(tempfile.mkdtemp(prefix="det-aug-"))
    request_cleanup = lambda: shutil.rmtree(base, ignore_errors=True)  # noqa: E731
    ckpt = base / "ckpt"
    ckpt.mkdir()
    fw = base / "fw"
    shutil.copytree(pathlib.Path(__file__).resolve().parent.parent / "determined_1_amd", fw / "determined_1_amd",
                    ignore=shutil.ignore_patterns("__pycache__", "miopen_db", "_native", "build"))
    for p in [base, fw] + list(fw.rglob("*")):
        os.chmod(p, 0o755 if p.is_dir() else 0o644)
    os.chmod(ckpt, 0o777)
    try:
        _run_cluster(tmp_path, cfg, ckpt, fw)
    finally:
        request_cleanup()


def _run_cluster(tmp_path, cfg, ckpt, fw):
    with LocalCluster(agents=1, slots_per_agent=1, log_dir=str(tmp_path), tick_ms=50, checkpoint_dir=str(ckpt),
                      master_args=["--config-file", str(cfg)], framework_root=str(fw)) as c:
        admin = MasterClient(c.address)
        admin.login("admin", "")
        admin.post("/users", {"username": "alice", "password": "pw"})
        admin.post("/users", {"username": "bob", "password": "pw"})
        # the CLI (admin): det user link-with-agent-user alice ...
        env = dict(os.environ, DET_MASTER=c.address, DET_USER_TOKEN=admin.session.headers["Authorization"][7:])
        r = subprocess.run([sys.executable, "-m", "determined_1_amd.cli", "user", "link-with-agent-user", "alice",
                            "--agent-uid", "4321", "--agent-user", "alice-host", "--agent-gid", "4321",
                            "--agent-group", "alice-grp"], capture_output=True, text=True, timeout=60, env=env)
        assert r.returncode == 0, r.stderr
        users = {u["username"]: u for u in admin.get("/users")}
        assert users["alice"]["agent_user_group"] == {"uid": 4321, "gid": 4321, "user": "alice-host",
                                                      "group": "alice-grp"}
        # only an admin may link; invalid groups are refused
        alice = MasterClient(c.address)
        alice.session.headers["Authorization"] = "Bearer " + alice.post("/login", {"username": "alice",
                                                                                    "password": "pw"})["token"]
        with pytest.raises(Exception, match="403"):
            alice.patch("/users/bob", {"agent_user_group": {"uid": 0, "gid": 0, "user": "root", "group": "root"}})
        with pytest.raises(Exception, match="400"):
            admin.patch("/users/bob", {"agent_user_group": {"uid": -1, "gid": 0, "user": "x", "group": "x"}})

        ids = _cmd_ids(alice)
        assert (ids["uid"], ids["gid"], ids["user"]) == (4321, 4321, "alice-host"), ids
        assert ids["passwd"].startswith("alice-host:x:4321:4321:")
        bob = MasterClient(c.address)
        bob.session.headers["Authorization"] = "Bearer " + bob.post("/login", {"username": "bob",
                                                                                "password": "pw"})["token"]
        ids = _cmd_ids(bob)  # unlinked: the master's default account
        assert (ids["uid"], ids["gid"], ids["user"]) == (4322, 4322, "det-default"), ids

        # a trial of alice's experiment runs as her account too (harness through the zygote)
        exp = {"description": "aug", "entrypoint": "model_def:NoOpTrial",
               "hyperparameters": {"global_batch_size": 4, "metrics_base": 0.9},
               "searcher": {"name": "single", "metric": "validation_error", "max_length": {"batches": 2}},
               "scheduling_unit": 1,
               "environment": {"environment_variables": ["DET_PRINT_UID=1"]}}
        eid = alice.create_experiment(exp, read_context(NOOP))["id"]
        state = alice.wait_for_experiment(eid, timeout=180)
        if state != "COMPLETED":
            t = alice.experiment(eid)["trials"]
            msg = "\n".join(l["message"] for l in alice.get(f"/trials/{t[0]['id']}/logs"))[-3000:] if t else ""
            pytest.fail(f"experiment {state}: {msg}")
        assert admin.experiment(eid)["owner"] == "alice"
        tid = alice.experiment(eid)["trials"][0]["id"]
        logs = "\n".join(l["message"] for l in alice.get(f"/trials/{tid}/logs"))
        assert "trial process uid=4321 gid=4321" in logs, logs[-2000:]
