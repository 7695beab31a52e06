"""Shell tasks (det shell start/open; exec/shell.py): a bash on a pty inside a command task,
reached through the master's /proxy with a per-shell token; exit status propagates; a wrong token
is refused; notebook tasks fail loudly when Jupyter is absent."""
import os
import re
import subprocess
import sys

import pytest
import requests

from determined_1_amd.api import MasterClient
from determined_1_amd.deploy import LocalCluster


@pytest.fixture(scope="module")
def cluster(tmp_path_factory):
    d = tmp_path_factory.mktemp("shell")
    with LocalCluster(agents=1, slots_per_agent=1, log_dir=str(d), tick_ms=50) as c:
        yield c


def _det(c, home, *argv, stdin=None, timeout=120):
    env = dict(os.environ, HOME=str(home))
    return subprocess.run([sys.executable, "-m", "determined_1_amd.cli", "-m", c.address, *argv], input=stdin,
                          capture_output=True, text=True, timeout=timeout, env=env)


def test_shell_roundtrip_and_exit_code(cluster, tmp_path):
    r = _det(cluster, tmp_path, "shell", "start", "-d")
    assert r.returncode == 0, r.stderr
    sid = int(re.search(r"Shell (\d+) ready", r.stderr).group(1))
    r = _det(cluster, tmp_path, "shell", "open", str(sid), stdin="echo hello-$((2+3)); exit 3\n")
    assert "hello-5" in r.stdout, (r.stdout, r.stderr)
    assert r.returncode == 3
    # token guard: the proxied API refuses a wrong token
    bad = requests.get(f"http://{cluster.address}/proxy/cmd-{sid}/status", params={"token": "nope"}, timeout=10)
    assert bad.status_code in (403, 404)  # 404 once the task has exited
    other_home = tmp_path / "other"
    other_home.mkdir()
    r = _det(cluster, other_home, "shell", "open", str(sid))
    assert r.returncode != 0 and "no token" in r.stderr


def test_notebook_without_jupyter_fails_loudly(cluster, tmp_path):
    try:
        import jupyter_server  # noqa: F401
        pytest.skip("jupyter is installed here")
    except ImportError:
        pass
    r = _det(cluster, tmp_path, "notebook", "start", "--slots", "0", "--timeout", "30")
    assert r.returncode != 0 and "neither jupyter_server nor notebook is installed" in r.stderr
    rows = MasterClient(cluster.address).get("/commands", type="notebook")
    assert rows and rows[-1]["state"] == "TERMINATED"


def test_shell_token_never_returned_by_the_api(cluster, tmp_path):
    """The per-shell token reaches only the task's environment: no command/shell listing returns it
    (it used to sit in environment.environment_variables of the stored config)."""
    r = _det(cluster, tmp_path, "shell", "start", "-d")
    assert r.returncode == 0, r.stderr
    sid = int(re.search(r"Shell (\d+) ready", r.stderr).group(1))
    import json

    token_file = tmp_path / ".det-mi355x" / ("shells-" + cluster.address.replace(":", "_") + ".json")
    token = json.loads(token_file.read_text())[str(sid)]
    client = MasterClient(cluster.address)
    bodies = [client.get("/commands"), client.get(f"/commands/{sid}"),
              requests.get(f"http://{cluster.address}/api/v1/shells", timeout=10).text,
              requests.get(f"http://{cluster.address}/api/v1/shells/{sid}", timeout=10).text]
    for b in bodies:
        assert token not in (b if isinstance(b, str) else json.dumps(b))
    # ... and the shell still authenticates with it
    ok = requests.get(f"http://{cluster.address}/proxy/cmd-{sid}/status", params={"token": token}, timeout=10)
    assert ok.status_code == 200, ok.text
    client.post(f"/commands/{sid}/kill")
