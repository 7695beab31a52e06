"""``det tunnel`` (reference cli/determined_cli/tunnel.py): a command task runs a raw TCP echo
service (not HTTP) and reports its port; the master splices a WebSocket upgrade of /proxy/cmd-<id>/
onto a TCP connection to it.  Checked: binary-safe round trips of every byte value through the
--listen forwarder (two concurrent connections), the stdio mode as a subprocess (the ssh
ProxyCommand usage), and a refused tunnel to a service that is not ready."""
import os
import socket
import subprocess
import sys
import threading
import time

import pytest

from determined_1_amd.api import MasterClient
from determined_1_amd.cli import tunnel
from determined_1_amd.deploy import LocalCluster
from determined_1_amd.harness._ws import WebSocketError

ECHO = r"""
import os, socket, threading
from determined_1_amd.api.request import MasterClient
srv = socket.socket(); srv.bind(("127.0.0.1", 0)); srv.listen(8)
def serve(c):
    while True:
        b = c.recv(65536)
        if not b:
            break
        c.sendall(b[::-1])  # reversed, so an echo of the wrong bytes cannot pass
    c.close()
MasterClient(os.environ["DET_MASTER"]).post("/commands/%s/ready" % os.environ["DET_TASK_ID"][4:],
                                            {"port": srv.getsockname()[1]})
print("echo ready", flush=True)
while True:
    c, _ = srv.accept()
    threading.Thread(target=serve, args=(c,), daemon=True).start()
"""


@pytest.fixture(scope="module")
def cluster(tmp_path_factory):
    d = tmp_path_factory.mktemp("tunnel")
    with LocalCluster(agents=1, slots_per_agent=1, log_dir=str(d), tick_ms=50) as c:
        yield c


@pytest.fixture(scope="module")
def echo_cmd(cluster):
    client = MasterClient(cluster.address)
    cid = client.post("/commands", {"config": {"entrypoint": [sys.executable, "-c", ECHO], "resources": {"slots": 0},
                                               "description": "tcp echo"}, "context": []})["id"]
    deadline = time.time() + 60
    while time.time() < deadline:
        c = client.get(f"/commands/{cid}")
        if c.get("service_address"):
            break
        assert c["state"] != "TERMINATED", c
        time.sleep(0.2)
    else:
        pytest.fail("echo service never became ready")
    yield cid
    client.post(f"/commands/{cid}/kill")


def _roundtrip(port, payload):
    s = socket.create_connection(("127.0.0.1", port), timeout=20)
    got = b""
    for i in range(0, len(payload), 4096):  # the echo reverses per recv chunk: send in fixed pieces
        piece = payload[i:i + 4096]
        s.sendall(piece)
        buf = b""
        while len(buf) < len(piece):
            b = s.recv(65536)
            assert b, "tunnel closed early"
            buf += b
        got += buf[::-1]
    s.close()
    return got


def test_listen_mode_binary_roundtrip(cluster, echo_cmd):
    ready, stop = threading.Event(), threading.Event()
    t = threading.Thread(target=tunnel.tunnel_listen, args=(cluster.address, str(echo_cmd), 0),
                         kwargs={"ready": ready, "stop": stop}, daemon=True)
    t.start()
    assert ready.wait(10)
    payload = bytes(range(256)) * 64  # every byte value, 16 KiB
    results = {}

    def worker(k):
        results[k] = _roundtrip(ready.port, payload)

    ws = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for w in ws:
        w.start()
    for w in ws:
        w.join(60)
    stop.set()
    t.join(5)
    assert results == {0: payload, 1: payload}


def test_stdio_mode_subprocess(cluster, echo_cmd):
    data = b"det-tunnel\x00\xff\n"
    p = subprocess.run([sys.executable, "-m", "determined_1_amd.cli.tunnel", cluster.address, f"cmd-{echo_cmd}"],
                       input=data, capture_output=True, timeout=60,
                       env=dict(os.environ, PYTHONPATH=os.pathsep.join(sys.path)))
    assert p.stdout == data[::-1], (p.stdout, p.stderr)


def test_tunnel_to_missing_service_is_refused(cluster):
    with pytest.raises((WebSocketError, OSError)):
        ws = tunnel.open_tunnel(cluster.address, "cmd-999999")
        # the master accepts the upgrade only to close it at once: the first read sees the close
        if ws.recv_bytes() is None:
            raise WebSocketError("closed")


def test_tunnel_requires_a_session_under_require_auth(tmp_path):
    """the tunnel's WebSocket upgrade is gated like /proxy -- without a session token the
    master answers 401 before switching protocols; with the CLI's token the stream works."""
    with LocalCluster(agents=1, slots_per_agent=1, log_dir=str(tmp_path), tick_ms=50,
                      master_args=["--require-auth"]) as c:
        client = MasterClient(c.address)
        tok = client.login("determined", "")
        cid = client.post("/commands", {"config": {"entrypoint": [sys.executable, "-c", ECHO], "resources": {"slots": 0},
                                                   "description": "tcp echo"}, "context": [],
                                        "secret_environment": [f"DET_USER_TOKEN={tok}"]})["id"]
        deadline = time.time() + 60
        while time.time() < deadline and not client.get(f"/commands/{cid}").get("service_address"):
            time.sleep(0.2)
        try:
            with pytest.raises(WebSocketError, match="401"):
                tunnel.open_tunnel(c.address, f"cmd-{cid}", token="")
            with pytest.raises(WebSocketError, match="401"):
                tunnel.open_tunnel(c.address, f"cmd-{cid}", token="not-a-session")
            ws = tunnel.open_tunnel(c.address, f"cmd-{cid}", token=tok)
            ws.send_binary(b"abc")
            assert ws.recv_bytes() == b"cba"
            ws.close()
        finally:
            client.post(f"/commands/{cid}/kill")
