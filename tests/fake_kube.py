"""In-process fake Kubernetes API server + kubelet for the Kubernetes resource manager tests
(the reference tests its pod logic against a mocked client, master/internal/kubernetes/
mock_client_test.go; this goes one step further and actually runs the pods).

Implements the REST subset the master uses (plain HTTP, like ``kubectl proxy``):
  GET    /api/v1/nodes
  POST   /api/v1/namespaces/{ns}/configmaps        DELETE .../configmaps/{name}
  POST   /api/v1/namespaces/{ns}/pods              GET .../pods?labelSelector=k=v
  GET    /api/v1/namespaces/{ns}/pods/{name}       DELETE .../pods/{name}
  GET    /api/v1/namespaces/{ns}/pods/{name}/log?follow=true   (chunked)
The "kubelet" materialises ConfigMap volumes under a per-pod root (env values pointing into a
mount path are rewritten to it), starts the container command as a local process group with the
pod's env and working directory, and moves the pod Pending -> Running -> Succeeded/Failed.
"""
import json
import os
import pathlib
import re
import shutil
import signal
import subprocess
import sys
import tempfile
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional
from urllib.parse import parse_qs, urlparse


class FakeKube:
    def __init__(self, nodes: int = 1, gpus_per_node: int = 2, resource: str = "amd.com/gpu",
                 extra_env: Optional[Dict[str, str]] = None, start_delay: float = 0.2) -> None:
        self.nodes = [{"metadata": {"name": f"node-{i}", "labels": {"kubernetes.io/hostname": f"node-{i}"}},
                       "spec": {}, "status": {"allocatable": {resource: str(gpus_per_node), "cpu": "8"}}}
                      for i in range(nodes)]
        self.pods: Dict[str, Dict[str, Any]] = {}
        self.configmaps: Dict[str, Dict[str, Any]] = {}
        self.procs: Dict[str, subprocess.Popen] = {}
        self.lock = threading.Lock()
        self.root = pathlib.Path(tempfile.mkdtemp(prefix="fake-kube-"))
        self.extra_env = dict(extra_env or {})
        self.start_delay = start_delay
        self.created: List[Dict[str, Any]] = []  # every pod spec ever posted (assertions)
        self.deleted: List[str] = []
        self.server = ThreadingHTTPServer(("127.0.0.1", 0), self._handler())
        self.server.daemon_threads = True
        self.thread = threading.Thread(target=self.server.serve_forever, daemon=True)

    @property
    def address(self) -> str:
        return f"127.0.0.1:{self.server.server_address[1]}"

    def __enter__(self) -> "FakeKube":
        self.thread.start()
        return self

    def __exit__(self, *exc: Any) -> None:
        self.server.shutdown()
        with self.lock:
            procs = list(self.procs.values())
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        shutil.rmtree(self.root, ignore_errors=True)

    # --------------------------------------------------------------------------- kubelet
    def _run_pod(self, name: str) -> None:
        time.sleep(self.start_delay)
        with self.lock:
            pod = self.pods.get(name)
            if pod is None:
                return
        c = pod["spec"]["containers"][0]
        proot = self.root / name
        mounts = {}
        for vol in pod["spec"].get("volumes", []):
            cm = self.configmaps.get(vol.get("configMap", {}).get("name", ""))
            vdir = proot / "volumes" / vol["name"]
            vdir.mkdir(parents=True, exist_ok=True)
            for k, v in (cm or {}).get("data", {}).items():
                (vdir / k).write_text(v)
            mounts[vol["name"]] = vdir
        remap = {}
        for vm in c.get("volumeMounts", []):
            remap[vm["mountPath"]] = str(mounts[vm["name"]])
        workdir = proot / "workdir"
        workdir.mkdir(parents=True, exist_ok=True)
        env = {k: v for k, v in os.environ.items() if k in ("PATH", "HOME", "LANG", "TMPDIR", "PYTHONPATH")}
        env.update(self.extra_env)
        for e in c.get("env", []):
            v = e.get("value", "")
            for mp, real in remap.items():
                if v.startswith(mp):
                    v = real + v[len(mp):]
            env[e["name"]] = v
        env["DET_WORKDIR"] = str(workdir)
        log = open(proot / "log", "wb")
        cmd = [sys.executable if a == "python3" else a for a in c["command"] + c.get("args", [])]
        p = subprocess.Popen(cmd, cwd=str(workdir), env=env, stdout=log, stderr=subprocess.STDOUT,
                             start_new_session=True)
        with self.lock:
            self.procs[name] = p
            if name in self.pods:
                self.pods[name]["status"] = {"phase": "Running", "podIP": "127.0.0.1", "hostIP": "127.0.0.1"}
        rc = p.wait()
        log.close()
        with self.lock:
            if name in self.pods:
                self.pods[name]["status"] = {
                    "phase": "Succeeded" if rc == 0 else "Failed", "podIP": "127.0.0.1",
                    "containerStatuses": [{"name": c["name"], "state": {"terminated": {
                        "exitCode": rc if rc >= 0 else 128 - rc, "reason": "Completed" if rc == 0 else "Error"}}}]}

    def _delete_pod(self, name: str, grace: float) -> None:
        with self.lock:
            p = self.procs.get(name)
            self.deleted.append(name)
        if p is not None and p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM if grace > 0 else signal.SIGKILL)
            except ProcessLookupError:
                pass
            try:
                p.wait(timeout=max(grace, 0.1))
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
        with self.lock:
            self.pods.pop(name, None)

    # ----------------------------------------------------------------------------- HTTP
    def _handler(self):
        kube = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a: Any) -> None:
                pass

            def _send(self, code: int, obj: Any) -> None:
                body = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _body(self) -> Any:
                n = int(self.headers.get("Content-Length", "0") or 0)
                return json.loads(self.rfile.read(n) or b"{}") if n else {}

            def do_GET(self) -> None:
                u = urlparse(self.path)
                q = parse_qs(u.query)
                if u.path == "/api/v1/nodes":
                    return self._send(200, {"kind": "NodeList", "items": kube.nodes})
                m = re.match(r"^/api/v1/namespaces/([^/]+)/pods$", u.path)
                if m:
                    sel = q.get("labelSelector", [""])[0]
                    k, _, v = sel.partition("=")
                    with kube.lock:
                        items = [p for p in kube.pods.values()
                                 if not sel or p["metadata"].get("labels", {}).get(k) == v]
                        items = json.loads(json.dumps(items))
                    return self._send(200, {"kind": "PodList", "items": items})
                m = re.match(r"^/api/v1/namespaces/([^/]+)/pods/([^/]+)/log$", u.path)
                if m:
                    return self._logs(m.group(2), q.get("follow", ["false"])[0] == "true")
                m = re.match(r"^/api/v1/namespaces/([^/]+)/pods/([^/]+)$", u.path)
                if m:
                    with kube.lock:
                        p = kube.pods.get(m.group(2))
                    return self._send(200, p) if p else self._send(404, {"kind": "Status", "code": 404})
                self._send(404, {"kind": "Status", "code": 404})

            def _logs(self, name: str, follow: bool) -> None:
                path = kube.root / name / "log"
                self.send_response(200)
                self.send_header("Content-Type", "text/plain")
                self.send_header("Transfer-Encoding", "chunked")
                self.end_headers()
                pos = 0
                while True:
                    data = path.read_bytes()[pos:] if path.exists() else b""
                    if data:
                        pos += len(data)
                        self.wfile.write(b"%x\r\n%s\r\n" % (len(data), data))
                        self.wfile.flush()
                    with kube.lock:
                        pod = kube.pods.get(name)
                        done = pod is None or pod["status"].get("phase") in ("Succeeded", "Failed")
                    if not follow or (done and not data):
                        break
                    time.sleep(0.05)
                self.wfile.write(b"0\r\n\r\n")
                self.wfile.flush()

            def do_POST(self) -> None:
                u = urlparse(self.path)
                obj = self._body()
                m = re.match(r"^/api/v1/namespaces/([^/]+)/(pods|configmaps)$", u.path)
                if not m:
                    return self._send(404, {"kind": "Status", "code": 404})
                name = obj["metadata"]["name"]
                with kube.lock:
                    store = kube.pods if m.group(2) == "pods" else kube.configmaps
                    if name in store:
                        return self._send(409, {"kind": "Status", "code": 409, "reason": "AlreadyExists"})
                    if m.group(2) == "pods":
                        obj["status"] = {"phase": "Pending"}
                        kube.created.append(json.loads(json.dumps(obj)))
                    store[name] = obj
                if m.group(2) == "pods":
                    threading.Thread(target=kube._run_pod, args=(name,), daemon=True).start()
                self._send(201, obj)

            def do_DELETE(self) -> None:
                u = urlparse(self.path)
                body = self._body()
                m = re.match(r"^/api/v1/namespaces/([^/]+)/(pods|configmaps)/([^/]+)$", u.path)
                if not m:
                    return self._send(404, {"kind": "Status", "code": 404})
                name = m.group(3)
                if m.group(2) == "configmaps":
                    with kube.lock:
                        kube.configmaps.pop(name, None)
                    return self._send(200, {"kind": "Status", "status": "Success"})
                with kube.lock:
                    exists = name in kube.pods
                if not exists:
                    return self._send(404, {"kind": "Status", "code": 404})
                grace = float(body.get("gracePeriodSeconds", 30)) if isinstance(body, dict) else 30.0
                threading.Thread(target=kube._delete_pod, args=(name, min(grace, 5.0)), daemon=True).start()
                self._send(200, {"kind": "Status", "status": "Success"})

        return H
