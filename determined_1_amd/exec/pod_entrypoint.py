"""Entrypoint of a Kubernetes pod started by the master's Kubernetes resource manager
(native/src/kubernetes.cc; reference master/internal/kubernetes/spec.go, whose pods run
``/run/determined/train/entrypoint.sh`` after an init container unpacks the run archives).

What det-agent does before starting a container, done inside the pod:

  1. read the container spec the master put in the pod's ConfigMap (``$DET_SPEC_FILE``);
  2. fetch the model definition / command context from the master (``spec.context_url``) and
     write it, plus the spec's extra files, into the working directory;
  3. make a relative ``DET_LATEST_CHECKPOINT`` absolute, put the working directory on
     ``PYTHONPATH``;
  4. run the command after ``--`` (the trial harness by default) as a child process and exit with
     its status, forwarding SIGTERM so a pod deletion stops the trial gracefully.

    python -m determined_1_amd.exec.pod_entrypoint -- python3 -m determined_1_amd.exec.harness
"""
import base64
import json
import os
import pathlib
import signal
import subprocess
import sys
from typing import Any, Dict, List

import requests

from determined_1_amd.api.request import make_url, master_tls


def materialize(spec: Dict[str, Any], workdir: pathlib.Path, master: str) -> None:
    exp_id = spec.get("experiment_id", 0)
    url = spec.get("context_url") or f"/experiments/{exp_id}/model_def"
    r = requests.get(make_url(master, url), timeout=60, verify=master_tls(master)[1])
    r.raise_for_status()
    for f in r.json().get("files", []):
        rel = f.get("path", "")
        if not rel or ".." in pathlib.PurePosixPath(rel).parts:
            continue
        dst = workdir / rel
        if f.get("type") == "dir" or rel.endswith("/"):
            dst.mkdir(parents=True, exist_ok=True)
            continue
        dst.parent.mkdir(parents=True, exist_ok=True)
        dst.write_bytes(base64.b64decode(f.get("content", "")))
    for f in spec.get("files", []):
        dst = workdir / f.get("path", "")
        dst.parent.mkdir(parents=True, exist_ok=True)
        dst.write_bytes(base64.b64decode(f.get("content", "")))


def main(argv: List[str]) -> int:
    cmd = argv[argv.index("--") + 1:] if "--" in argv else [sys.executable, "-m", "determined_1_amd.exec.harness"]
    spec_file = os.environ.get("DET_SPEC_FILE", "/run/determined/spec/spec.json")
    spec = json.loads(pathlib.Path(spec_file).read_text())
    workdir = pathlib.Path(os.environ.get("DET_WORKDIR", os.getcwd()))
    workdir.mkdir(parents=True, exist_ok=True)
    master = os.environ["DET_MASTER"]
    materialize(spec, workdir, master)
    env = dict(os.environ)
    latest = env.get("DET_LATEST_CHECKPOINT", "")
    if latest and not latest.startswith("/"):
        env["DET_LATEST_CHECKPOINT"] = str(workdir / latest)
    env["PYTHONPATH"] = os.pathsep.join([p for p in [str(workdir), env.get("PYTHONPATH", "")] if p])
    print(f"[pod] {spec.get('task_id') or 'trial ' + str(spec.get('trial_id'))}: running {' '.join(cmd)}", flush=True)
    child = subprocess.Popen(cmd, cwd=str(workdir), env=env)

    def forward(signum: int, _frame: Any) -> None:
        try:
            child.send_signal(signum)
        except ProcessLookupError:
            pass

    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    rc = child.wait()
    return rc if rc >= 0 else 128 - rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
