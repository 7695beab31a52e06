"""Notebook task (``det notebook start``; SURVEY M21, reference
``master/internal/command/notebook_manager.go``): runs JupyterLab (or classic Notebook) in the
task container behind the master's ``/proxy/cmd-<id>/`` with a per-notebook token, and reports its
port with ``POST /commands/<id>/ready``.

Jupyter is not part of the MI355X image used here; when neither ``jupyter_server`` nor
``notebook`` is importable the task fails immediately with that message instead of pretending to
serve.

    python -m determined_1_amd.exec.notebook        (inside the task; env DET_NOTEBOOK_TOKEN)
"""
import importlib.util
import os
import socket
import subprocess
import sys
import time


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("0.0.0.0", 0))
        return s.getsockname()[1]


def main() -> int:
    app = "jupyter_server" if importlib.util.find_spec("jupyter_server") else \
        "notebook" if importlib.util.find_spec("notebook") else None
    if app is None:
        print("notebook: neither jupyter_server nor notebook is installed in this image", file=sys.stderr)
        return 3
    task = os.environ.get("DET_TASK_ID", "")
    port = _free_port()
    token = os.environ.get("DET_NOTEBOOK_TOKEN", "")
    base = f"/proxy/{task}/" if task else "/"
    mod = "jupyterlab" if importlib.util.find_spec("jupyterlab") else app
    argv = [sys.executable, "-m", mod, "--no-browser", "--ip=0.0.0.0", f"--port={port}",
            f"--ServerApp.base_url={base}", f"--ServerApp.token={token}", "--ServerApp.allow_origin=*"]
    proc = subprocess.Popen(argv)
    deadline = time.time() + 120
    while time.time() < deadline and proc.poll() is None:
        try:
            socket.create_connection(("127.0.0.1", port), timeout=1).close()
            break
        except OSError:
            time.sleep(0.5)
    master = os.environ.get("DET_MASTER")
    if proc.poll() is None and master and task.startswith("cmd-"):
        from determined_1_amd.api.request import MasterClient

        MasterClient(master).post(f"/commands/{task[4:]}/ready", {"port": port})
    return proc.wait()


if __name__ == "__main__":
    sys.exit(main())
