"""Scalar dashboard service for ``det tensorboard start`` (reference
``master/internal/command/tensorboard*.go`` launches stock TensorBoard on the trials' event files).

The ``tensorboard`` package is not installed on MI355X images here, so this is a small
stdlib HTTP server over the same event files (``<storage>/tensorboard/experiment/<e>/trial/<t>``,
written by ``MetricWriter`` and synced by ``TensorboardManager``).  It serves the scalar subset of
TensorBoard's HTTP API, so tools that read scalars from TensorBoard keep working, plus an HTML page
with one SVG chart per tag:

    GET /                                         HTML dashboard
    GET /data/runs                                ["exp1/trial3", ...]
    GET /data/plugin/scalars/tags                 {run: {tag: {"displayName", "description"}}}
    GET /data/plugin/scalars/scalars?run=&tag=    [[wall_time, step, value], ...]

Started as a command task: it binds an ephemeral port and reports it with
``POST /commands/<id>/ready``; the master then proxies ``/proxy/cmd-<id>/...`` to it.

    python -m determined_1_amd.tensorboard.serve --experiment-ids 1,2 [--trial-ids 5] [--port 0]
"""
import argparse
import glob
import html
import json
import logging
import os
import sys
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, List, Optional, Tuple

from determined_1_amd.tensorboard.events import read_scalars
from determined_1_amd.tensorboard.manager import get_base_path

Series = Dict[str, List[Tuple[float, int, float]]]


class RunIndex:
    """run name ("exp<e>/trial<t>") -> event directory; rescanned on every request so a running
    experiment's new files and new trials show up."""

    def __init__(self, dirs: Dict[str, str]) -> None:
        self.dirs = dirs

    def runs(self) -> List[str]:
        return sorted(r for r, d in self.dirs.items() if glob.glob(os.path.join(d, "**", "*tfevents*"), recursive=True))

    def scalars(self, run: str) -> Series:
        out = {}  # type: Series
        d = self.dirs.get(run)
        if not d:
            return out
        for f in sorted(glob.glob(os.path.join(d, "**", "*tfevents*"), recursive=True)):
            try:
                for wall, step, tag, value in read_scalars(f):
                    out.setdefault(tag, []).append((wall, step, value))
            except (ValueError, OSError, IndexError):
                continue  # a file being appended to may end mid-record
        for v in out.values():
            v.sort(key=lambda r: (r[1], r[0]))
        return out


def _svg(points: List[Tuple[float, int, float]], w: int = 360, h: int = 180) -> str:
    if not points:
        return ""
    xs = [p[1] for p in points]
    ys = [p[2] for p in points]
    x0, x1 = min(xs), max(xs) or 1
    y0, y1 = min(ys), max(ys)
    if y1 == y0:
        y1 = y0 + 1.0
    sx = lambda x: 30 + (w - 40) * ((x - x0) / ((x1 - x0) or 1))  # noqa: E731
    sy = lambda y: h - 20 - (h - 30) * ((y - y0) / (y1 - y0))  # noqa: E731
    path = " ".join(f"{sx(x):.1f},{sy(y):.1f}" for x, y in zip(xs, ys))
    return (f'<svg width="{w}" height="{h}"><rect width="{w}" height="{h}" fill="#fafafa" stroke="#ccc"/>'
            f'<polyline fill="none" stroke="#e8590c" stroke-width="1.5" points="{path}"/>'
            f'<text x="32" y="12" font-size="10">{y1:.4g}</text><text x="32" y="{h - 22}" font-size="10">{y0:.4g}</text>'
            f'<text x="{w - 60}" y="{h - 5}" font-size="10">step {x1}</text></svg>')


def make_handler(index: RunIndex):
    class Handler(BaseHTTPRequestHandler):
        def log_message(self, fmt, *args):  # quiet: the master ships stdout as task logs
            logging.debug(fmt, *args)

        def _send(self, code: int, body: str, ctype: str = "application/json") -> None:
            data = body.encode()
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def do_GET(self) -> None:  # noqa: N802
            u = urllib.parse.urlparse(self.path)
            q = dict(urllib.parse.parse_qsl(u.query))
            path = u.path.rstrip("/") or "/"
            if path == "/data/runs":
                return self._send(200, json.dumps(index.runs()))
            if path == "/data/plugin/scalars/tags":
                out = {r: {t: {"displayName": t, "description": ""} for t in index.scalars(r)} for r in index.runs()}
                return self._send(200, json.dumps(out))
            if path == "/data/plugin/scalars/scalars":
                pts = index.scalars(q.get("run", "")).get(q.get("tag", ""))
                if pts is None:
                    return self._send(404, json.dumps({"error": "unknown run/tag"}))
                return self._send(200, json.dumps([[w, s, v] for w, s, v in pts]))
            if path in ("/", "/index.html"):
                parts = ["<html><head><title>Determined MI355X scalars</title></head><body>"]
                for r in index.runs():
                    parts.append(f"<h3>{html.escape(r)}</h3><div>")
                    for tag, pts in sorted(index.scalars(r).items()):
                        parts.append(f'<figure style="display:inline-block"><figcaption>{html.escape(tag)}'
                                     f"</figcaption>{_svg(pts)}</figure>")
                    parts.append("</div>")
                parts.append("</body></html>")
                return self._send(200, "".join(parts), "text/html")
            return self._send(404, json.dumps({"error": "not found"}))

    return Handler


def resolve_runs(master: Optional[str], experiment_ids: List[int], trial_ids: List[int],
                 storage_override: Optional[str]) -> Dict[str, str]:
    """Map each requested trial to its event directory using the experiment's checkpoint storage."""
    runs = {}
    if storage_override:
        storage = {"type": "shared_fs", "host_path": storage_override}
    for eid in experiment_ids:
        tids = []
        if master:
            from determined_1_amd.api.request import MasterClient

            cl = MasterClient(master)
            exp = cl.experiment(eid)
            if not storage_override:
                storage = exp["config"].get("checkpoint_storage", {})
            tids = [t["id"] for t in exp.get("trials", [])]
        if trial_ids:
            tids = [t for t in tids if t in trial_ids] or list(trial_ids)
        for t in tids:
            runs[f"exp{eid}/trial{t}"] = get_base_path(storage, str(eid), str(t))
    return runs


def main(argv: Optional[List[str]] = None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s [tensorboard] %(message)s")
    ap = argparse.ArgumentParser()
    ap.add_argument("--experiment-ids", default="")
    ap.add_argument("--trial-ids", default="")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--storage-path", default=None, help="override the experiments' shared_fs host_path")
    args = ap.parse_args(argv)
    master = os.environ.get("DET_MASTER")
    eids = [int(x) for x in args.experiment_ids.split(",") if x]
    tids = [int(x) for x in args.trial_ids.split(",") if x]
    index = RunIndex(resolve_runs(master, eids, tids, args.storage_path))
    srv = ThreadingHTTPServer((args.host, args.port), make_handler(index))
    port = srv.server_address[1]
    logging.info("serving %d runs on port %d", len(index.dirs), port)
    task = os.environ.get("DET_TASK_ID", "")
    if master and task.startswith("cmd-"):
        from determined_1_amd.api.request import MasterClient

        MasterClient(master).post(f"/commands/{task[4:]}/ready", {"port": port})
        logging.info("registered with the master: /proxy/%s/", task)
    sys.stdout.flush()
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
