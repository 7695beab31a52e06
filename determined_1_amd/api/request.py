"""Thin HTTP client for the det-master REST API (reference ``api/request.py:93``,
``api/experiment.py:196-325``)."""
import json
import os
import time
from typing import Any, Dict, Iterator, List, Optional, Tuple, Union

import requests


def parse_master_address(addr: Optional[str]) -> Tuple[str, int]:
    addr = addr or os.environ.get("DET_MASTER", "127.0.0.1:8080")
    addr = addr.replace("https://", "").replace("http://", "").rstrip("/")
    if ":" in addr:
        h, p = addr.rsplit(":", 1)
        return h, int(p)
    return addr, 8080


def _truthy(v: Optional[str]) -> bool:
    return (v or "").strip().lower() in ("1", "true", "yes", "on")


def master_tls(master: Optional[str] = None) -> Tuple[bool, Union[bool, str]]:
    """(use TLS, requests ``verify``) for the master.  TLS when the address is ``https://...`` or
    ``DET_USE_TLS`` is true (the master sets it, with ``DET_MASTER_CERT_FILE``, in every task it
    starts: reference ``harness/determined/exec/harness.py:161-163``); the server certificate is
    verified against ``DET_MASTER_CERT_FILE`` when set, else the system CA bundle."""
    addr = master or os.environ.get("DET_MASTER", "")
    use = addr.startswith("https://") or _truthy(os.environ.get("DET_USE_TLS"))
    cert = os.environ.get("DET_MASTER_CERT_FILE")
    return use, (cert if cert else True)


def make_url(master: str, path: str) -> str:
    h, p = parse_master_address(master)
    return f"{'https' if master_tls(master)[0] else 'http'}://{h}:{p}{path}"


class APIError(RuntimeError):
    def __init__(self, status: int, msg: str) -> None:
        super().__init__(f"master returned {status}: {msg}")
        self.status = status


TOKEN_FILE = os.path.join(os.path.expanduser("~"), ".det-mi355x", "token.json")


def _load_token(master: str) -> Optional[str]:
    if os.environ.get("DET_USER_TOKEN"):
        return os.environ["DET_USER_TOKEN"]
    try:
        with open(TOKEN_FILE) as f:
            return json.load(f).get(master)
    except (OSError, ValueError):
        return None


def save_token(master: str, token: Optional[str]) -> None:
    os.makedirs(os.path.dirname(TOKEN_FILE), exist_ok=True)
    try:
        with open(TOKEN_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        d = {}
    if token is None:
        d.pop(master, None)
    else:
        d[master] = token
    with open(TOKEN_FILE, "w") as f:
        json.dump(d, f)
    os.chmod(TOKEN_FILE, 0o600)


class MasterClient:
    def __init__(self, master: Optional[str] = None, timeout: float = 60.0) -> None:
        self.master = master or os.environ.get("DET_MASTER", "127.0.0.1:8080")
        self.timeout = timeout
        self.session = requests.Session()
        # passed per request: requests lets $REQUESTS_CA_BUNDLE override a session-level verify
        self.verify = master_tls(self.master)[1]
        self.session.verify = self.verify
        tok = _load_token(self.master)
        if tok:
            self.session.headers["Authorization"] = f"Bearer {tok}"

    def login(self, username: str, password: str = "") -> str:
        tok = self.post("/login", {"username": username, "password": password})["token"]
        self.session.headers["Authorization"] = f"Bearer {tok}"
        save_token(self.master, tok)
        return tok

    def _call(self, method: str, path: str, body: Any = None, params: Optional[Dict[str, Any]] = None) -> Any:
        r = self.session.request(method, make_url(self.master, path), params=params,
                                 data=None if body is None else json.dumps(body), timeout=self.timeout,
                                 headers={"Content-Type": "application/json"}, verify=self.verify)
        if r.status_code >= 300:
            try:
                msg = r.json().get("error", r.text)
            except ValueError:
                msg = r.text
            raise APIError(r.status_code, msg)
        return r.json() if r.text else None

    def get(self, path: str, **params: Any) -> Any:
        return self._call("GET", path, params=params or None)

    def post(self, path: str, body: Any = None) -> Any:
        return self._call("POST", path, body)

    def patch(self, path: str, body: Any) -> Any:
        return self._call("PATCH", path, body)

    def put(self, path: str, body: Any) -> Any:
        return self._call("PUT", path, body)

    def delete(self, path: str) -> Any:
        return self._call("DELETE", path)

    # ------------------------------------------------------------------------ experiments
    def create_experiment(self, config: Dict[str, Any], model_definition: List[Dict[str, Any]],
                          activate: bool = True, template: Optional[str] = None,
                          validate_only: bool = False, parent_id: Optional[int] = None) -> Dict[str, Any]:
        body = {"config": config, "model_definition": model_definition, "activate": activate,
                "validate_only": validate_only}
        if template:
            body["template"] = template
        if parent_id is not None:
            body["parent_id"] = parent_id
        return self.post("/experiments", body)

    def experiment(self, exp_id: int) -> Dict[str, Any]:
        return self.get(f"/experiments/{exp_id}")

    def set_state(self, exp_id: int, state: str) -> Dict[str, Any]:
        return self.patch(f"/experiments/{exp_id}", {"state": state})

    def wait_for_experiment(self, exp_id: int, timeout: float = 3600.0, poll: float = 0.5) -> str:
        deadline = time.time() + timeout
        while time.time() < deadline:
            st = self.experiment(exp_id)["state"]
            if st in ("COMPLETED", "CANCELED", "ERROR"):
                return st
            time.sleep(poll)
        raise TimeoutError(f"experiment {exp_id} did not finish in {timeout}s")

    # ------------------------------------------------------------------ /api/v1 streams
    def stream(self, path: str, **params: Any) -> Iterator[Dict[str, Any]]:
        """A server-streaming /api/v1 RPC: one ``{"result": ...}`` JSON object per line over a
        chunked response (grpc-gateway framing); yields each ``result``."""
        q = {k: ("true" if v is True else "false" if v is False else v) for k, v in params.items() if v is not None}
        r = self.session.get(make_url(self.master, path), params=q, stream=True, timeout=(self.timeout, None),
                             verify=self.verify)
        try:
            if r.status_code >= 300:
                try:
                    msg = r.json().get("error", r.text)
                except ValueError:
                    msg = r.text
                raise APIError(r.status_code, msg)
            for line in r.iter_lines():
                line = line.strip()
                if not line:
                    continue
                msg = json.loads(line)
                if "error" in msg:
                    raise APIError(500, str(msg["error"]))
                yield msg.get("result", msg)
        finally:
            r.close()

    def trial_logs(self, trial_id: int, follow: bool = False, tail: Optional[int] = None,
                   **filters: Any) -> Iterator[Dict[str, Any]]:
        """TrialLogs (``GET /api/v1/trials/:id/logs``): ``follow`` streams until the trial ends;
        ``tail=N`` starts N matching lines before the end; filters: rank_ids, container_ids,
        stdtypes (lists or comma strings)."""
        params: Dict[str, Any] = {"follow": follow}
        if tail:
            params["offset"] = -int(tail)
        for k, v in filters.items():
            if v is not None:
                params[k] = ",".join(str(x) for x in v) if isinstance(v, (list, tuple)) else v
        yield from self.stream(f"/api/v1/trials/{trial_id}/logs", **params)

    def trials_sample(self, exp_id: int, metric: str, metric_type: str = "METRIC_TYPE_VALIDATION",
                      period_seconds: float = 30, **params: Any) -> Iterator[Dict[str, Any]]:
        """TrialsSample (``/api/v1/experiments/:id/metrics-stream/trials-sample``)."""
        yield from self.stream(f"/api/v1/experiments/{exp_id}/metrics-stream/trials-sample", metric_name=metric,
                               metric_type=metric_type, period_seconds=period_seconds, **params)

    def metric_batches(self, exp_id: int, metric: str, metric_type: str = "METRIC_TYPE_VALIDATION",
                       period_seconds: float = 30) -> Iterator[Dict[str, Any]]:
        yield from self.stream(f"/api/v1/experiments/{exp_id}/metrics-stream/batches", metric_name=metric,
                               metric_type=metric_type, period_seconds=period_seconds)
