"""In-memory Elasticsearch stand-in for the master's elastic log backend tests.

It models the parts of Elasticsearch whose semantics the backend depends on, not only the request
shapes (``native/src/elastic_logs.cc``):

* ``_bulk`` index actions; documents become searchable only after a refresh -- an explicit
  ``POST /<index>/_refresh`` or the periodic one every ``refresh_interval`` seconds (1 s, like a
  real index), so a client that reads right after writing sees nothing unless it keeps its own
  copy;
* mappings: ``PUT /<index>`` with explicit ``mappings``, ``GET /<index>/_mapping``, and dynamic
  mapping on the first document otherwise -- strings become ``text`` with a ``keyword``
  sub-field, like Elasticsearch's default.  A ``term`` query on a ``text`` field matches the
  analysed tokens only ("trial-7" -> "trial", "7"), so it never matches a whole stream name;
  ``<field>.keyword`` matches exactly;
* ``_search`` with a bool filter of term + range clauses, ``sort`` and ``size``;
  ``_delete_by_query`` with a term query;
* fault injection: ``bulk_delay`` seconds of latency per ``_bulk`` and ``fail_every`` = n makes
  every n-th ``_bulk`` answer 503.

Unknown indices answer 404 like the real server.  Every request is recorded for assertions."""
import json
import re
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import urlparse


def _tokens(v):
    return re.findall(r"[a-z0-9]+", str(v).lower())


class FakeElastic:
    def __init__(self, bulk_delay: float = 0.0, fail_every: int = 0, refresh_interval: float = 1.0):
        self.indices = {}  # index -> {_id: source} (every indexed document, searchable or not)
        self.visible = {}  # index -> set of searchable _ids
        self.mappings = {}  # index -> {field: {"type": ..., "fields": {...}}}
        self.requests = []
        self.bulk_calls = 0
        self.bulk_failures = 0
        self.bulk_delay = bulk_delay
        self.fail_every = fail_every
        self.refresh_interval = refresh_interval
        self.lock = threading.Lock()
        self._stop = threading.Event()
        fake = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _send(self, code, obj):
                b = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)

            def _do(self, method):
                n = int(self.headers.get("Content-Length", "0") or 0)
                body = self.rfile.read(n).decode() if n else ""
                path = urlparse(self.path).path
                if path == "/_bulk":
                    if fake.bulk_delay:
                        time.sleep(fake.bulk_delay)  # a slow cluster, outside the lock
                with fake.lock:
                    fake.requests.append((path, self.headers.get("Content-Type"), body))
                    code, out = fake.handle(method, path, body)
                self._send(code, out)

            def do_POST(self):
                self._do("POST")

            def do_PUT(self):
                self._do("PUT")

            def do_GET(self):
                self._do("GET")

        self.server = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.port = self.server.server_address[1]
        self.thread = threading.Thread(target=self.server.serve_forever, daemon=True)
        self.refresher = threading.Thread(target=self._periodic_refresh, daemon=True)

    def __enter__(self):
        self.thread.start()
        self.refresher.start()
        return self

    def __exit__(self, *a):
        self._stop.set()
        self.server.shutdown()
        self.server.server_close()

    def _periodic_refresh(self):
        while not self._stop.wait(self.refresh_interval):
            with self.lock:
                for idx in self.indices:
                    self.visible[idx] = set(self.indices[idx])

    def dynamic_index(self, index, docs):
        """Create ``index`` the way a real cluster does when the first document arrives without a
        mapping (strings -> text + keyword sub-field), and make the documents searchable."""
        with self.lock:
            for i, d in enumerate(docs):
                self._index_doc(index, str(i), d)
            self.visible[index] = set(self.indices[index])

    def _index_doc(self, index, _id, doc):
        m = self.mappings.setdefault(index, {})
        for k, v in doc.items():
            if k not in m:
                m[k] = {"type": "long"} if isinstance(v, int) and not isinstance(v, bool) else \
                    {"type": "text", "fields": {"keyword": {"type": "keyword"}}}
        self.indices.setdefault(index, {})[_id] = doc
        self.visible.setdefault(index, set())

    def _match(self, index, src, flt):
        m = self.mappings.get(index, {})
        for f in flt:
            if "term" in f:
                (k, v), = f["term"].items()
                if k.endswith(".keyword"):
                    base = k[:-len(".keyword")]
                    if "keyword" not in m.get(base, {}).get("fields", {}) or src.get(base) != v:
                        return False
                elif m.get(k, {}).get("type") == "text":
                    # the analysed field holds tokens: only a single-token value can match one
                    if str(v).lower() not in _tokens(src.get(k)):
                        return False
                elif src.get(k) != v:
                    return False
            elif "range" in f:
                (k, r), = f["range"].items()
                x = src.get(k)
                if x is None or ("gt" in r and not x > r["gt"]) or ("lt" in r and not x < r["lt"]):
                    return False
        return True

    def handle(self, method, path, body):
        if path == "/_bulk":
            self.bulk_calls += 1
            if self.fail_every and self.bulk_calls % self.fail_every == 0:
                self.bulk_failures += 1
                return 503, {"error": {"type": "unavailable_shards_exception"}, "status": 503}
            lines = [l for l in body.split("\n") if l.strip()]
            items = []
            for meta, doc in zip(lines[0::2], lines[1::2]):
                act = json.loads(meta)["index"]
                self._index_doc(act["_index"], act["_id"], json.loads(doc))
                items.append({"index": {"_id": act["_id"], "status": 201}})
            return 200, {"errors": False, "items": items}
        parts = path.strip("/").split("/")
        if method == "PUT" and len(parts) == 1:
            if parts[0] in self.indices:
                return 400, {"error": {"type": "resource_already_exists_exception"}, "status": 400}
            q = json.loads(body or "{}")
            self.mappings[parts[0]] = dict(q.get("mappings", {}).get("properties", {}))
            self.indices[parts[0]] = {}
            self.visible[parts[0]] = set()
            return 200, {"acknowledged": True, "index": parts[0]}
        if len(parts) != 2 or parts[0] not in self.indices:
            return 404, {"error": {"type": "index_not_found_exception"}, "status": 404}
        idx = parts[0]
        docs = self.indices[idx]
        if parts[1] == "_mapping":
            return 200, {idx: {"mappings": {"properties": self.mappings.get(idx, {})}}}
        if parts[1] == "_refresh":
            self.visible[idx] = set(docs)
            return 200, {"_shards": {"successful": 1}}
        q = json.loads(body or "{}")
        if parts[1] == "_search":
            flt = q.get("query", {}).get("bool", {}).get("filter", [])
            hits = [(i, s) for i, s in docs.items() if i in self.visible[idx] and self._match(idx, s, flt)]
            for key in reversed(q.get("sort", [])):
                (k, order), = key.items()
                hits.sort(key=lambda h: h[1].get(k), reverse=order == "desc")
            hits = hits[:q.get("size", 10)]
            return 200, {"hits": {"total": {"value": len(hits)}, "hits": [{"_id": i, "_source": s} for i, s in hits]}}
        if parts[1] == "_delete_by_query":
            gone = [i for i, s in docs.items() if self._match(idx, s, [q["query"]])]
            for i in gone:
                del docs[i]
                self.visible[idx].discard(i)
            return 200, {"deleted": len(gone)}
        return 400, {"error": "unsupported"}
