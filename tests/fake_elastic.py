"""In-memory Elasticsearch stand-in for the master's elastic log backend tests: the subset of the REST
API ``native/src/elastic_logs.cc`` speaks (``_bulk`` index actions, ``_search`` with a bool filter
of term + range clauses, ``sort`` and ``size``, ``_delete_by_query`` with a term query).  Unknown
indices answer 404 like the real server.  Every request is recorded for assertions."""
import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import urlparse


class FakeElastic:
    def __init__(self):
        self.indices = {}  # index -> {_id: source}
        self.requests = []
        self.lock = threading.Lock()
        fake = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, obj):
                b = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)

            def do_POST(self):
                n = int(self.headers.get("Content-Length", "0"))
                body = self.rfile.read(n).decode()
                path = urlparse(self.path).path
                with fake.lock:
                    fake.requests.append((path, self.headers.get("Content-Type"), body))
                    code, out = fake.handle(path, body)
                self._send(code, out)

        self.server = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.port = self.server.server_address[1]
        self.thread = threading.Thread(target=self.server.serve_forever, daemon=True)

    def __enter__(self):
        self.thread.start()
        return self

    def __exit__(self, *a):
        self.server.shutdown()
        self.server.server_close()

    @staticmethod
    def _match(src, flt):
        for f in flt:
            if "term" in f:
                (k, v), = f["term"].items()
                if src.get(k) != v:
                    return False
            elif "range" in f:
                (k, r), = f["range"].items()
                x = src.get(k)
                if x is None or ("gt" in r and not x > r["gt"]) or ("lt" in r and not x < r["lt"]):
                    return False
        return True

    def handle(self, path, body):
        if path == "/_bulk":
            lines = [l for l in body.split("\n") if l.strip()]
            items = []
            for meta, doc in zip(lines[0::2], lines[1::2]):
                act = json.loads(meta)["index"]
                self.indices.setdefault(act["_index"], {})[act["_id"]] = json.loads(doc)
                items.append({"index": {"_id": act["_id"], "status": 201}})
            return 200, {"errors": False, "items": items}
        parts = path.strip("/").split("/")
        if len(parts) != 2 or parts[0] not in self.indices:
            return 404, {"error": {"type": "index_not_found_exception"}, "status": 404}
        docs = self.indices[parts[0]]
        q = json.loads(body or "{}")
        if parts[1] == "_search":
            flt = q.get("query", {}).get("bool", {}).get("filter", [])
            hits = [(i, s) for i, s in docs.items() if self._match(s, flt)]
            for key in reversed(q.get("sort", [])):
                (k, order), = key.items()
                hits.sort(key=lambda h: h[1].get(k), reverse=order == "desc")
            hits = hits[:q.get("size", 10)]
            return 200, {"hits": {"total": {"value": len(hits)}, "hits": [{"_id": i, "_source": s} for i, s in hits]}}
        if parts[1] == "_delete_by_query":
            gone = [i for i, s in docs.items() if self._match(s, [q["query"]])]
            for i in gone:
                del docs[i]
            return 200, {"deleted": len(gone)}
        return 400, {"error": "unsupported"}
