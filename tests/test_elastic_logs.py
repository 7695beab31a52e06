"""Trial logs in Elasticsearch (reference master/internal/elastic/elastic_trial_logs.go:38-95 and
master/internal/config/elastic.go: ``logging: {type: elastic, host, port}``).

det-master runs with ``logging.type: elastic`` against an in-memory Elasticsearch stand-in
(``tests/fake_elastic.py``): a no-op experiment's trial logs are shipped with ``_bulk`` and never
written to the local segments, and the log endpoints (filters, tail, offset paging, the
``/api/v1`` TrialLogs stream) are answered from ``_search``.  No real Elasticsearch is available
here, so wire compatibility beyond the request shapes the fake checks is parity unpinned.
"""
import json
import pathlib

from determined_1_amd.api import MasterClient, read_context
from determined_1_amd.deploy import LocalCluster
from fake_elastic import FakeElastic

NOOP = pathlib.Path(__file__).resolve().parent / "fixtures" / "no_op"


def test_trial_logs_in_elasticsearch(tmp_path):
    with FakeElastic() as es:
        cfg = tmp_path / "master.yaml"
        cfg.write_text(f"logging:\n  type: elastic\n  host: 127.0.0.1\n  port: {es.port}\n  index: det-test-logs\n")
        with LocalCluster(agents=1, slots_per_agent=1, log_dir=str(tmp_path), tick_ms=50,
                          master_args=["--config-file", str(cfg)]) as c:
            cl = MasterClient(c.address)
            assert cl.get("/api/v1/master/config")["config"]["logging"]["type"] == "elastic"
            exp = {"description": "es", "entrypoint": "model_def:NoOpTrial",
                   "hyperparameters": {"global_batch_size": 4, "metrics_base": 0.9},
                   "searcher": {"name": "single", "metric": "validation_error", "max_length": {"batches": 4}},
                   "scheduling_unit": 2}
            eid = cl.create_experiment(exp, read_context(NOOP))["id"]
            assert cl.wait_for_experiment(eid, timeout=240) == "COMPLETED"
            tid = cl.experiment(eid)["trials"][0]["id"]
            logs = cl.get(f"/trials/{tid}/logs")
            assert logs and [l["id"] for l in logs] == list(range(1, len(logs) + 1))
            # every line went through _bulk (ndjson) into the configured index
            stored = [s for i, s in es.indices["det-test-logs"].items() if s["stream"] == f"trial-{tid}"]
            assert len(stored) == len(logs)
            assert all(ct == "application/x-ndjson" for p, ct, _ in es.requests if p == "/_bulk")
            # nothing landed in the local segments
            assert not list(pathlib.Path(tmp_path).rglob(f"trial-{tid}.jsonl"))

            # offset paging, tail and filters are answered from _search
            n = len(logs)
            assert [l["id"] for l in cl.get(f"/trials/{tid}/logs", offset=2, limit=3)] == [3, 4, 5]
            assert [l["id"] for l in cl.get(f"/trials/{tid}/logs", limit=2, tail="true")] == [n - 1, n]
            word = logs[0]["message"].split()[0] if logs[0]["message"].split() else ""
            hits = cl.get(f"/trials/{tid}/logs", contains=word)
            assert hits and all(word in l["message"] for l in hits)

            # lines shipped after a restart continue the id sequence (max id read back from ES)
            cl.post("/trial_logs", [{"trial_id": tid, "message": "late line", "rank_id": 0}])
            tail = cl.get(f"/trials/{tid}/logs", limit=1, tail="true")
            assert tail[0]["id"] == n + 1 and tail[0]["message"] == "late line"

        # a second master over the same Elasticsearch index sees the same logs and continues the ids
        (tmp_path / "m2").mkdir()
        with LocalCluster(agents=0, slots_per_agent=1, log_dir=str(tmp_path / "m2"), tick_ms=50,
                          master_args=["--config-file", str(cfg)]) as c2:
            cl2 = MasterClient(c2.address)
            assert len(cl2.get(f"/trials/{tid}/logs")) == n + 1
            cl2.post("/trial_logs", [{"trial_id": tid, "message": "after restart", "rank_id": 0}])
            assert cl2.get(f"/trials/{tid}/logs", limit=1, tail="true")[0]["id"] == n + 2
    searches = [json.loads(b) for p, _, b in es.requests if p.endswith("/_search")]
    assert searches and all(s["query"]["bool"]["filter"][0] == {"term": {"stream": f"trial-{tid}"}} for s in searches)


def test_elastic_logging_config_validation(tmp_path):
    import subprocess

    from determined_1_amd.deploy.local import native_binary

    cfg = tmp_path / "master.yaml"
    cfg.write_text("logging:\n  type: elastic\n")
    p = subprocess.run([native_binary("det-master"), "--config-file", str(cfg), "--port", "1"], capture_output=True,
                       text=True, timeout=30)
    assert p.returncode != 0 and "logging.host is required" in (p.stdout + p.stderr)


def _debug_stats(cl):
    return cl.get("/debug/stats")


def test_log_shipping_off_the_agent_socket_under_a_slow_failing_elasticsearch(tmp_path):
    """VERDICT r3 / ADVICE r3: with Elasticsearch answering each _bulk after 1 s and failing every
    3rd one, a trial printing 2,000 lines/s still completes promptly, the agent's
    ContainerStateChanged messages are handled within 100 ms of being sent (log lines are queued,
    never shipped on the socket thread), and every line ends up in the index exactly once with
    contiguous ids (failed batches are retried)."""
    import time

    steps, per_step = 3, 2000
    with FakeElastic(bulk_delay=1.0, fail_every=3) as es:
        cfg = tmp_path / "master.yaml"
        cfg.write_text(f"logging:\n  type: elastic\n  host: 127.0.0.1\n  port: {es.port}\n  index: det-load\n")
        with LocalCluster(agents=1, slots_per_agent=1, log_dir=str(tmp_path), tick_ms=50,
                          master_args=["--config-file", str(cfg)]) as c:
            cl = MasterClient(c.address)
            exp = {"description": "es-load", "entrypoint": "model_def:NoOpTrial",
                   "hyperparameters": {"global_batch_size": 4, "metrics_base": 0.9, "log_lines": per_step,
                                       "log_seconds": 1.0},
                   "searcher": {"name": "single", "metric": "validation_error", "max_length": {"batches": steps}},
                   "scheduling_unit": 1, "min_validation_period": {"batches": steps}}
            t0 = time.time()
            eid = cl.create_experiment(exp, read_context(NOOP))["id"]
            assert cl.wait_for_experiment(eid, timeout=180) == "COMPLETED"
            elapsed = time.time() - t0
            tid = cl.experiment(eid)["trials"][0]["id"]
            st = _debug_stats(cl)
            lat = st["agent_state_latency_ms"]
            assert lat["count"] >= 2 and lat["max"] < 100.0, lat
            deadline = time.time() + 120
            while time.time() < deadline:
                ship = _debug_stats(cl)["log_shipping"]
                if ship["pending_lines"] == 0 and ship["inflight_lines"] == 0:
                    break
                time.sleep(0.5)
            assert ship["pending_lines"] == 0 and ship["inflight_lines"] == 0, ship
            assert ship["failed_batches"] >= 1 and es.bulk_failures >= 1  # the retries were exercised
            logs = cl.get(f"/trials/{tid}/logs")
            ids = [l["id"] for l in logs]
            assert ids == list(range(1, len(ids) + 1))
            spam = [l["message"] for l in logs if l["message"].startswith("spam ")]
            assert len(spam) == steps * per_step and len(set(spam)) == len(spam)
            with es.lock:
                stored = [s for s in es.indices["det-load"].values() if s["stream"] == f"trial-{tid}"]
            assert sorted(s["id"] for s in stored) == ids  # exactly once, contiguous
    # the trial was not throttled by the 1 s _bulk latency (one request per line would need hours)
    assert elapsed < 150, elapsed


def test_existing_dynamic_index_is_queried_on_the_keyword_subfield(tmp_path):
    """an index Elasticsearch created with its dynamic mapping holds `stream` as analysed
    text; a term query on it matches nothing.  The backend reads the mapping and filters on
    stream.keyword (the reference's choice), so reads, the id sequence and deletes all work."""
    with FakeElastic() as es:
        es.dynamic_index("det-dyn", [{"stream": "trial-999", "id": 1, "message": "older cluster"}])
        cfg = tmp_path / "master.yaml"
        cfg.write_text(f"logging:\n  type: elastic\n  host: 127.0.0.1\n  port: {es.port}\n  index: det-dyn\n")
        with LocalCluster(agents=0, slots_per_agent=1, log_dir=str(tmp_path), tick_ms=50,
                          master_args=["--config-file", str(cfg)]) as c:
            cl = MasterClient(c.address)
            got = cl.get("/trials/999/logs")
            assert [l["message"] for l in got] == ["older cluster"]
            cl.post("/trial_logs", [{"trial_id": 999, "message": "new line", "rank_id": 0}])
            assert [l["id"] for l in cl.get("/trials/999/logs")] == [1, 2]  # continues after the existing id
    searches = [json.loads(b) for p, _, b in es.requests if p.endswith("/_search")]
    assert searches and all(s["query"]["bool"]["filter"][0] == {"term": {"stream.keyword": "trial-999"}}
                            for s in searches)
