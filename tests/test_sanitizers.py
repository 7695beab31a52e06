"""Sanitizers over the native control plane, in the suite so a regression fails CI.

* ThreadSanitizer and AddressSanitizer builds of the C++ unit tests (clang from ROCm's LLVM: gcc
  11's libtsan misses the ``pthread_cond_clockwait`` interceptor and reports false double locks);
* an end-to-end run of an ASan-built det-master with two ASan-built det-agents driving an
  adaptive ASHA experiment through trial processes; any sanitizer report in any log fails.
Host code only: GPU sanitizers are not available on this pool."""
import os
import pathlib
import subprocess

import pytest

REPO = pathlib.Path(__file__).resolve().parent.parent
NATIVE = REPO / "native"
CLANG = pathlib.Path("/opt/rocm/lib/llvm/bin/clang++")

pytestmark = [pytest.mark.slow, pytest.mark.skipif(not CLANG.exists(), reason="ROCm clang not installed")]


def _make(san: str, target: str, env: dict) -> subprocess.CompletedProcess:
    return subprocess.run(["make", "-C", str(NATIVE), f"SAN={san}", "-j8", target], capture_output=True, text=True,
                          timeout=1500, env=env)


@pytest.mark.parametrize("san,opts", [
    ("thread", {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66 second_deadlock_stack=1"}),
    ("address", {"ASAN_OPTIONS": "detect_leaks=1 halt_on_error=1 exitcode=67",
                 "LSAN_OPTIONS": "exitcode=67"}),
])
def test_native_unit_tests_clean_under_sanitizer(san, opts):
    env = dict(os.environ, **opts)
    r = _make(san, "test", env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "ThreadSanitizer" not in out and "AddressSanitizer" not in out and "LeakSanitizer" not in out, out[-6000:]
    assert "PASS" in out


def test_asan_master_and_agents_run_asha(tmp_path, monkeypatch):
    env = dict(os.environ)
    r = _make("address", "all", env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    bindir = NATIVE / "build-address" / "bin"
    monkeypatch.setenv("DET_NATIVE_BIN_DIR", str(bindir))
    monkeypatch.setenv("ASAN_OPTIONS", "detect_leaks=0 halt_on_error=1 abort_on_error=0")
    from determined_1_amd.api import MasterClient, read_context
    from determined_1_amd.deploy import LocalCluster

    noop = REPO / "tests" / "fixtures" / "no_op"
    c = LocalCluster(agents=2, slots_per_agent=2, store_dir=str(tmp_path / "store"),
                     checkpoint_dir=str(tmp_path / "ckpt"), log_dir=str(tmp_path), tick_ms=50)
    c.up()
    try:
        cfg = {"description": "asan-asha", "entrypoint": "model_def:NoOpTrial", "scheduling_unit": 5,
               "hyperparameters": {"global_batch_size": 4,
                                   "metrics_base": {"type": "double", "minval": 0.5, "maxval": 0.9}},
               "searcher": {"name": "adaptive_asha", "metric": "validation_error", "max_length": {"batches": 40},
                            "max_trials": 6, "divisor": 4, "max_rungs": 3, "mode": "aggressive"}}
        cl = MasterClient(c.address)
        eid = cl.create_experiment(cfg, read_context(noop))["id"]
        assert cl.wait_for_experiment(eid, timeout=300) == "COMPLETED"
        assert len(cl.experiment(eid)["trials"]) == 6
    finally:
        c.down()
    logs = "".join(p.read_text(errors="replace") for p in tmp_path.glob("*.log"))
    assert logs, "no master/agent logs captured"
    assert "AddressSanitizer" not in logs and "runtime error" not in logs, logs[-6000:]
