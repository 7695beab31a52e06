"""ASHA trials/hr on a real cluster (BASELINE north-star #2): det-master + det-agent (GPU slots from
KFD) on this host running the 16-trial adaptive_asha CIFAR-10 experiment of
examples/computer_vision/cifar10_pytorch/adaptive.yaml (reference adaptive.yaml:26-31: max_length
32 epochs of 50,000 records, validation every epoch) UNCHANGED by default.

Reports trials completed / hour, wall time, the GPU-busy fraction sampled from amdgpu sysfs, slot
occupancy (container-seconds / (wall x slots)) and the scheduler idle fraction (1 - occupancy), plus
per-container startup phases from the harness timeline.

    python scripts/bench_asha.py [--slots 8] [--timeout 3600]            # the BASELINE shape
    python scripts/bench_asha.py --max-length-batches 300                 # scaled-down smoke run
"""
import argparse
import json
import os
import pathlib
import sys
import threading
import time

import yaml

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def summarize_timelines(cl, trials, t0):
    """Mean seconds per trial container spent in each harness phase (from DET_TIMELINE logs);
    full per-trial timelines go to $DET_BENCH_LOGDIR/asha_timeline.txt."""
    import re
    from collections import defaultdict

    pat = re.compile(r"\[timeline\] \+([0-9.]+)s (.*)$")
    phases = defaultdict(list)
    lines = []
    for t in trials:
        by_container = defaultdict(list)
        for rec in cl.get(f"/trials/{t['id']}/logs"):
            m = pat.search(rec.get("message", ""))
            if m:
                by_container[rec.get("container_id")].append((float(m.group(1)), m.group(2)))
        for cid, marks in by_container.items():
            lines.append(f"trial {t['id']} container {cid}")
            prev = 0.0
            workload = 0.0
            for ts, label in marks:
                lines.append(f"  +{ts:8.3f}s (+{ts - prev:6.3f}) {label}")
                if label.startswith("done "):
                    workload += ts - prev
                elif not label.startswith("start "):
                    phases[label].append(ts - prev)
                else:
                    phases["between workloads"].append(ts - prev)
                prev = ts
            phases["workloads"].append(workload)
            phases["total"].append(prev)
    out_dir = os.environ.get("DET_BENCH_LOGDIR", "/tmp")
    with open(os.path.join(out_dir, "asha_timeline.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    n = max(1, len(phases["total"]))
    out = {k: round(sum(v) / n, 3) for k, v in phases.items()}
    out["_containers"] = len(phases["total"])
    return out


def _ts(s):
    from datetime import datetime

    return datetime.strptime(s.rstrip("Z")[:26], "%Y-%m-%dT%H:%M:%S.%f").timestamp() if s else None


def idle_breakdown(cl, trials, slots, t_start, t_end):
    """Split idle slot-seconds into "no trial exists to run" (searcher-bound: ASHA has not created or
    promoted work for the slot) and "a live trial has no running container" (scheduling, container
    start, or a trial parked between rungs until ASHA promotes it), from the master's trial
    start/end times and the first / last log record of each trial container."""
    from collections import defaultdict

    alive, busy = [], []
    for t in trials:
        a, b = _ts(t.get("start_time")), _ts(t.get("end_time")) or t_end
        if a is not None:
            alive.append((a, b))
        spans = defaultdict(list)
        for rec in cl.get(f"/trials/{t['id']}/logs"):
            ts = _ts(rec.get("timestamp"))
            if ts is not None:
                spans[rec.get("container_id")].append(ts)
        busy += [(min(v), max(v)) for v in spans.values() if v]
    step = 0.05
    n = int((t_end - t_start) / step) + 1
    idle = searcher = parked = 0.0
    for i in range(n):
        t = t_start + i * step
        nb = sum(1 for a, b in busy if a <= t < b)
        na = sum(1 for a, b in alive if a <= t < b)
        idle += max(0, slots - nb) * step
        searcher += max(0, slots - max(na, nb)) * step
        parked += max(0, min(na, slots) - nb) * step
    tot = slots * (t_end - t_start)
    return {"idle_frac": round(idle / tot, 3), "idle_no_trial_frac": round(searcher / tot, 3),
            "idle_trial_without_container_frac": round(parked / tot, 3)}


def control_plane_breakdown(cl, trials, slots, t_start, t_end):
    """Idle slot time by cause, from the master's [sched] events (resources requested / allocated per
    trial task) and each trial container's log records:

      * ``work``: container time from the harness's "controller ready" mark to its last record;
      * ``container_init``: container time before "controller ready" (process start, imports, storage
        probe, rendezvous, trial construction) -- control plane;
      * ``waiting``: slots free while a task that asked for resources has no container yet (the
        scheduler, the agent's container launch) -- control plane;
      * ``no_runnable_trial``: the rest -- no trial had work for the slot (ASHA waits on rung results
        before promoting or creating; inherent to the search).
    Fractions are of slots x wall."""
    import re
    from collections import defaultdict

    pat = re.compile(r"\[sched\] event=(\w+) request=(\S+) trial=(\d+) task=(\S+)")
    req, alloc = {}, {}
    rid_of_task = {}
    for rec in cl.get("/logs", limit=25000):
        m = pat.search(rec.get("message", ""))
        if not m:
            continue
        ev, rid, _, task = m.groups()
        ts = _ts(rec.get("time"))
        rid_of_task[task] = rid
        (req if ev == "requested" else alloc).setdefault(task, ts)
    by_rid = {t.get("request_id"): t for t in trials}
    cont_spans = defaultdict(list)  # trial id -> [(first, ready, last)]
    for t in trials:
        spans = defaultdict(list)
        ready = {}
        for rec in cl.get(f"/trials/{t['id']}/logs"):
            ts = _ts(rec.get("timestamp"))
            if ts is None:
                continue
            cid = rec.get("container_id")
            spans[cid].append(ts)
            if "controller ready" in rec.get("message", "") and cid not in ready:
                ready[cid] = ts
        for cid, v in spans.items():
            cont_spans[t["id"]].append((min(v), ready.get(cid, min(v)), max(v)))
    waits = []  # (from request, until the task's container's first record)
    for task, t0 in req.items():
        t = by_rid.get(rid_of_task.get(task))
        if t is None:
            continue
        after = sorted(c[0] for c in cont_spans.get(t["id"], []) if c[0] >= t0 - 0.5)
        waits.append((t0, after[0] if after else t_end))
    step = 0.02
    n = int((t_end - t_start) / step) + 1
    work = init = waiting = 0.0
    allc = [c for v in cont_spans.values() for c in v]
    for i in range(n):
        t = t_start + i * step
        nw = sum(1 for a, r, b in allc if r <= t < b)
        ni = sum(1 for a, r, b in allc if a <= t < r)
        nwait = sum(1 for a, b in waits if a <= t < b)
        free = max(0, slots - nw - ni)
        work += min(slots, nw) * step
        init += min(slots - min(slots, nw), ni) * step
        waiting += min(free, nwait) * step
    tot = slots * (t_end - t_start)
    out = {"work_frac": work / tot, "container_init_frac": init / tot, "waiting_frac": waiting / tot}
    out["no_runnable_trial_frac"] = max(0.0, 1.0 - sum(out.values()))
    out["control_plane_idle_frac"] = out["container_init_frac"] + out["waiting_frac"]
    out = {k: round(v, 4) for k, v in out.items()}
    out["tasks"] = len(req)
    out["mean_wait_s"] = round(sum(b - a for a, b in waits) / max(1, len(waits)), 3)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-length-batches", type=int, default=0,
                    help="scale the search down to this many batches (0 = the reference's 32 epochs)")
    ap.add_argument("--max-trials", type=int, default=16)
    ap.add_argument("--slots", type=int, default=0, help="GPU slots to use (0 = every GPU the agent detects)")
    ap.add_argument("--timeout", type=float, default=3600)
    ap.add_argument("--no-zygote", action="store_true", help="cold python exec per container (A/B)")
    ap.add_argument("--seed", type=int, default=1, help="reproducibility.experiment_seed (fixes the sampled hparams)")
    ap.add_argument("--no-hip-graph", action="store_true", help="eager train_batch (A/B)")
    ap.add_argument("--artificial-slots", type=int, default=0, help="CPU dry run without GPUs")
    ap.add_argument("--validation-records", type=int, default=0,
                    help="shrink the validation set (scaled-down CPU runs; 0 = CIFAR-10's 10,000)")
    ap.add_argument("--amp", default=None, help="override hyperparameters.amp (O0 = fp32, the reference precision)")
    ap.add_argument("--modelled-batch-ms", type=float, default=0.0,
                    help="run scripts/asha_model's trial: each batch waits this long (the MI355X time at batch 32) "
                         "instead of computing -- the control plane at the real shape on CPU slots")
    ap.add_argument("--graph-batches", type=int, default=0,
                    help="override optimizations.hip_graph_batches (train steps per hipGraph replay)")
    args = ap.parse_args()
    from determined_1_amd import gpu
    from determined_1_amd.api import MasterClient, read_context
    from determined_1_amd.deploy import LocalCluster

    ex = REPO / "examples" / "computer_vision" / "cifar10_pytorch"
    if args.modelled_batch_ms:
        ex = REPO / "scripts" / "asha_model"
    cfg = yaml.safe_load((ex / "adaptive.yaml").read_text())
    cfg["searcher"]["max_trials"] = args.max_trials
    cfg.setdefault("reproducibility", {})["experiment_seed"] = args.seed
    if args.no_hip_graph:
        cfg.setdefault("optimizations", {})["hip_graph"] = False
    if args.graph_batches:
        cfg.setdefault("optimizations", {})["hip_graph_batches"] = args.graph_batches
    if args.amp:
        cfg["hyperparameters"]["amp"] = args.amp
    if args.validation_records:
        cfg["hyperparameters"]["validation_records"] = args.validation_records
    if args.max_length_batches:
        cfg["searcher"]["max_length"] = {"batches": args.max_length_batches}
        # validate only where the searcher asks (end of each rung); the real config validates every
        # epoch = 1/32 of max_length, which a scaled-down max_length would turn into a validation storm
        cfg.pop("min_validation_period", None)
        cfg["scheduling_unit"] = 50
        cfg.pop("records_per_epoch", None)
    env_vars = cfg.setdefault("environment", {}).setdefault("environment_variables", [])
    env_vars.append("DET_TIMELINE=1")
    if args.modelled_batch_ms:
        env_vars.append(f"DET_MODEL_BATCH_MS={args.modelled_batch_ms}")
    env_vars.append("PYTHONFAULTHANDLER=1")  # a crashing trial logs its Python stack
    if args.artificial_slots:
        env_vars.append("OMP_NUM_THREADS=1")  # N CPU trial processes share the host's cores
        if not args.modelled_batch_ms:
            # a scheduler dry run: a 10k-record validation pass per rung on one CPU thread per trial
            # would dominate the wall time it measures (the modelled trial keeps the real 10k)
            cfg["hyperparameters"]["validation_records"] = 512
    busy = []
    stop = threading.Event()

    def sample() -> None:
        while not stop.wait(0.5):
            u = gpu.utilization()
            if u:
                busy.append(sum(x.get("gpu_busy_percent", 0) for x in u) / len(u))

    visible = ",".join(str(i) for i in range(args.slots)) if args.slots and not args.artificial_slots else None
    with LocalCluster(agents=1, slots_per_agent=args.artificial_slots, gpu=args.artificial_slots == 0,
                      log_dir=os.environ.get("DET_BENCH_LOGDIR", "/tmp"), visible_gpus=visible,
                      agent_args=["--no-zygote"] if args.no_zygote else []) as c:
        if args.artificial_slots == 0:
            c.wait_for_slots(args.slots or 1, timeout=60)
        cl = MasterClient(c.address)
        th = threading.Thread(target=sample, daemon=True)
        th.start()
        t0 = time.time()
        eid = cl.create_experiment(cfg, read_context(ex))["id"]
        state = None
        last = 0.0
        peak_busy = 0
        while time.time() - t0 < args.timeout:  # progress line every 20 s (long runs must not look hung)
            ex = cl.experiment(eid)
            state = ex["state"]
            peak_busy = max(peak_busy, sum(1 for a in cl.get("/agents") for sl in a["slots"] if sl.get("task")))
            if state in ("COMPLETED", "CANCELED", "ERROR"):
                break
            if time.time() - last > 20:
                last = time.time()
                ts = ex["trials"]
                print(f"[bench_asha] +{time.time() - t0:6.0f}s state={state} trials={len(ts)} "
                      f"completed={sum(t['state'] == 'COMPLETED' for t in ts)} "
                      f"batches={sum(t.get('total_batches_processed', 0) for t in ts)}", file=sys.stderr, flush=True)
            # 0.2 s: the wall clock is read when the poll sees COMPLETED, so a coarse poll inflates it
            # (a 2 s poll quantised every run of the 16-trial shape to 64.2 s)
            time.sleep(0.2)
        wall = time.time() - t0
        stop.set()
        e = cl.experiment(eid)
        done = sum(1 for t in e["trials"] if t["state"] == "COMPLETED")
        timeline = summarize_timelines(cl, e["trials"], t0)
        restarted = [t for t in e["trials"] if t.get("restarts", 0) or t["state"] != "COMPLETED"]
        if restarted:  # keep the tail of every failing trial's log next to the timeline
            with open(os.path.join(os.environ.get("DET_BENCH_LOGDIR", "/tmp"), "asha_failed_trials.txt"), "w") as f:
                for t in restarted:
                    recs = cl.get(f"/trials/{t['id']}/logs")
                    f.write(f"==== trial {t['id']} state={t['state']} restarts={t.get('restarts')}\n")
                    f.write("\n".join(r.get("message", "").rstrip() for r in recs[-150:]) + "\n")
        slots = sum(len(a["slots"]) for a in cl.get("/agents"))
        try:
            idle = idle_breakdown(cl, e["trials"], slots, t0, t0 + wall)
        except Exception as ex:  # diagnostics only
            idle = {"error": f"{type(ex).__name__}: {ex}"[:200]}
        try:
            cp = control_plane_breakdown(cl, e["trials"], slots, t0, t0 + wall)
        except Exception as ex:  # diagnostics only
            cp = {"error": f"{type(ex).__name__}: {ex}"[:200]}
        containers = timeline.pop("_containers", 0)
        if "work_frac" in cp:
            # the master's round trip between a container's workloads (sequencer, searcher, socket) is
            # control plane too: taken out of "work"
            bw = timeline.get("between workloads", 0.0) * containers / max(1e-9, wall * slots)
            cp["between_workloads_frac"] = round(bw, 4)
            cp["work_frac"] = round(cp["work_frac"] - bw, 4)
            cp["control_plane_idle_frac"] = round(cp["control_plane_idle_frac"] + bw, 4)
        # slot occupancy from the container log spans (idle_breakdown); the per-container timeline
        # totals are kept for the phase split only
        occupancy = (1.0 - idle["idle_frac"]) if "idle_frac" in idle else \
            timeline.get("total", 0.0) * containers / max(1e-9, wall * slots)
        records = sum(t.get("total_batches_processed", 0) * t.get("hparams", {}).get("global_batch_size", 0)
                      for t in e["trials"])
        print(json.dumps({"metric": "ASHA trials/hr (16-trial adaptive_asha CIFAR-10)",
                          "value": round(done * 3600.0 / wall, 2), "unit": "trials/hr", "state": state,
                          "trials_completed": done, "wall_s": round(wall, 1), "slots": slots,
                          "containers": containers, "train_records": records,
                          "gpu_busy_frac": round(sum(busy) / len(busy) / 100.0, 3) if busy else None,
                          "slot_occupancy": round(occupancy, 3), "scheduler_idle_frac": round(1 - occupancy, 3),
                          "peak_busy_slots": peak_busy, "idle_breakdown": idle, "control_plane": cp,
                          "modelled_batch_ms": args.modelled_batch_ms or None,
                          "zygote": not args.no_zygote, "per_container_s": timeline,
                          "hip_graph": bool((cfg.get("optimizations") or {}).get("hip_graph", False)),
                          "hip_graph_batches": (cfg.get("optimizations") or {}).get("hip_graph_batches", 1),
                          "experiment_seed": args.seed,
                          "config": {"max_length": cfg["searcher"]["max_length"], "max_trials": args.max_trials,
                                     "records_per_epoch": cfg.get("records_per_epoch"),
                                     "min_validation_period": cfg.get("min_validation_period"),
                                     "searcher": "adaptive_asha", "amp": cfg["hyperparameters"].get("amp")}}),
              flush=True)


if __name__ == "__main__":
    main()
