"""``det`` CLI: experiment / trial / checkpoint / model / agent / slot / template / preview-search /
deploy / version (reference ``cli/determined_cli/cli.py:73-171``, ``experiment.py``, ``trial.py``).

    python -m determined_1_amd.cli -m 127.0.0.1:8080 experiment create const.yaml model_dir
"""
import argparse
import json
import os
import pathlib
import sys
import time
from typing import Any, Dict, List

import yaml

from determined_1_amd import __version__
from determined_1_amd.api import MasterClient, read_context
from determined_1_amd.api.request import make_url
from determined_1_amd.config import merge_with_defaults, validate_experiment_config


def _load_config(path: str) -> Dict[str, Any]:
    with open(path) as f:
        return yaml.safe_load(f) or {}


def _table(rows: List[Dict[str, Any]], cols: List[str]) -> str:
    if not rows:
        return "(none)"
    w = {c: max(len(c), *(len(str(r.get(c, ""))) for r in rows)) for c in cols}
    line = " | ".join(c.ljust(w[c]) for c in cols)
    out = [line, "-+-".join("-" * w[c] for c in cols)]
    for r in rows:
        out.append(" | ".join(str(r.get(c, "")).ljust(w[c]) for c in cols))
    return "\n".join(out)


def make_test_config(cfg: Dict[str, Any]) -> Dict[str, Any]:
    """Test mode (reference ``api/experiment.py:258-299``): 1-batch single search, validation every
    batch, no restarts, sampled hyperparameters."""
    import random

    c = json.loads(json.dumps(cfg))
    hps = {}
    for name, hp in (c.get("hyperparameters") or {}).items():
        if not isinstance(hp, dict) or "type" not in hp:
            hps[name] = hp
        elif hp["type"] == "const":
            hps[name] = hp["val"]
        elif hp["type"] == "int":
            hps[name] = random.randint(hp["minval"], hp["maxval"])
        elif hp["type"] == "double":
            hps[name] = random.uniform(hp["minval"], hp["maxval"])
        elif hp["type"] == "log":
            hps[name] = hp.get("base", 10.0) ** random.uniform(hp["minval"], hp["maxval"])
        elif hp["type"] == "categorical":
            hps[name] = random.choice(hp["vals"])
    c["hyperparameters"] = {k: {"type": "const", "val": v} for k, v in hps.items()}
    metric = c.get("searcher", {}).get("metric", "validation_loss")
    c["searcher"] = {"name": "single", "metric": metric, "max_length": {"batches": 1},
                     "smaller_is_better": c.get("searcher", {}).get("smaller_is_better", True)}
    c["scheduling_unit"] = 1
    c["min_validation_period"] = {"batches": 1}
    c["max_restarts"] = 0
    cs = c.setdefault("checkpoint_storage", {})
    cs.update({"save_experiment_best": 0, "save_trial_best": 0, "save_trial_latest": 0})
    c.pop("min_checkpoint_period", None)
    return c


# --------------------------------------------------------------------------- experiment
def cmd_experiment_create(args: argparse.Namespace) -> None:
    cfg = _load_config(args.config_file)
    for kv in args.config or []:
        k, v = kv.split("=", 1)
        node = cfg
        parts = k.split(".")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = yaml.safe_load(v)
    if args.test_mode:
        cfg = make_test_config(cfg)
    errs = validate_experiment_config(merge_with_defaults(cfg))
    if errs:
        sys.exit("invalid experiment config:\n  " + "\n  ".join(errs))
    if args.local:
        from determined_1_amd.experimental import run_local_test

        run_local_test(cfg, args.model_def)
        print("local test mode passed")
        return
    client = MasterClient(args.master)
    ctx = read_context(pathlib.Path(args.model_def))
    r = client.create_experiment(cfg, ctx, activate=not args.paused, template=args.template)
    eid = r["id"]
    print(f"Created experiment {eid}")
    if args.test_mode or args.follow:
        st = _follow(client, eid)
        if args.test_mode:
            if st != "COMPLETED":
                sys.exit(f"test experiment {eid} ended in state {st}")
            client.patch(f"/experiments/{eid}", {"archived": True})
            print("Model definition test succeeded!")


def _follow(client: MasterClient, eid: int) -> str:
    seen = {}  # type: Dict[int, int]
    while True:
        e = client.experiment(eid)
        for t in e.get("trials", []):
            off = seen.get(t["id"], 0)
            for l in client.get(f"/trials/{t['id']}/logs", offset=off):
                print(f"[trial {t['id']}] {l['message']}")
                seen[t["id"]] = l["id"]
        if e["state"] in ("COMPLETED", "CANCELED", "ERROR"):
            print(f"Experiment {eid} {e['state']}")
            return e["state"]
        time.sleep(1.0)


def cmd_experiment_list(args: argparse.Namespace) -> None:
    rows = MasterClient(args.master).get("/experiments", all="true" if args.all else "false")
    print(_table(rows, ["id", "state", "searcher", "num_trials", "progress", "start_time", "description"]))


def cmd_experiment_describe(args: argparse.Namespace) -> None:
    e = MasterClient(args.master).experiment(args.experiment_id)
    if args.json:
        print(json.dumps(e, indent=2))
        return
    print(f"Experiment {e['id']}: {e['state']}  progress={e.get('progress')}  searcher={e['config']['searcher'].get('name')}")
    print(_table(e["trials"], ["id", "state", "total_batches_processed", "best_validation_metric", "restarts"]))


def _set_state(state: str):
    def f(args: argparse.Namespace) -> None:
        MasterClient(args.master).set_state(args.experiment_id, state)
        print(f"experiment {args.experiment_id}: {state}")

    return f


def cmd_experiment_kill(args: argparse.Namespace) -> None:
    MasterClient(args.master).post(f"/experiments/{args.experiment_id}/kill")
    print(f"killed experiment {args.experiment_id}")


def cmd_experiment_archive(args: argparse.Namespace, archived: bool = True) -> None:
    MasterClient(args.master).patch(f"/experiments/{args.experiment_id}", {"archived": archived})


def cmd_experiment_delete(args: argparse.Namespace) -> None:
    MasterClient(args.master).delete(f"/experiments/{args.experiment_id}")
    print(f"deleted experiment {args.experiment_id}")


def cmd_experiment_wait(args: argparse.Namespace) -> None:
    st = MasterClient(args.master).wait_for_experiment(args.experiment_id, timeout=args.timeout)
    print(st)
    if st != "COMPLETED":
        sys.exit(1)


def cmd_experiment_download_model_def(args: argparse.Namespace) -> None:
    import base64

    md = MasterClient(args.master).get(f"/experiments/{args.experiment_id}/model_def")
    out = pathlib.Path(args.output_dir)
    for f in md["files"]:
        p = out.joinpath(f["path"])
        if f.get("type") == "dir":
            p.mkdir(parents=True, exist_ok=True)
            continue
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(base64.b64decode(f["content"]))
    print(f"wrote {len(md['files'])} entries to {out}")


def cmd_experiment_metrics(args: argparse.Namespace) -> None:
    """Follows ``/api/v1/experiments/:id/metrics-stream/trials-sample`` (the WebUI's learning-curve
    feed): one line per new (trial, batches, value) point until the experiment ends."""
    c = MasterClient(args.master)
    mtype = "METRIC_TYPE_TRAINING" if args.type == "training" else "METRIC_TYPE_VALIDATION"
    for msg in c.trials_sample(args.experiment_id, args.metric, mtype, period_seconds=args.period,
                               max_trials=args.max_trials):
        for t in msg.get("trials", []):
            for d in t.get("data", []):
                print(f"trial {t['trialId']}\tbatches {d['batches']}\t{args.metric} {d['value']:.6g}", flush=True)
        if not args.follow:
            return


def cmd_experiment_config(args: argparse.Namespace) -> None:
    print(yaml.safe_dump(MasterClient(args.master).experiment(args.experiment_id)["config"], sort_keys=False), end="")


def cmd_experiment_list_trials(args: argparse.Namespace) -> None:
    e = MasterClient(args.master).experiment(args.experiment_id)
    rows = [{"id": t["id"], "state": t["state"], "batches": t.get("total_batches_processed", 0),
             "best": t.get("best_validation_metric"), "hparams": json.dumps(t.get("hparams", {}))} for t in e["trials"]]
    print(_table(rows, ["id", "state", "batches", "best", "hparams"]))


def cmd_experiment_label(args: argparse.Namespace) -> None:
    c = MasterClient(args.master)
    e = c.experiment(args.experiment_id)
    labels = list(e.get("labels") or e["config"].get("labels") or [])
    if args.action == "add" and args.label not in labels:
        labels.append(args.label)
    elif args.action == "remove":
        labels = [l for l in labels if l != args.label]
    c.patch(f"/experiments/{args.experiment_id}", {"labels": labels})


def cmd_experiment_set(args: argparse.Namespace) -> None:
    """reference ``det experiment set {description,gc-policy,max-slots,weight,priority}``."""
    c = MasterClient(args.master)
    eid = args.experiment_id
    if args.field == "description":
        body = {"description": args.value}
    elif args.field == "gc-policy":
        keys = ("save_experiment_best", "save_trial_best", "save_trial_latest")
        vals = dict(zip(keys, (int(v) for v in args.value.split(","))))
        if len(vals) != 3:
            sys.exit("gc-policy takes SAVE_EXPERIMENT_BEST,SAVE_TRIAL_BEST,SAVE_TRIAL_LATEST")
        body = {"checkpoint_storage": vals}
    elif args.field == "max-slots":
        body = {"resources": {"max_slots": int(args.value)}}
    elif args.field == "weight":
        body = {"resources": {"weight": float(args.value)}}
    else:
        body = {"resources": {"priority": int(args.value)}}
    c.patch(f"/experiments/{eid}", body)


def cmd_experiment_download(args: argparse.Namespace) -> None:
    """Download the experiment's top-N checkpoints (reference ``det experiment download``)."""
    from determined_1_amd.experimental import Determined

    exp = Determined(args.master).get_experiment(args.experiment_id)
    for ck in exp.top_n_checkpoints(args.top_n):
        path = ck.download(args.output_dir)
        print(f"checkpoint {ck.uuid} -> {path}")


def cmd_experiment_checkpoints(args: argparse.Namespace) -> None:
    rows = MasterClient(args.master).get(f"/experiments/{args.experiment_id}/checkpoints")
    if args.best is not None:
        rows = rows[: args.best]
    print(_table(rows, ["uuid", "trial_id", "step_id", "total_batches_processed", "searcher_metric", "state"]))


# ------------------------------------------------------------------------------- trial
def cmd_trial_describe(args: argparse.Namespace) -> None:
    t = MasterClient(args.master).get(f"/trials/{args.trial_id}")
    if args.json:
        print(json.dumps(t, indent=2))
        return
    print(f"Trial {t['id']} (experiment {t['experiment_id']}): {t['state']}  hparams={json.dumps(t['hparams'])}")
    rows = [{"step": s["step_id"], "state": s["state"], "batches": s.get("num_batches"),
             "metrics": json.dumps((s.get("metrics") or {}).get("avg_metrics"))} for s in t["steps"]]
    print(_table(rows, ["step", "state", "batches", "metrics"]))


def cmd_trial_logs(args: argparse.Namespace) -> None:
    """Streams ``GET /api/v1/trials/:id/logs`` (reference ``det trial logs``)."""
    c = MasterClient(args.master)
    filters = {}
    if args.rank is not None:
        filters["rank_ids"] = [args.rank]
    if args.stdtype:
        filters["stdtypes"] = [args.stdtype]
    for l in c.trial_logs(args.trial_id, follow=args.follow, tail=args.tail, **filters):
        if args.contains and args.contains not in l["message"]:
            continue
        print(l["message"], flush=True)


def cmd_trial_download(args: argparse.Namespace) -> None:
    """reference ``det trial download``: the trial's best (default), latest or given checkpoint."""
    from determined_1_amd.experimental import Determined

    t = Determined(args.master).get_trial(args.trial_id)
    ck = t.select_checkpoint(latest=args.latest, best=not args.latest and not args.uuid, uuid=args.uuid)
    print(f"checkpoint {ck.uuid} -> {ck.download(args.output_dir)}")


def cmd_master_logs(args: argparse.Namespace) -> None:
    """Streams ``GET /api/v1/master/logs``; ``--tail N`` starts N lines before the end."""
    c = MasterClient(args.master)
    offset = 0
    if args.tail:
        ids = [l["logEntry"]["id"] for l in c.stream("/api/v1/master/logs", limit=100000)]
        offset = ids[-args.tail] - 1 if len(ids) >= args.tail else 0
    for l in c.stream("/api/v1/master/logs", offset=offset, follow=args.follow):
        print(l["logEntry"]["message"], flush=True)


def cmd_trial_kill(args: argparse.Namespace) -> None:
    MasterClient(args.master).post(f"/trials/{args.trial_id}/kill")


# -------------------------------------------------------------------------- checkpoint
def cmd_checkpoint_describe(args: argparse.Namespace) -> None:
    print(json.dumps(MasterClient(args.master).get(f"/checkpoints/{args.uuid}"), indent=2))


def cmd_checkpoint_download(args: argparse.Namespace) -> None:
    from determined_1_amd.experimental import Determined

    path = Determined(args.master).get_checkpoint(args.uuid).download(args.output_dir)
    print(path)


# ----------------------------------------------------------------------- agents / slots
def cmd_agent_list(args: argparse.Namespace) -> None:
    rows = [{"id": a["id"], "resource_pool": a.get("resource_pool"), "slots": len(a["slots"]),
             "used": sum(1 for s in a["slots"] if s["task"]), "enabled": a["enabled"], "label": a["label"]}
            for a in MasterClient(args.master).get("/agents")]
    print(_table(rows, ["id", "resource_pool", "slots", "used", "enabled", "label"]))


def cmd_slot_list(args: argparse.Namespace) -> None:
    rows = []
    for a in MasterClient(args.master).get("/agents"):
        for s in a["slots"]:
            rows.append({"agent": a["id"], "slot": s["id"], "type": s["type"], "uuid": s["uuid"],
                         "enabled": s["enabled"], "task": s["task"]})
    print(_table(rows, ["agent", "slot", "type", "uuid", "enabled", "task"]))


def _slot_toggle(enable: bool):
    def f(args: argparse.Namespace) -> None:
        path = f"/agents/{args.agent_id}/slots/{args.slot_id}/" if args.slot_id is not None else f"/agents/{args.agent_id}/"
        MasterClient(args.master).post(path + ("enable" if enable else "disable"))

    return f


def cmd_resource_pools(args: argparse.Namespace) -> None:
    print(_table(MasterClient(args.master).get("/resource_pools"),
                 ["name", "scheduler", "num_slots", "slots_used", "num_tasks", "tasks_pending"]))


# ---------------------------------------------------------------------------- templates
def cmd_template_list(args: argparse.Namespace) -> None:
    print(_table(MasterClient(args.master).get("/templates"), ["name"]))


def cmd_template_set(args: argparse.Namespace) -> None:
    MasterClient(args.master).put(f"/templates/{args.name}", {"config": _load_config(args.template_file)})


def cmd_template_describe(args: argparse.Namespace) -> None:
    print(yaml.safe_dump(MasterClient(args.master).get(f"/templates/{args.name}")["config"]))


def cmd_template_remove(args: argparse.Namespace) -> None:
    MasterClient(args.master).delete(f"/templates/{args.name}")


# ------------------------------------------------------------------------------- models
def cmd_model_create(args: argparse.Namespace) -> None:
    print(json.dumps(MasterClient(args.master).post(f"/models/{args.name}", {"description": args.description or ""})))


def cmd_model_list(args: argparse.Namespace) -> None:
    print(_table(MasterClient(args.master).get("/models"), ["name", "description", "creation_time"]))


def cmd_model_describe(args: argparse.Namespace) -> None:
    print(json.dumps(MasterClient(args.master).get(f"/models/{args.name}"), indent=2))


def cmd_model_register(args: argparse.Namespace) -> None:
    print(json.dumps(MasterClient(args.master).post(f"/models/{args.name}/versions", {"checkpoint_uuid": args.uuid})))


# -------------------------------------------------------------------------------- users
def cmd_user_login(args: argparse.Namespace) -> None:
    import getpass

    pw = args.password if args.password is not None else getpass.getpass(f"Password for user '{args.username}': ")
    MasterClient(args.master).login(args.username, pw)
    print(f"logged in as {args.username}")


def cmd_user_logout(args: argparse.Namespace) -> None:
    from determined_1_amd.api.request import save_token

    c = MasterClient(args.master)
    c.post("/logout")
    save_token(c.master, None)


def cmd_user_whoami(args: argparse.Namespace) -> None:
    print(MasterClient(args.master).get("/me")["username"])


def cmd_user_list(args: argparse.Namespace) -> None:
    rows = MasterClient(args.master).get("/users")
    for r in rows:
        g = r.get("agent_user_group") or {}
        r["agent_user"] = f"{g['user']}:{g['group']} ({g['uid']}:{g['gid']})" if g else ""
    print(_table(rows, ["username", "admin", "active", "agent_user"]))


def cmd_user_create(args: argparse.Namespace) -> None:
    MasterClient(args.master).post("/users", {"username": args.username, "password": args.password or "",
                                              "admin": args.admin})


def cmd_user_change_password(args: argparse.Namespace) -> None:
    MasterClient(args.master).patch(f"/users/{args.username}", {"password": args.password})


def cmd_user_link_with_agent_user(args: argparse.Namespace) -> None:
    """Tasks of ``det_username`` run on agents as this host account (reference
    cli/determined_cli/user.py:165-185 link_with_agent_user); admin only."""
    for flag in ("agent_uid", "agent_user", "agent_gid", "agent_group"):
        if getattr(args, flag) is None:
            raise SystemExit(f"--{flag.replace('_', '-')} argument required")
    MasterClient(args.master).patch(f"/users/{args.det_username}", {"agent_user_group": {
        "uid": args.agent_uid, "user": args.agent_user, "gid": args.agent_gid, "group": args.agent_group}})
    print(f"linked {args.det_username} with {args.agent_user}:{args.agent_group} "
          f"({args.agent_uid}:{args.agent_gid}) on the agents")


# ----------------------------------------------------------------------------- commands
def cmd_command_run(args: argparse.Namespace) -> None:
    cfg = {"entrypoint": args.entrypoint, "resources": {"slots": args.slots},
           "description": args.description or " ".join(args.entrypoint)}
    if args.config_file:
        cfg.update(_load_config(args.config_file))
    ctx = read_context(pathlib.Path(args.context)) if args.context else []
    client = MasterClient(args.master)
    cid = client.post("/commands", {"config": cfg, "context": ctx})["id"]
    print(f"Launched command {cid}")
    if args.detach:
        return
    off = 0
    while True:
        for l in client.get(f"/commands/{cid}/logs", offset=off):
            print(l["message"])
            off = l["id"]
        c = client.get(f"/commands/{cid}")
        if c["state"] == "TERMINATED":
            for l in client.get(f"/commands/{cid}/logs", offset=off):
                print(l["message"])
            if c.get("exit_code", 0) != 0:
                sys.exit(c.get("exit_code", 1))
            return
        time.sleep(0.5)


def cmd_command_list(args: argparse.Namespace) -> None:
    print(_table(MasterClient(args.master).get("/commands"), ["id", "state", "description", "agent", "exit_code"]))


def cmd_command_logs(args: argparse.Namespace) -> None:
    for l in MasterClient(args.master).get(f"/commands/{args.command_id}/logs"):
        print(l["message"])


def cmd_tensorboard_start(args: argparse.Namespace) -> None:
    """``det tensorboard start <exp ids>``: a zero-slot command task running the scalar dashboard
    (determined_1_amd/tensorboard/serve.py), reachable through the master's /proxy/cmd-<id>/."""
    client = MasterClient(args.master)
    eids = ",".join(str(e) for e in args.experiment_ids)
    argv = ["python3", "-m", "determined_1_amd.tensorboard.serve", "--experiment-ids", eids]
    if args.trial_ids:
        argv += ["--trial-ids", ",".join(str(t) for t in args.trial_ids)]
    cfg = {"entrypoint": argv, "type": "tensorboard", "resources": {"slots": 0},
           "description": f"TensorBoard (Experiment {eids})"}
    cid = client.post("/commands", {"config": cfg, "context": []})["id"]
    url = make_url(client.master, f"/proxy/cmd-{cid}/")
    if not args.detach:
        deadline = time.time() + args.timeout
        while time.time() < deadline:
            c = client.get(f"/commands/{cid}")
            if c.get("ready") or c.get("state") == "TERMINATED":
                break
            time.sleep(0.5)
    print(f"TensorBoard {cid}: {url}")


def cmd_tensorboard_list(args: argparse.Namespace) -> None:
    rows = MasterClient(args.master).get("/commands", type="tensorboard")
    print(_table(rows, ["id", "state", "description", "ready", "service_address"]))


def cmd_command_kill(args: argparse.Namespace) -> None:
    MasterClient(args.master).post(f"/commands/{args.command_id}/kill")


def _start_task(client: MasterClient, kind: str, argv: List[str], secret_env: List[str], slots: int,
                description: str, wait: float) -> int:
    """Start a command task; ``secret_env`` ("K=V") reaches only the container's environment -- the
    master keeps it out of the stored config that GET /commands returns."""
    cfg = {"entrypoint": argv, "type": kind, "resources": {"slots": slots}, "description": description}
    cid = client.post("/commands", {"config": cfg, "context": [], "secret_environment": secret_env})["id"]
    deadline = time.time() + wait
    while time.time() < deadline:
        c = client.get(f"/commands/{cid}")
        if c.get("ready") or c.get("state") == "TERMINATED":
            break
        time.sleep(0.2)
    return cid


def cmd_shell_start(args: argparse.Namespace) -> None:
    """``det shell start``: a shell task (exec/shell.py) with a fresh token; attaches unless -d."""
    import secrets

    client = MasterClient(args.master)
    token = secrets.token_hex(16)
    cid = _start_task(client, "shell", ["python3", "-m", "determined_1_amd.exec.shell"],
                      [f"DET_SHELL_TOKEN={token}"], args.slots, "Shell", args.timeout)
    _save_shell_token(client.master, cid, token)
    c = client.get(f"/commands/{cid}")
    if not c.get("ready"):
        sys.exit(f"shell {cid} did not become ready (state {c.get('state')})")
    print(f"Shell {cid} ready", file=sys.stderr)
    if not args.detach:
        from determined_1_amd.exec.shell import open_shell

        sys.exit(open_shell(client, cid, token))


def _shell_token_path(master: str) -> str:
    return os.path.join(os.path.expanduser("~"), ".det-mi355x", "shells-" + master.replace(":", "_") + ".json")


def _save_shell_token(master: str, cid: int, token: str) -> None:
    p = _shell_token_path(master)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    data = json.load(open(p)) if os.path.exists(p) else {}
    data[str(cid)] = token
    fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    with os.fdopen(fd, "w") as f:
        json.dump(data, f)


def cmd_shell_open(args: argparse.Namespace) -> None:
    from determined_1_amd.exec.shell import open_shell

    client = MasterClient(args.master)
    p = _shell_token_path(client.master)
    token = (json.load(open(p)) if os.path.exists(p) else {}).get(str(args.shell_id))
    if not token:
        sys.exit(f"no token for shell {args.shell_id}: only the CLI that started it can open it")
    sys.exit(open_shell(client, args.shell_id, token))


def cmd_notebook_start(args: argparse.Namespace) -> None:
    import secrets

    client = MasterClient(args.master)
    token = secrets.token_hex(16)
    cid = _start_task(client, "notebook", ["python3", "-m", "determined_1_amd.exec.notebook"],
                      [f"DET_NOTEBOOK_TOKEN={token}"], args.slots, "Notebook", args.timeout)
    c = client.get(f"/commands/{cid}")
    if not c.get("ready"):
        logs = "\n".join(l["message"] for l in client.get(f"/commands/{cid}/logs"))
        sys.exit(f"notebook {cid} did not become ready (state {c.get('state')}):\n{logs}")
    print(f"Notebook {cid}: {make_url(client.master, f'/proxy/cmd-{cid}/')}?token={token}")


def cmd_task_list(kind: str):
    def f(args: argparse.Namespace) -> None:
        rows = MasterClient(args.master).get("/commands", type=kind)
        print(_table(rows, ["id", "state", "description", "ready", "service_address"]))

    return f


# ---------------------------------------------------------------------------- misc
def cmd_preview_search(args: argparse.Namespace) -> None:
    cfg = _load_config(args.config_file)
    if args.master_side:
        r = MasterClient(args.master).post("/searcher/preview", {"config": cfg})
        results = r["results"]
    else:
        from determined_1_amd.searcher import simulate_config

        results = simulate_config(cfg)["results"]
    total = sum(results.values())
    print(f"Using search configuration:\n{yaml.safe_dump(cfg.get('searcher', {}))}")
    print(f"This search will create a total of {total} trial(s).")
    for ops, n in sorted(results.items(), key=lambda kv: -kv[1]):
        print(f"  {n:5d} trial(s): {ops}")


def cmd_version(args: argparse.Namespace) -> None:
    print(f"client: {__version__}")
    try:
        print("master:", json.dumps(MasterClient(args.master, timeout=3).get("/info")))
    except Exception as e:  # noqa: BLE001
        print(f"master: unreachable ({e})")


def cmd_master_config(args: argparse.Namespace) -> None:
    print(json.dumps(MasterClient(args.master).get("/master/config"), indent=2))


def _cloud_deploy(cloud: str, rest: List[str]) -> int:
    from determined_1_amd.deploy import cloud_deploy

    return cloud_deploy.main([cloud] + rest)


def cmd_deploy_local(args: argparse.Namespace) -> None:
    from determined_1_amd.deploy import LocalCluster

    c = LocalCluster(agents=args.agents, slots_per_agent=args.artificial_slots, port=args.port,
                     store_dir=args.store_dir, checkpoint_dir=args.checkpoint_dir, gpu=args.gpu,
                     scheduler=args.scheduler)
    c.up()
    print(f"cluster up: DET_MASTER={c.address}  (Ctrl-C to stop)")
    grpc_server = None
    if args.grpc_port is not None:  # the gRPC wire protocol of the master API (determined_1_amd/rpc)
        from determined_1_amd.rpc.server import serve

        grpc_server, gport = serve(c.address, args.grpc_port)
        print(f"gRPC determined.api.v1.Determined on 127.0.0.1:{gport}")
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        if grpc_server is not None:
            grpc_server.stop(0)
        c.down()


def cmd_tunnel(args: argparse.Namespace) -> None:
    from determined_1_amd.cli import tunnel

    argv = [args.master, args.service]
    if args.listen is not None:
        argv += ["--listen", str(args.listen)]
    for k in ("cert_file", "cert_name"):
        if getattr(args, k):
            argv += ["--" + k.replace("_", "-"), getattr(args, k)]
    tunnel.main(argv)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="det", description="Determined (MI355X-native) command line")
    p.add_argument("-m", "--master", default=os.environ.get("DET_MASTER", "127.0.0.1:8080"))
    sub = p.add_subparsers(dest="cmd")

    e = sub.add_parser("experiment", aliases=["e"]).add_subparsers(dest="sub")
    c = e.add_parser("create")
    c.add_argument("config_file")
    c.add_argument("model_def")
    c.add_argument("--test-mode", "--test", action="store_true")
    c.add_argument("--local", action="store_true")
    c.add_argument("--paused", action="store_true")
    c.add_argument("--follow", "-f", action="store_true")
    c.add_argument("--template")
    c.add_argument("--config", action="append", help="override: key.sub=value")
    c.set_defaults(func=cmd_experiment_create)
    ls = e.add_parser("list")
    ls.add_argument("--all", "-a", action="store_true")
    ls.set_defaults(func=cmd_experiment_list)
    for name, fn in (("describe", cmd_experiment_describe),):
        d = e.add_parser(name)
        d.add_argument("experiment_id", type=int)
        d.add_argument("--json", action="store_true")
        d.set_defaults(func=fn)
    for name, fn in (("activate", _set_state("ACTIVE")), ("pause", _set_state("PAUSED")),
                     ("cancel", _set_state("STOPPING_CANCELED")), ("kill", cmd_experiment_kill),
                     ("archive", cmd_experiment_archive), ("unarchive", lambda a: cmd_experiment_archive(a, False)),
                     ("delete", cmd_experiment_delete)):
        d = e.add_parser(name)
        d.add_argument("experiment_id", type=int)
        d.set_defaults(func=fn)
    w = e.add_parser("wait")
    w.add_argument("experiment_id", type=int)
    w.add_argument("--timeout", type=float, default=86400)
    w.set_defaults(func=cmd_experiment_wait)
    dm = e.add_parser("download-model-def")
    dm.add_argument("experiment_id", type=int)
    dm.add_argument("--output-dir", default=".")
    dm.set_defaults(func=cmd_experiment_download_model_def)
    lc = e.add_parser("list-checkpoints")
    lc.add_argument("experiment_id", type=int)
    lc.add_argument("--best", type=int)
    lc.set_defaults(func=cmd_experiment_checkpoints)
    x = e.add_parser("config")
    x.add_argument("experiment_id", type=int)
    x.set_defaults(func=cmd_experiment_config)
    x = e.add_parser("list-trials", aliases=["lt"])
    x.add_argument("experiment_id", type=int)
    x.set_defaults(func=cmd_experiment_list_trials)
    x = e.add_parser("label")
    x.add_argument("action", choices=["add", "remove"])
    x.add_argument("experiment_id", type=int)
    x.add_argument("label")
    x.set_defaults(func=cmd_experiment_label)
    x = e.add_parser("set")
    x.add_argument("field", choices=["description", "gc-policy", "max-slots", "weight", "priority"])
    x.add_argument("experiment_id", type=int)
    x.add_argument("value")
    x.set_defaults(func=cmd_experiment_set)
    x = e.add_parser("download")
    x.add_argument("experiment_id", type=int)
    x.add_argument("--top-n", type=int, default=1)
    x.add_argument("--output-dir", default=None)
    x.set_defaults(func=cmd_experiment_download)
    mt = e.add_parser("metrics", help="stream a metric's learning curves (TrialsSample)")
    mt.add_argument("experiment_id", type=int)
    mt.add_argument("--metric", required=True)
    mt.add_argument("--type", choices=["training", "validation"], default="validation")
    mt.add_argument("--follow", "-f", action="store_true")
    mt.add_argument("--period", type=float, default=5.0)
    mt.add_argument("--max-trials", type=int, default=25)
    mt.set_defaults(func=cmd_experiment_metrics)

    t = sub.add_parser("trial", aliases=["t"]).add_subparsers(dest="sub")
    d = t.add_parser("describe")
    d.add_argument("trial_id", type=int)
    d.add_argument("--json", action="store_true")
    d.set_defaults(func=cmd_trial_describe)
    lg = t.add_parser("logs")
    lg.add_argument("trial_id", type=int)
    lg.add_argument("--follow", "-f", action="store_true")
    lg.add_argument("--tail", type=int)
    lg.add_argument("--rank", type=int)
    lg.add_argument("--stdtype", choices=["stdout", "stderr"])
    lg.add_argument("--contains")
    lg.set_defaults(func=cmd_trial_logs)
    k = t.add_parser("kill")
    k.add_argument("trial_id", type=int)
    k.set_defaults(func=cmd_trial_kill)
    x = t.add_parser("download")
    x.add_argument("trial_id", type=int)
    g = x.add_mutually_exclusive_group()
    g.add_argument("--best", action="store_true", default=True)
    g.add_argument("--latest", action="store_true")
    g.add_argument("--uuid")
    x.add_argument("--output-dir", default=None)
    x.set_defaults(func=cmd_trial_download)

    ck = sub.add_parser("checkpoint", aliases=["c"]).add_subparsers(dest="sub")
    d = ck.add_parser("describe")
    d.add_argument("uuid")
    d.set_defaults(func=cmd_checkpoint_describe)
    dl = ck.add_parser("download")
    dl.add_argument("uuid")
    dl.add_argument("--output-dir", "-o", default=None)
    dl.set_defaults(func=cmd_checkpoint_download)

    ag = sub.add_parser("agent", aliases=["a"]).add_subparsers(dest="sub")
    ag.add_parser("list").set_defaults(func=cmd_agent_list)
    for name, en in (("enable", True), ("disable", False)):
        x = ag.add_parser(name)
        x.add_argument("agent_id")
        x.set_defaults(func=_slot_toggle(en), slot_id=None)
    sl = sub.add_parser("slot", aliases=["s"]).add_subparsers(dest="sub")
    sl.add_parser("list").set_defaults(func=cmd_slot_list)
    for name, en in (("enable", True), ("disable", False)):
        x = sl.add_parser(name)
        x.add_argument("agent_id")
        x.add_argument("slot_id", type=int)
        x.set_defaults(func=_slot_toggle(en))
    rp = sub.add_parser("resource-pool", aliases=["rp"]).add_subparsers(dest="sub")
    rp.add_parser("list").set_defaults(func=cmd_resource_pools)

    tp = sub.add_parser("template", aliases=["tpl"]).add_subparsers(dest="sub")
    tp.add_parser("list").set_defaults(func=cmd_template_list)
    x = tp.add_parser("set")
    x.add_argument("name")
    x.add_argument("template_file")
    x.set_defaults(func=cmd_template_set)
    for name, fn in (("describe", cmd_template_describe), ("remove", cmd_template_remove)):
        x = tp.add_parser(name)
        x.add_argument("name")
        x.set_defaults(func=fn)

    md = sub.add_parser("model", aliases=["m"]).add_subparsers(dest="sub")
    x = md.add_parser("create")
    x.add_argument("name")
    x.add_argument("--description")
    x.set_defaults(func=cmd_model_create)
    md.add_parser("list").set_defaults(func=cmd_model_list)
    x = md.add_parser("describe")
    x.add_argument("name")
    x.set_defaults(func=cmd_model_describe)
    x = md.add_parser("register-version")
    x.add_argument("name")
    x.add_argument("uuid")
    x.set_defaults(func=cmd_model_register)

    us = sub.add_parser("user", aliases=["u"]).add_subparsers(dest="sub")
    x = us.add_parser("login")
    x.add_argument("username", nargs="?", default="determined")
    x.add_argument("--password")
    x.set_defaults(func=cmd_user_login)
    us.add_parser("logout").set_defaults(func=cmd_user_logout)
    us.add_parser("whoami").set_defaults(func=cmd_user_whoami)
    us.add_parser("list").set_defaults(func=cmd_user_list)
    x = us.add_parser("create")
    x.add_argument("username")
    x.add_argument("--password")
    x.add_argument("--admin", action="store_true")
    x.set_defaults(func=cmd_user_create)
    x = us.add_parser("change-password")
    x.add_argument("username")
    x.add_argument("password")
    x.set_defaults(func=cmd_user_change_password)
    x = us.add_parser("link-with-agent-user", help="link a user with a UID/GID on the agents")
    x.add_argument("det_username")
    x.add_argument("--agent-uid", type=int, help="UID on the agent to run tasks as")
    x.add_argument("--agent-user", help="user on the agent to run tasks as")
    x.add_argument("--agent-gid", type=int, help="GID on the agent to run tasks as")
    x.add_argument("--agent-group", help="group on the agent to run tasks as")
    x.set_defaults(func=cmd_user_link_with_agent_user)

    cm = sub.add_parser("command", aliases=["cmd"]).add_subparsers(dest="sub")
    x = cm.add_parser("run")
    x.add_argument("entrypoint", nargs="+")
    x.add_argument("--slots", type=int, default=0)
    x.add_argument("--config-file")
    x.add_argument("--context")
    x.add_argument("--description")
    x.add_argument("--detach", "-d", action="store_true")
    x.set_defaults(func=cmd_command_run)
    cm.add_parser("list").set_defaults(func=cmd_command_list)
    for name, fn in (("logs", cmd_command_logs), ("kill", cmd_command_kill)):
        x = cm.add_parser(name)
        x.add_argument("command_id", type=int)
        x.set_defaults(func=fn)
    tb = sub.add_parser("tensorboard").add_subparsers(dest="sub")
    x = tb.add_parser("start")
    x.add_argument("experiment_ids", type=int, nargs="+")
    x.add_argument("--trial-ids", type=int, nargs="*")
    x.add_argument("--detach", "-d", action="store_true")
    x.add_argument("--timeout", type=float, default=60)
    x.set_defaults(func=cmd_tensorboard_start)
    tb.add_parser("list").set_defaults(func=cmd_tensorboard_list)
    x = tb.add_parser("kill")
    x.add_argument("command_id", type=int)
    x.set_defaults(func=cmd_command_kill)
    sh = sub.add_parser("shell").add_subparsers(dest="sub")
    x = sh.add_parser("start")
    x.add_argument("--slots", type=int, default=0)
    x.add_argument("--detach", "-d", action="store_true")
    x.add_argument("--timeout", type=float, default=60)
    x.set_defaults(func=cmd_shell_start)
    x = sh.add_parser("open")
    x.add_argument("shell_id", type=int)
    x.set_defaults(func=cmd_shell_open)
    nb = sub.add_parser("notebook").add_subparsers(dest="sub")
    x = nb.add_parser("start")
    x.add_argument("--slots", type=int, default=1)
    x.add_argument("--timeout", type=float, default=120)
    x.set_defaults(func=cmd_notebook_start)
    for grp, kind in ((sh, "shell"), (nb, "notebook")):
        grp.add_parser("list").set_defaults(func=cmd_task_list(kind))
        for name, fn in (("logs", cmd_command_logs), ("kill", cmd_command_kill)):
            x = grp.add_parser(name)
            x.add_argument("command_id", type=int)
            x.set_defaults(func=fn)

    tn = sub.add_parser("tunnel", help="TCP stream to a task service through the master (stdio or --listen PORT)")
    tn.add_argument("service", help="command id or cmd-<id>")
    tn.add_argument("--listen", type=int, default=None)
    tn.add_argument("--cert-file")
    tn.add_argument("--cert-name")
    tn.set_defaults(func=cmd_tunnel)

    ps = sub.add_parser("preview-search")
    ps.add_argument("config_file")
    ps.add_argument("--master-side", action="store_true")
    ps.set_defaults(func=cmd_preview_search)
    sub.add_parser("version").set_defaults(func=cmd_version)
    mc = sub.add_parser("master").add_subparsers(dest="sub")
    mc.add_parser("config").set_defaults(func=cmd_master_config)
    x = mc.add_parser("logs")
    x.add_argument("--follow", "-f", action="store_true")
    x.add_argument("--tail", type=int, default=0)
    x.set_defaults(func=cmd_master_logs)

    dp = sub.add_parser("deploy").add_subparsers(dest="sub")
    lo = dp.add_parser("local")
    lo.add_argument("--agents", type=int, default=1)
    lo.add_argument("--artificial-slots", type=int, default=0)
    lo.add_argument("--gpu", action="store_true")
    lo.add_argument("--port", type=int, default=8080)
    lo.add_argument("--store-dir")
    lo.add_argument("--checkpoint-dir")
    lo.add_argument("--scheduler", default="fair_share")
    lo.add_argument("--grpc-port", type=int, default=None,
                    help="also serve the master API over gRPC (determined.api.v1.Determined) on this port")
    lo.set_defaults(func=cmd_deploy_local)
    for cloud in ("aws", "gcp"):
        x = dp.add_parser(cloud, help=f"master VM on {cloud.upper()} with the {cloud} agent provisioner",
                          add_help=False)
        x.add_argument("rest", nargs=argparse.REMAINDER)
        x.set_defaults(func=lambda a, cloud=cloud: sys.exit(_cloud_deploy(cloud, a.rest)))
    return p


def main(argv: List[str] = None) -> None:
    p = build_parser()
    args = p.parse_args(argv)
    if not getattr(args, "func", None):
        p.print_help()
        sys.exit(2)
    args.func(args)
