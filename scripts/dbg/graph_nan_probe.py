"""Locate the O2 hipGraph + dropout NaN of the CIFAR trial (README round 4, VERDICT r4 "weak" #1).

Runs the real CIFAR PyTorchTrial controller with per-batch (or chunked) graphs and checks, around
every replay, the invariants a correct replay must keep:

  * the bf16 model arena equals the fp32 master rounded to bf16 (nothing else writes parameters);
  * the gradient arena is zero after the step (zero_grad ran last);
  * the static input buffers hold the batch that was copied in;
  * loss, masters and optimizer state are finite.

On the first violation it dumps the pre-replay state (masters, RMSprop state, batch) and, on the
same box, re-runs that batch eagerly from the dumped state with many fresh dropout masks to see
whether any legitimate step produces a non-finite value.

Variants replace the model's dropout layers to separate the RNG kernel from the rest:
  torch    -- stock nn.Dropout / nn.Dropout2d (fused native_dropout kernel)
  randmask -- mask from torch.rand (uniform_ Philox kernel) * x
  bankmask -- mask read from a fixed bank by a device counter (no RNG kernel in the graph)

    python scripts/dbg/graph_nan_probe.py --variant torch --batches 2000 --out gpurun_out/nan
"""
import argparse
import json
import math
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
EX = os.path.join(REPO, "examples", "computer_vision", "cifar10_pytorch")
sys.path.insert(0, REPO)
sys.path.insert(0, EX)


def patch_dropout(model, variant):
    import torch
    import torch.nn as nn

    mods = [m for m in model.modules() if isinstance(m, nn.modules.dropout._DropoutNd) and m.p > 0]
    if variant == "none":
        for m in mods:
            m.p = 0.0
        return mods
    if variant == "torch":
        return mods

    def fwd(self, x):
        if not self.training:
            return x
        keep = 1.0 - self.p
        shape = tuple(x.shape[:2]) + (1,) * (x.dim() - 2) if isinstance(self, nn.Dropout2d) else tuple(x.shape)
        if variant == "randmask":
            m = (torch.rand(shape, device=x.device) < keep).to(x.dtype)
        else:
            if getattr(self, "_bank", None) is None:
                g = torch.Generator(device=x.device)
                g.manual_seed(1234 + id(self) % 1000)
                self._bank = (torch.rand((64,) + shape, device=x.device, generator=g) < keep).to(x.dtype)
                self._ctr = torch.zeros((), dtype=torch.long, device=x.device)
            m = self._bank.index_select(0, (self._ctr % 64).view(1))[0][: x.shape[0]]
            self._ctr.add_(1)
        return x * m * (1.0 / keep)

    for m in mods:
        m.forward = types.MethodType(fwd, m)
    return mods


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="torch", choices=("torch", "randmask", "bankmask", "none"))
    ap.add_argument("--separate-pools", action="store_true", help="each chunk graph captures into its own memory pool")
    ap.add_argument("--native", action="store_true", help="the native CNN kernels instead of torch layers")
    ap.add_argument("--amp", default="O2")
    ap.add_argument("--batches", type=int, default=2000)
    ap.add_argument("--graph-batches", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--out", default="gpurun_out/nanprobe")
    ap.add_argument("--eager-trials", type=int, default=64)
    ap.add_argument("--check-every", type=int, default=1,
                    help="synchronise and check invariants every N replays (1: every replay, as round-5 s2)")
    ap.add_argument("--loss", default="native", choices=("native", "torch", "torch_ce", "torch_acc"),
                    help="torch: round-4 train_batch (F.cross_entropy on out.float() + argmax accuracy); torch_ce / "
                         "torch_acc: only that half in torch, the other from the fused native kernel")
    ap.add_argument("--r4-model", action="store_true",
                    help="round-4 model: element Dropout after the first pool and RMSprop alpha 0.99")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    os.environ["DET_GRAPH_LIBRARY_CONVS"] = "1"  # capture the torch (MIOpen) layers anyway: this probe is about that defect
    import torch
    import torch.nn.functional as F

    from determined_1_amd import workload
    from determined_1_amd.experimental import make_controller
    from determined_1_amd.pytorch import _graph
    import model_def

    cfg = {"hyperparameters": {"global_batch_size": args.batch, "learning_rate": args.lr, "train_records": 50000,
                               "learning_rate_decay": 1e-6, "layer1_dropout": 0.25, "layer2_dropout": 0.25,
                               "layer3_dropout": 0.5, "amp": args.amp},
           "searcher": {"name": "single", "metric": "validation_error", "max_length": {"batches": args.batches}},
           "records_per_epoch": 50000, "scheduling_unit": 250,
           "optimizations": {"hip_graph": not args.no_graph, "hip_graph_batches": args.graph_batches}}

    step_losses = []

    def keep(r):
        m = r.get("metrics", {}).get("avg_metrics", {}) if isinstance(r, dict) else {}
        step_losses.append(float(m.get("loss", float("nan"))))

    def stream():
        done, step = 0, 1
        while done < args.batches:
            n = min(250, args.batches - done)
            yield workload.train_workload(step, num_batches=n, total_batches_processed=done), [], keep
            done += n
            step += 1
        yield workload.terminate_workload(step, total_batches_processed=done), [], workload.ignore_response

    # the torch layers by default: this probe is about torch dropout under replays
    os.environ["DET_NATIVE_CNN"] = "1" if args.native else "0"
    ctrl = make_controller(model_def.CIFARTrial, cfg, stream(), use_gpu=True, trial_seed=args.seed)
    trial = ctrl.trial
    if args.loss != "native":
        import torch.nn.functional as F

        native_ce = model_def.cross_entropy

        def loss_fn(out, y, with_accuracy=False, with_error=False):
            if args.loss == "torch":  # exactly round 4's train_batch
                lt, at = F.cross_entropy(out.float(), y), (out.argmax(1) == y).float().mean()
            else:
                ln, an = native_ce(out, y, with_accuracy=True)
                lt = F.cross_entropy(out.float(), y) if args.loss in ("torch", "torch_ce") else ln
                at = (out.argmax(1) == y).float().mean() if args.loss in ("torch", "torch_acc") else an
            outs = (lt,) + ((at,) if with_accuracy else ()) + ((1.0 - at,) if with_error else ())
            return outs if len(outs) > 1 else lt

        model_def.cross_entropy = loss_fn
    if args.r4_model:
        import torch.nn as nn

        trial.model.net[5] = nn.Dropout(trial.model.net[5].p)
        for g in trial.opt.param_groups:
            g["alpha"] = 0.99
    patch_dropout(trial.model, args.variant)
    ctx = ctrl.context
    state = {"batch": 0, "violation": None, "log": [], "t0": time.time()}
    names = {id(p): n for n, p in trial.model.named_parameters()}

    def fused():
        return [st.fused for st in ctx._opt_states if st.fused is not None]

    def snapshot():
        snap = []
        for f in fused():
            for gi, gs in enumerate(f.groups):
                for ai, a in enumerate(gs.arenas):
                    slots = {k: v.detach().clone() for k, v in gs.slots.get(ai, {}).items() if k != "master"}
                    snap.append({"master": a.master.detach().clone(), "param": a.flat_param.detach().clone(),
                                 "slots": slots, "names": [names.get(id(p), "?") for p in a.params],
                                 "offsets": list(a.offsets), "numels": list(a.numels)})
        return snap

    def check(tag, out, static_in=None, srcs=None):
        torch.cuda.synchronize()
        b = state["batch"]
        v = []
        loss = out.get("loss") if isinstance(out, dict) else out
        if loss is not None and not torch.isfinite(loss.float()).all():
            v.append("loss non-finite")
        for f in fused():
            for a in f.arenas:
                if not torch.isfinite(a.master).all():
                    bad = [names.get(id(p), "?") for p, pv in zip(a.params, a.param_views)
                           if not torch.isfinite(pv.float()).all()]
                    v.append(f"master non-finite {bad}")
                if a.has_master and not torch.equal(a.flat_param, a.master.to(a.flat_param.dtype)):
                    d = (a.flat_param.float() - a.master.to(a.flat_param.dtype).float()).abs()
                    v.append(f"model arena != bf16(master) at {int((d > 0).sum())} elements (max {float(d.max())})")
                if bool((a.flat_grad != 0).any()):
                    v.append(f"grad arena nonzero after step at {int((a.flat_grad != 0).sum())} elements")
        if static_in is not None:
            for d, s in zip(static_in, srcs):
                if not torch.equal(d, s):
                    v.append("static input differs from the batch copied in")
        if srcs:
            y = srcs[-1]
            if y.dtype == torch.long and (int(y.min()) < 0 or int(y.max()) > 9):
                v.append(f"label out of range [{int(y.min())}, {int(y.max())}]")
        if b % 100 == 0 or v:
            mx = max(float(a.master.abs().max()) for f in fused() for a in f.arenas)
            state["log"].append({"batch": b, "tag": tag, "loss": float(loss.float().mean()) if loss is not None else None,
                                 "max_abs_master": mx})
        return v

    orig_replay = _graph.TrainStepGraph._replay
    orig_eager = _graph.TrainStepGraph._eager
    pre = {"snap": None, "batch": None}

    def replay(self, g, leaves):
        every = args.check_every
        due = (state["batch"] + 1) % every == 0
        if state["violation"] is None and every == 1:
            pre["snap"] = snapshot()
            pre["batch"] = [x.detach().clone() for x in leaves if isinstance(x, torch.Tensor)]
        out = orig_replay(self, g, leaves)
        state["batch"] += 1
        if state["violation"] is None and due:
            v = check("replay", out, g.static_in, pre["batch"]) if every == 1 else check("replay", out)
            if v:
                state["violation"] = {"batch": state["batch"], "what": v, "tag": "replay"}
        return out

    def eager(self, batch, epoch_idx, batch_idx):
        capturing = torch.cuda.is_current_stream_capturing()
        if not capturing and state["violation"] is None:
            pre["snap"] = snapshot()
            pre["batch"] = [x.detach().clone() for x in batch if isinstance(x, torch.Tensor)]
        out = orig_eager(self, batch, epoch_idx, batch_idx)
        if not capturing:
            state["batch"] += 1
            if state["violation"] is None:
                v = check("eager", out, None, pre["batch"])
                if v:
                    state["violation"] = {"batch": state["batch"], "what": v, "tag": "eager"}
        return out

    orig_chunk = _graph.TrainStepGraph.run_chunk
    orig_cap_chunk = _graph.TrainStepGraph._capture_chunk
    state["chunks"] = 0

    def run_chunk(self, chunk, epoch_idx, batch_idx, capture=True):
        out = orig_chunk(self, chunk, epoch_idx, batch_idx, capture)
        if out is None:
            return out
        state["chunks"] += 1
        state["batch"] += len(chunk)
        if state["violation"] is None and state["chunks"] % max(1, args.check_every // 20) == 0:
            torch.cuda.synchronize()
            losses = out["loss"].float()
            v = []
            if not torch.isfinite(losses).all():
                first = int((~torch.isfinite(losses)).nonzero()[0])
                v.append(f"chunk loss non-finite from step {first} of {len(chunk)}")
            for f in fused():
                for a in f.arenas:
                    if not torch.isfinite(a.master).all():
                        v.append("master non-finite")
            if state["chunks"] % 5 == 0 or v:
                state["log"].append({"batch": state["batch"], "tag": "chunk", "loss": float(losses.mean()),
                                     "chunk_losses": [round(float(x), 4) for x in losses],
                                     "max_abs_master": max(float(a.master.abs().max()) for f in fused() for a in f.arenas)})
            if v:
                state["violation"] = {"batch": state["batch"], "what": v, "tag": "chunk", "epoch_idx": epoch_idx,
                                      "batch_idx": batch_idx, "chunk_losses": [float(x) for x in losses]}
        return out

    def capture_chunk(self, *a, **kw):
        if not args.separate_pools:
            return orig_cap_chunk(self, *a, **kw)
        keep = self.pool
        self.pool = torch.cuda.graph_pool_handle()
        try:
            return orig_cap_chunk(self, *a, **kw)
        finally:
            self.pool = keep

    _graph.TrainStepGraph.run_chunk = run_chunk
    _graph.TrainStepGraph._capture_chunk = capture_chunk
    _graph.TrainStepGraph._replay = replay
    _graph.TrainStepGraph._eager = eager
    if args.no_graph:
        # no graph object: wrap train_batch itself
        tb = trial.train_batch

        def _tb(batch, epoch_idx, batch_idx):
            if state["violation"] is None:
                pre["snap"] = snapshot()
                pre["batch"] = [x.detach().clone() for x in batch if isinstance(x, torch.Tensor)]
            out = tb(batch=batch, epoch_idx=epoch_idx, batch_idx=batch_idx)
            state["batch"] += 1
            if state["violation"] is None:
                v = check("nograph", out, None, pre["batch"])
                if v:
                    state["violation"] = {"batch": state["batch"], "what": v, "tag": "nograph"}
            return out

        trial.train_batch = lambda batch, epoch_idx, batch_idx: _tb(batch, epoch_idx, batch_idx)
    ctrl.run()
    res = {"variant": args.variant, "amp": args.amp, "seed": args.seed, "lr": args.lr,
           "graph_batches": args.graph_batches, "no_graph": args.no_graph, "batches_seen": state["batch"],
           "graph": ctrl._graph.stats() if getattr(ctrl, "_graph", None) is not None else None,
           "violation": state["violation"], "wall_s": round(time.time() - state["t0"], 1),
           "step_losses": [round(x, 4) for x in step_losses],
           "chunks_checked": state.get("chunks"), "final_masters_finite": all(bool(torch.isfinite(a.master).all()) for f in fused() for a in f.arenas)}
    tag = (f"{args.variant}_{args.amp}_g{0 if args.no_graph else args.graph_batches}_s{args.seed}"
           f"_c{args.check_every}{'_r4' if args.r4_model else ''}_{args.loss}{'_sep' if args.separate_pools else ''}"
           f"{'_native' if args.native else ''}")
    with open(os.path.join(args.out, f"{tag}.log.jsonl"), "w") as fh:
        for r in state["log"]:
            fh.write(json.dumps(r) + "\n")
    if state["violation"] is not None and pre["snap"] is not None and args.check_every == 1:
        torch.save({"snap": pre["snap"], "batch": pre["batch"]}, os.path.join(args.out, f"{tag}_pre.pt"))
        res["eager_replays"] = eager_replays(pre, args, trial)
    print(json.dumps(res, default=str), flush=True)


def eager_replays(pre, args, trial):
    """Re-run the violating batch eagerly from the dumped pre-replay state with fresh masks, in the
    trial's precision and in fp32: does any legitimate step go non-finite?"""
    import copy
    import torch
    import torch.nn as nn
    from determined_1_amd.models import CIFAR10CNN
    from determined_1_amd.ops.functional import u8_normalize
    import model_def

    snap = pre["snap"]
    x_u8, y = pre["batch"][0], pre["batch"][-1]
    out = {}
    for dt in (torch.bfloat16, torch.float32):
        net = CIFAR10CNN(0.25, 0.25, 0.5).cuda().to(memory_format=torch.channels_last)
        byname = dict(net.named_parameters())
        for a in snap:
            for n, off, k in zip(a["names"], a["offsets"], a["numels"]):
                key = n.split("module.", 1)[-1]
                if key in byname:
                    p = byname[key]
                    with torch.no_grad():
                        p.copy_(a["master"][off:off + k].view_as(p))
        net = net.to(dt)
        net.train()
        worst = {"finite_all": True, "max_loss": 0.0, "max_grad": 0.0}
        for t in range(args.eager_trials):
            net.zero_grad(set_to_none=True)
            xx = u8_normalize(x_u8.contiguous(), model_def.MEAN, model_def.STD, out_dtype=dt)
            o = net(xx)
            loss = nn.functional.cross_entropy(o.float(), y)
            loss.backward()
            gmax = max(float(p.grad.float().abs().max()) for p in net.parameters())
            fin = bool(torch.isfinite(loss)) and math.isfinite(gmax)
            worst["finite_all"] &= fin
            worst["max_loss"] = max(worst["max_loss"], float(loss))
            worst["max_grad"] = max(worst["max_grad"], gmax)
        out[str(dt)] = worst
    return out


if __name__ == "__main__":
    main()
