"""Does a multi-batch (chunk) graph replay compute the same K training steps as K per-batch replays
and as K eager steps?  (the O2 CIFAR trial went non-finite only with chunked graphs.)

Warms a CIFAR controller up until both the per-batch and the 20-batch graph are captured, then,
from ONE saved state (fp32 masters, bf16 model arena, RMSprop slots, dropout bank counters), runs
the same K batches three ways -- chunk replay, per-batch replays, eager -- and compares losses and
final parameters.  Dropout uses a fixed mask bank indexed by a device counter (``bankmask``) so all
three see the same masks; ``--variant none`` drops dropout, ``torch`` keeps torch's RNG dropout
(then only the statistics can agree).

    python scripts/dbg/chunk_vs_batch.py --amp O2 --rounds 4 --out gpurun_out/cvb
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
EX = os.path.join(REPO, "examples", "computer_vision", "cifar10_pytorch")
sys.path.insert(0, REPO)
sys.path.insert(0, EX)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="bankmask", choices=("bankmask", "none", "torch"))
    ap.add_argument("--amp", default="O2")
    ap.add_argument("--native", action="store_true", help="the native CNN kernels (default: torch layers)")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--out", default="gpurun_out/cvb")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    os.environ["DET_GRAPH_LIBRARY_CONVS"] = "1"
    os.environ["DET_NATIVE_CNN"] = "1" if args.native else "0"
    import torch

    from determined_1_amd import workload
    from determined_1_amd.experimental import make_controller
    from determined_1_amd.pytorch._data import BatchChunk
    import model_def
    from graph_nan_probe import patch_dropout

    cfg = {"hyperparameters": {"global_batch_size": 32, "learning_rate": args.lr, "train_records": 50000,
                               "learning_rate_decay": 1e-6, "layer1_dropout": 0.25, "layer2_dropout": 0.25,
                               "layer3_dropout": 0.5, "amp": args.amp},
           "searcher": {"name": "single", "metric": "validation_error", "max_length": {"batches": 200}},
           "records_per_epoch": 50000, "scheduling_unit": 100,
           "optimizations": {"hip_graph": True, "hip_graph_batches": args.k}}

    def stream():
        yield workload.train_workload(1, num_batches=100, total_batches_processed=0), [], workload.ignore_response
        yield workload.terminate_workload(1, total_batches_processed=100), [], workload.ignore_response

    ctrl = make_controller(model_def.CIFARTrial, cfg, stream(), use_gpu=True, trial_seed=1)
    trial = ctrl.trial
    if args.variant == "none":
        for m in trial.model.modules():
            if isinstance(m, torch.nn.modules.dropout._DropoutNd):
                m.p = 0.0
    elif args.variant == "bankmask":
        patch_dropout(trial.model, "bankmask")
    ctrl.run()
    G = ctrl._graph
    st = G.stats()
    assert G.chunk_graphs, st
    ckey, cg = next(iter(G.chunk_graphs.items()))
    epoch_idx, bidx = 0, 100
    fused = [s.fused for s in ctrl.context._opt_states if s.fused is not None]
    banks = [m for m in trial.model.modules() if getattr(m, "_ctr", None) is not None]

    def state():
        s = []
        for f in fused:
            for gs in f.groups:
                for ai, a in enumerate(gs.arenas):
                    s.append((a, ai, a.master.detach().clone() if a.has_master else None, a.flat_param.detach().clone(),
                              {k: v.detach().clone() for k, v in gs.slots.get(ai, {}).items() if k != "master"}, gs))
        return s, [m._ctr.clone() for m in banks], [(gs.step.clone() if gs.step is not None else None, gs.momentum_ready)
                                                      for f in fused for gs in f.groups]

    def restore(saved):
        s, ctrs, host = saved
        with torch.no_grad():
            for a, ai, master, param, slots, gs in s:
                if master is not None:
                    a.master.copy_(master)
                a.flat_param.copy_(param)
                a.flat_grad.zero_()
                for k, v in slots.items():
                    gs.slots[ai][k].copy_(v)
            for m, c in zip(banks, ctrs):
                m._ctr.copy_(c)
        for (step, ready), gs in zip(host, [gs for f in fused for gs in f.groups]):
            if step is not None:
                gs.step.copy_(step)
            gs.momentum_ready = ready
        torch.cuda.synchronize()

    def params():
        return torch.cat([a.master.detach().float().reshape(-1) if a.has_master else a.flat_param.detach().float()
                          for f in fused for a in f.arenas])

    sizes = (32,) * args.k
    x_like, y_like = cg.static_in[0], cg.static_in[-1]
    src = trial.build_training_data_loader().dataset
    results = []
    t0 = time.time()
    for r in range(args.rounds):
        idx = list(range(r * 32 * args.k, (r + 1) * 32 * args.k))
        xb, yb = src.__getitems__(idx)
        xb = torch.as_tensor(xb).to("cuda")
        yb = torch.as_tensor(yb).to("cuda")
        assert xb.shape == x_like.shape and xb.dtype == x_like.dtype and yb.shape == y_like.shape, (xb.shape, x_like.shape)
        chunk = BatchChunk((xb, yb), sizes)
        saved = state()
        out = {}
        # (1) chunk replay
        stacked = G.run_chunk(chunk, epoch_idx, bidx, capture=True)
        torch.cuda.synchronize()
        assert stacked is not None, "chunk graph did not replay"
        out["chunk"] = (stacked["loss"].float().cpu(), params())
        # (2) per-batch replays
        restore(saved)
        losses = []
        for i, b in enumerate(chunk.batches):
            losses.append(G.run(b, epoch_idx, bidx + i)["loss"].float())
        torch.cuda.synchronize()
        out["batch"] = (torch.stack(losses).cpu(), params())
        # (3) eager
        restore(saved)
        losses = []
        for i, b in enumerate(chunk.batches):
            losses.append(G._eager(b, epoch_idx, bidx + i)["loss"].detach().float())
        torch.cuda.synchronize()
        out["eager"] = (torch.stack(losses).cpu(), params())
        p0 = saved[0]
        base = torch.cat([(m if m is not None else p).float().reshape(-1) for _, _, m, p, _, _ in p0])
        upd = float((out["eager"][1] - base).norm())
        row = {"round": r, "update_norm_eager": upd}
        for a, b in (("chunk", "batch"), ("chunk", "eager"), ("batch", "eager")):
            la, pa = out[a]
            lb, pb = out[b]
            row[f"{a}_vs_{b}"] = {"loss_max_abs": float((la - lb).abs().max()), "param_diff_norm": float((pa - pb).norm()),
                                  "param_diff_rel_update": float((pa - pb).norm()) / max(upd, 1e-30),
                                  "bitwise": bool(torch.equal(pa, pb))}
        row["losses"] = {k: [round(float(v), 4) for v in out[k][0][:6]] for k in out}
        row["finite"] = {k: bool(torch.isfinite(out[k][1]).all()) for k in out}
        # continue from the chunk result so later rounds start from a trained state
        results.append(row)
        print(json.dumps(row), flush=True)
    res = {"variant": args.variant, "amp": args.amp, "native": args.native, "k": args.k, "graph": G.stats(),
           "wall_s": round(time.time() - t0, 1), "rounds": results}
    tag = f"cvb_{args.variant}_{args.amp}{'_native' if args.native else ''}"
    with open(os.path.join(args.out, tag + ".json"), "w") as fh:
        json.dump(res, fh)
    print(json.dumps({k: v for k, v in res.items() if k != "rounds"}), flush=True)


if __name__ == "__main__":
    main()
