"""hipGraph replay of the O2 CIFAR-10 trial with its dropout layers.

Round 4 kept half-precision models with dropout eager after every replayed O2 CIFAR run went NaN.
Round 5 found the cause: half-precision convolutions on MIOpen mis-replay from a captured graph once
other MIOpen work runs between replays (pure-PyTorch reproduction: scripts/dbg/miopen_graph_repro.py;
pytorch/_graph.py LIBRARY_CONV_OPS note) -- dropout was incidental.  The trial now runs on the
native CNN kernels (no MIOpen), its graphs stay on, and the graph controller detects library
half-precision convolutions in its first warm-up step and keeps such a train_batch eager.
Round 6 pinned the mechanism underneath: the HIP runtime's captured small memsets (which MIOpen's
weight-gradient solvers issue) replay a stale pattern; with the graphs' memset nodes rewritten into
fill kernels (ops/csrc/det_graph.hip) MIOpen steps replay exactly and the probe is only armed when
that rewrite is off (profiles/r6_graph_memset_root_cause.txt).
"""
import os

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

EX = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "computer_vision",
                  "cifar10_pytorch")


def _run_cifar(amp, hip_graph, batches, seed=3, lr=1e-4):
    from determined_1_amd import workload
    from determined_1_amd.experimental import load_model_def, make_controller

    model_def = load_model_def(EX)  # a uniquely named module: other examples have a model_def too

    cfg = {"hyperparameters": {"global_batch_size": 32, "learning_rate": lr, "train_records": 50000, "amp": amp,
                               "learning_rate_decay": 1e-6, "layer1_dropout": 0.25, "layer2_dropout": 0.25,
                               "layer3_dropout": 0.5},
           "searcher": {"name": "single", "metric": "validation_error", "max_length": {"batches": batches}},
           "records_per_epoch": 50000, "scheduling_unit": 250,
           "optimizations": {"hip_graph": hip_graph, "hip_graph_batches": 20}}
    res = []

    def stream():
        done, step = 0, 1
        while done < batches:
            n = min(250, batches - done)
            yield workload.train_workload(step, num_batches=n, total_batches_processed=done), [], res.append
            done += n
            step += 1
        yield workload.terminate_workload(step, total_batches_processed=done), [], workload.ignore_response

    ctrl = make_controller(model_def.CIFARTrial, cfg, stream(), use_gpu=True, trial_seed=seed)
    ctrl.run()
    losses = [r["metrics"]["avg_metrics"]["loss"] for r in res]
    masters = [a.master for st in ctrl.context._opt_states if st.fused is not None for a in st.fused.arenas]
    finite = all(bool(torch.isfinite(m).all()) for m in masters)
    return losses, finite, ctrl._graph.stats() if ctrl._graph is not None else None


def test_o2_cifar_with_dropout_replays_2000_batches_in_20_batch_chunks_tracking_eager(gpu):
    """2000 batches (8 steps of 250, crossing no epoch) of the O2 trial with its three dropout layers,
    replayed in 20-batch chunk graphs: every step's loss finite and within a band of the eager run
    (different dropout draws, so not batch-exact): |graph - eager| <= 0.1 + 0.35 * eager per 250-batch
    step, and both learn (final step loss < 40 % of the first)."""
    lg, fin_g, st = _run_cifar("O2", True, 2000)
    le, fin_e, _ = _run_cifar("O2", False, 2000)
    assert st is not None and st["disabled"] is None and st["chunk_disabled"] is None and st["chunk_replays"] >= 80, st
    assert fin_g and fin_e
    assert len(lg) == len(le) == 8
    assert all(l == l and abs(l) < 1e3 for l in lg + le), (lg, le)
    for g, e in zip(lg, le):
        assert abs(g - e) <= 0.1 + 0.35 * e, (lg, le)
    assert lg[-1] < 0.4 * lg[0] and le[-1] < 0.4 * le[0], (lg, le)


class _HalfConvTrialNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 8, 3, padding=1)
        self.fc = nn.Linear(8, 10)

    def forward(self, x):
        return self.fc(torch.relu(self.conv(x)).mean((2, 3)))


def test_half_precision_library_convs_keep_train_batch_eager(gpu, monkeypatch):
    """With the captured-memset rewrite off, a train_batch whose bf16 convolutions go to MIOpen is
    detected in the first warm-up step and runs eagerly (finite, learning); the same model in fp32
    captures and replays.  With the rewrite on (default) nothing is flagged."""
    from determined_1_amd.pytorch import _graph
    from determined_1_amd.pytorch._graph import library_conv_reason

    net = _HalfConvTrialNet().to(gpu).to(torch.bfloat16)
    x = torch.randn(4, 3, 16, 16, device=gpu, dtype=torch.bfloat16)
    out, reason = library_conv_reason(lambda: net(x).float().square().mean())
    assert reason is None and torch.isfinite(out), reason
    monkeypatch.setattr(_graph, "FIX_MEMSETS", False)

    torch.manual_seed(0)
    for dtype, expect_hit in ((torch.bfloat16, True), (torch.float32, False)):
        net = _HalfConvTrialNet().to(gpu).to(dtype)
        x = torch.randn(4, 3, 16, 16, device=gpu, dtype=dtype)

        def step():
            loss = net(x).float().square().mean()
            loss.backward()
            return loss.detach()

        out, reason = library_conv_reason(step)
        assert torch.isfinite(out)
        assert (reason is not None) == expect_hit, reason
        if expect_hit:
            assert "MIOpen" in reason and "bfloat16" in reason and "not replay-safe" in reason
