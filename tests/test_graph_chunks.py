"""Multi-batch chunks (optimizations.hip_graph_batches, pytorch/_data.py ChunkedBatches /
ChunkPrefetcher, pytorch/_graph.py run_chunk): a chunked run must see exactly the batches of the
unchunked run, in order, never mixing epochs, through steps that end inside a chunk, a restore
offset and validation -- on the CPU (eager) here, and as multi-batch hipGraph replays on the GPU."""
import pytest
import torch
import torch.nn as nn

from determined_1_amd import pytorch
from determined_1_amd.pytorch._data import ChunkedBatches
from tests.utils import Recorder, run


class StackedRows(torch.utils.data.Dataset):
    """Rows depend only on their index; ``__getitems__`` returns them stacked."""

    def __init__(self, n: int, seed: int = 1) -> None:
        g = torch.Generator().manual_seed(seed)
        self.x = torch.randn(n, 3, 16, 16, generator=g)
        self.y = torch.randint(0, 10, (n,), generator=g)
        self.calls = 0

    def __len__(self) -> int:
        return len(self.y)

    def __getitems__(self, idx):
        self.calls += 1
        i = torch.as_tensor(list(idx))
        return self.x[i], self.y[i]


class StackedTrial(pytorch.PyTorchTrial):
    def __init__(self, context):
        self.context = context
        torch.manual_seed(0)
        net = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.ReLU(), nn.AdaptiveAvgPool2d(1), nn.Flatten(),
                            nn.Linear(8, 10))
        self.model = context.wrap_model(net)
        self.opt = context.wrap_optimizer(torch.optim.RMSprop(self.model.parameters(), lr=1e-3))
        self.seen = []

    def build_training_data_loader(self):
        self.train_ds = StackedRows(int(self.context.get_hparam("train_rows")))
        return pytorch.DataLoader(self.train_ds, batch_size=self.context.get_per_slot_batch_size(),
                                  collate_fn=pytorch.passthrough_collate)

    def build_validation_data_loader(self):
        return pytorch.DataLoader(StackedRows(72, seed=2), batch_size=self.context.get_per_slot_batch_size(),
                                  collate_fn=pytorch.passthrough_collate)

    def train_batch(self, batch, epoch_idx, batch_idx):
        x, y = batch
        if not x.is_cuda:  # (a host read would break a hipGraph capture)
            self.seen.append((epoch_idx, batch_idx, float(x[0, 0, 0, 0])))
        loss = nn.functional.cross_entropy(self.model(x).float(), y)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss}

    def evaluate_batch(self, batch):
        x, y = batch
        return {"validation_loss": nn.functional.cross_entropy(self.model(x).float(), y)}


class StackedTrialNoBatchIdx(StackedTrial):
    """The same step without reading batch_idx: the hipGraph builder refuses a train_batch that
    reads it (a replay would reuse the captured value); epoch_idx keys the graphs per epoch."""

    def train_batch(self, batch, epoch_idx, batch_idx):
        x, y = batch
        loss = nn.functional.cross_entropy(self.model(x).float(), y) * (1.0 + 0.0 * epoch_idx)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss}


def test_chunked_batches_respect_epochs_and_offsets():
    dl = pytorch.DataLoader(StackedRows(100), batch_size=10, collate_fn=pytorch.passthrough_collate)
    loader = dl.get_data_loader(repeat=True, skip=3)
    ds = loader.dataset
    it = ChunkedBatches(loader, 4, epoch_len=len(loader), start=3)
    sizes = [len(next(it)) for _ in range(5)]
    assert sizes == [4, 3, 4, 4, 2]  # batches 3-6, 7-9 | 10-13, 14-17, 18-19
    assert ds.calls == 5
    ref = iter(dl.get_data_loader(repeat=True, skip=3))
    it = ChunkedBatches(dl.get_data_loader(repeat=True, skip=3), 4, epoch_len=10, start=3)
    for _ in range(4):
        for b in next(it).batches:
            x, y = next(ref)
            assert torch.equal(b[0], x) and torch.equal(b[1], y)


def _run(monkeypatch, k, use_gpu=False, graph=False, rows=160, trial=StackedTrial):
    monkeypatch.setenv("DET_GRAPH_BATCHES", str(k))
    monkeypatch.setenv("DET_HIP_GRAPH", "1" if graph else "0")
    rec = Recorder().train(1, 13, 0).validate(1, 13).train(2, 9, 13).train(3, 11, 22).validate(3, 33)
    ctrl, resp = run(trial, {"global_batch_size": 16, "train_rows": rows}, rec, use_gpu=use_gpu,
                     records_per_epoch=rows)
    if use_gpu:
        torch.cuda.synchronize()
    params = torch.cat([p.detach().float().reshape(-1) for p in ctrl.context.models[0].parameters()]).cpu()
    losses = [float(b["loss"]) for r in resp if "batch_metrics" in r.get("metrics", {})
              for b in r["metrics"]["batch_metrics"]]
    vals = [r["metrics"]["validation_metrics"]["validation_loss"] for r in resp
            if "validation_metrics" in r.get("metrics", {})]
    return ctrl, params, losses, vals


def test_chunked_training_matches_unchunked_on_cpu(monkeypatch):
    c1, p1, l1, v1 = _run(monkeypatch, 1)
    c4, p4, l4, v4 = _run(monkeypatch, 4)
    assert c4._chunked and not c1._chunked
    assert len(l1) == len(l4) == 33 and len(v1) == len(v4) == 2
    assert [s[:2] for s in c1.trial.seen] == [s[:2] for s in c4.trial.seen]
    assert [s[2] for s in c1.trial.seen] == [s[2] for s in c4.trial.seen]
    torch.testing.assert_close(p4, p1, rtol=0, atol=0)
    assert l1 == l4
    assert v1 == pytest.approx(v4, rel=1e-6)
    # one dataset call per chunk (chunks of <= 4 batches, split at epoch ends 10/20/30)
    assert c4.trial.train_ds.calls <= 12


@pytest.mark.gpu
def test_multibatch_graph_replay_matches_eager(gpu, monkeypatch):
    # 30-batch epochs: train_batch reads epoch_idx (graphs are keyed per epoch) and only full
    # 4-batch chunks are captured, after one per-batch warm-up of their key, so an epoch needs
    # several full chunks to replay any (10-batch epochs have one full chunk after the first)
    _, p_e, l_e, v_e = _run(monkeypatch, 1, use_gpu=True, graph=False, rows=480, trial=StackedTrialNoBatchIdx)
    c, p_g, l_g, v_g = _run(monkeypatch, 4, use_gpu=True, graph=True, rows=480, trial=StackedTrialNoBatchIdx)
    assert c._graph is not None and c._graph.chunk_replays > 0, c._graph.stats() if c._graph else None
    assert c._eval_graph is not None and c._eval_graph.replays > 0
    assert len(l_g) == len(l_e)
    torch.testing.assert_close(torch.tensor(l_g), torch.tensor(l_e), rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(p_g, p_e, rtol=2e-3, atol=2e-3)
    assert v_g == pytest.approx(v_e, rel=2e-3)


def test_half_precision_dropout_model_is_graph_eligible():
    """The round-4 guard (half-precision model + torch dropout -> eager) is gone: its NaN was MIOpen
    half-precision convolutions mis-replaying (pytorch/_graph.py LIBRARY_CONV_OPS note), which the
    warm-up probe now detects instead.  Dropout itself never made a model ineligible again."""
    from types import SimpleNamespace

    from determined_1_amd.pytorch._graph import TrainStepGraph

    def ctx(model):
        return SimpleNamespace(device=torch.device("cuda"), dist_config=SimpleNamespace(use=False, aggregation_frequency=1),
                               _amp=None, _timers=SimpleNamespace(enabled=False), _opt_states=[], models=[model])

    drop = nn.Sequential(nn.Linear(4, 4), nn.Dropout(0.5)).to(torch.bfloat16)
    assert TrainStepGraph.ineligible_reason(ctx(drop)) == "no wrapped optimizer"


def test_library_conv_probe_passes_results_through_and_ignores_host_convs():
    """The probe runs the warm-up step unchanged (same result) and only flags convolutions that would
    go to MIOpen: CUDA inputs in bf16/fp16 (host convolutions, fp32 and Linear layers never)."""
    from determined_1_amd.pytorch._graph import LIBRARY_CONV_OPS, library_conv_reason

    conv = nn.Conv2d(3, 4, 3).to(torch.bfloat16)
    x = torch.randn(2, 3, 8, 8, dtype=torch.bfloat16, requires_grad=True)

    def step():
        y = conv(x).float().sum()
        y.backward()
        return y.detach()

    ref = step()
    out, reason = library_conv_reason(step)
    assert reason is None and torch.equal(out, ref)
    assert "aten::convolution" in LIBRARY_CONV_OPS and "aten::convolution_backward" in LIBRARY_CONV_OPS
