"""optimizations.hip_graph on a host without a GPU: the controller checks eligibility once and
keeps running train_batch eagerly."""
from tests.test_graph_gpu import ConvTrial
from tests.utils import Recorder, run


def test_hip_graph_ineligible_on_cpu(monkeypatch):
    monkeypatch.setenv("DET_HIP_GRAPH", "1")
    rec = Recorder().train(1, 4, 0)
    ctrl, resp = run(ConvTrial, {"opt": "sgd", "global_batch_size": 16}, rec, records_per_epoch=160)
    assert ctrl._graph_checked and ctrl._graph is None
    assert len(resp[0]["metrics"]["batch_metrics"]) == 4


def test_hip_graph_refuses_train_batch_reading_batch_idx(monkeypatch):
    """A replay reuses the captured batch_idx, so a train_batch that reads it runs eagerly
    (the contract was documented but not enforced)."""
    from determined_1_amd.pytorch import _graph

    monkeypatch.setattr(_graph.TrainStepGraph, "ineligible_reason", staticmethod(lambda ctx: None))
    monkeypatch.setattr(_graph.TrainStepGraph, "__init__", lambda self, *a, **k: None)

    def reads(batch, epoch_idx, batch_idx):
        return {"loss": batch * (batch_idx % 2)}

    def ignores(batch, epoch_idx, batch_idx):
        return {"loss": batch}

    g, reason = _graph.build(object(), reads, True)
    assert g is None and "batch_idx" in reason
    g, reason = _graph.build(object(), ignores, True)
    assert g is not None and reason is None
