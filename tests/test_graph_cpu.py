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
