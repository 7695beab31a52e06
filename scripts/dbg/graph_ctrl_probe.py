"""Controller-path hipGraph probe: the failing tests/test_graph_gpu.py case with knobs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from tests.test_graph_gpu import ConvTrial  # noqa: E402
from tests.utils import Recorder, run  # noqa: E402

os.environ["DET_HIP_GRAPH"] = "1"
rec = Recorder().train(1, 12, 0)
ctrl, resp = run(ConvTrial, {"opt": "sgd", "global_batch_size": 16}, rec, use_gpu=True, records_per_epoch=160)
torch.cuda.synchronize()
print("ctrl ok", ctrl._graph and ctrl._graph.stats(), flush=True)
