"""Which Python call sites issue the non-math launches of the ResNet-50 step (direct_copy /
fill / memset / cast kernels in profiles/r3_resnet50_steady_*.csv): torch.profiler over two
training batches of the bench trial, aggregated by op and stack."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from determined_1_amd import workload  # noqa: E402
from determined_1_amd.experimental import load_model_def, make_controller  # noqa: E402

BS = int(os.environ.get("BS", "256"))
Trial = load_model_def(os.path.join(REPO, "examples", "computer_vision", "resnet50_pytorch")).ResNetImageNetTrial
cfg = {"entrypoint": "model_def:ResNetImageNetTrial",
       "hyperparameters": {"global_batch_size": BS, "lr": 0.1, "momentum": 0.9, "weight_decay": 5e-5, "arch": "resnet50",
                           "amp": "O2", "channels_last": True, "fused_bn": True, "native_conv1x1": True,
                           "bn_prologue": False, "native_stem": True, "native_conv3x3": True, "image_size": 224},
       "searcher": {"name": "single", "metric": "validation_loss", "max_length": {"batches": 8}},
       "scheduling_unit": 8}
prof_box = {}


def stream():
    for i in range(4):
        yield workload.train_workload(1, num_batches=1, total_batches_processed=i), [], workload.ignore_response
    torch.cuda.synchronize()
    p = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True)
    p.__enter__()
    prof_box["p"] = p
    yield workload.train_workload(2, num_batches=2, total_batches_processed=4), [], workload.ignore_response
    torch.cuda.synchronize()
    p.__exit__(None, None, None)
    yield workload.terminate_workload(3), [], workload.ignore_response


torch.cuda.set_device(0)
ctrl = make_controller(Trial, cfg, stream(), trial_seed=1)
ctrl.run()
p = prof_box["p"]
want = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::zeros", "aten::_to_copy", "aten::clone", "aten::contiguous",
        "aten::add_", "aten::add", "aten::convolution_backward", "aten::sum")
for ev in p.key_averages(group_by_stack_n=8):
    if ev.key in want:
        stack = [s for s in ev.stack if "determined_1_amd" in s or "model_def" in s][:5]
        print(f"{ev.key:28s} calls={ev.count:4d} dev_us={ev.device_time_total:9.0f} shapes={ev.input_shapes if hasattr(ev, 'input_shapes') else ''}")
        for s in stack:
            print("      ", s)
print("---- kernels ----")
for ev in p.key_averages():
    if ev.device_time_total > 0 and any(k in ev.key for k in ("SubTensor", "copy", "Fill", "fill", "Cast", "elementwise")):
        print(f"{ev.key[:110]:110s} calls={ev.count:4d} dev_us={ev.device_time_total:9.0f}")
