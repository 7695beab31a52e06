"""Attribute the ResNet-50 step's leftover non-GEMM library launches (copies, adds, fills) to the
Python frames that issue them: runs ``bench.py`` in-process under ``torch.profiler`` with stacks
and prints, for each aten op that launches such a kernel, its device time and top user frames.

    python scripts/probe_small_launches.py --steps 3 --warmup 3
"""
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import bench  # noqa: E402

OPS = ("aten::copy_", "aten::add", "aten::add_", "aten::fill_", "aten::zero_", "aten::convolution_backward",
       "aten::mean", "aten::sum", "aten::clone", "aten::contiguous")

if __name__ == "__main__":
    sys.argv = ["bench.py"] + sys.argv[1:]
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
        bench.main()
    for e in prof.key_averages(group_by_input_shape=True):
        if e.key in OPS and e.device_time_total > 0:
            print(f"{e.key:32s} calls={e.count:5d} dev_ms={e.device_time_total / 1e3:8.3f} shapes={e.input_shapes}",
                  flush=True)
    avg = prof.key_averages(group_by_stack_n=12)
    rows = []
    for e in avg:
        if e.key in OPS and e.device_time_total > 0:
            rows.append(e)
    rows.sort(key=lambda e: -e.device_time_total)
    for e in rows[:25]:
        frames = [f for f in e.stack if "torch/" not in f][:6] or e.stack[:6]
        print(f"{e.key:32s} calls={e.count:5d} dev_ms={e.device_time_total / 1e3:8.3f}", flush=True)
        for f in frames:
            print("      " + f, flush=True)
