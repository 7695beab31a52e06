"""TensorBoard integration (reference ``harness/determined/tensorboard/``).

``tensorboard`` / TF are not installed, so the event files are written natively:
``EventFileWriter`` emits TFRecord-framed ``Event`` protos (hand-encoded protobuf, masked CRC32C)
that stock TensorBoard reads.  ``MetricWriter`` logs ``Determined/<metric>`` per training batch
and ``val_<metric>`` per validation (reference ``metric_writers/callback.py:20-55``);
``TensorboardManager`` syncs new/changed ``*tfevents*`` files from the local log dir to
``<storage>/tensorboard/experiment/<e>/trial/<t>`` (``tensorboard/base.py:6-55``).
"""
from determined_1_amd.tensorboard.events import EventFileWriter, crc32c, masked_crc32c, read_events, read_scalars
from determined_1_amd.tensorboard.manager import MetricWriter, TensorboardManager, build, get_base_path

__all__ = ["EventFileWriter", "MetricWriter", "TensorboardManager", "build", "crc32c", "get_base_path",
           "masked_crc32c", "read_events", "read_scalars"]
