"""Measured vendor-BLAS solutions for the GEMMs that stay on hipBLASLt / rocBLAS (MI355X, gfx950).

The dense layers of the transformer models (ops/transformer.py: BERT, ALBERT) multiply through
``torch.addmm`` / ``torch.mm``, which take the solution the library heuristic picks for a shape.
PyTorch's TunableOp can time every hipBLASLt and rocBLAS solution of a shape and keep the fastest;
the winners for the shapes the framework's models run are measured once on an MI355X
(``scripts/tune_gemms.py``) and shipped in ``tuned/gemm_gfx950.csv``.  A GPU trial loads that file
read-only at start-up: nothing is tuned at run time (a timing sweep inside a train step would stall
it and cannot run under hipGraph capture), and shapes the file does not list keep the heuristic.
The file's validator lines pin the torch / HIP / hipBLASLt / rocBLAS versions and the GPU arch it
was measured with; TunableOp ignores it on any other stack.

Opt-in (``DET_TUNED_GEMMS=1``, or ``=<path>`` for another file).  Measured on BERT-base SQuAD bs12
O2 in one session (profiles/r5_bert_sink_link_tuning_ab.jsonl, r5s24): with hipGraph replays the
tuned and heuristic solutions give the same 1,484 ex/s -- at these shapes the heuristic already
picks solutions as fast as the best measured ones -- while eager steps lose 10-14 % (1,199-1,220 vs
1,374) to TunableOp's per-call lookup on the host.  So the file is not loaded by default; it stays
for shapes where a sweep does find faster solutions (``scripts/tune_gemms.py``).
"""
import logging
import os
from typing import Dict, Optional

import torch

SHIPPED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "gemm_gfx950.csv")
_STATE = {"loaded": None}  # type: Dict[str, Optional[bool]]


def enable(path: Optional[str] = None) -> bool:
    """Load the measured solutions (once per process).  True when TunableOp now serves them."""
    if _STATE["loaded"] is not None:
        return bool(_STATE["loaded"])
    env = os.environ.get("DET_TUNED_GEMMS", "0")
    if env in ("", "0") or not torch.cuda.is_available():
        _STATE["loaded"] = False
        return False
    src = path or (env if env not in ("", "1") else SHIPPED)
    arch = torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName
    if not os.path.exists(src) or not arch.startswith("gfx950"):
        _STATE["loaded"] = False
        return False
    from torch.cuda import tunable

    # TunableOp fills its table lazily from its file name at the first tunable GEMM, so the file is
    # named rather than read here (a read_file before that first call is replaced by the lazy read);
    # with tuning off nothing is written back to it at exit
    tunable.set_filename(src, insert_device_ordinal=False)
    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.record_untuned_enable(False)
    ok = bool(tunable.read_file(src))
    if not ok:
        logging.warning("tuned GEMM file %s was not accepted (other torch/ROCm stack?): library heuristics", src)
        tunable.enable(False)
    _STATE["loaded"] = ok
    return ok


def entries(path: str = SHIPPED) -> Dict[str, str]:
    """``{op,shape: solution}`` of a TunableOp results file (validator lines skipped)."""
    out = {}
    with open(path) as f:
        for line in f:
            parts = line.strip().split(",")
            if len(parts) >= 3 and parts[0] != "Validator":
                out[parts[0] + "," + parts[1]] = parts[2]
    return out
