"""GPU discovery in the trial process (reference ``harness/determined/gpu.py`` parses
``nvidia-smi``).  MI355X: read the KFD topology (no HIP context is created, so this is safe before
the training processes fork) and optionally ``amd-smi`` for utilisation."""
import json
import os
import shutil
import subprocess
from typing import Any, Dict, List, Optional

KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


class GPU:
    def __init__(self, index: int, uuid: str, name: str, node: int) -> None:
        self.index = index
        self.uuid = uuid
        self.name = name
        self.node = node

    def __repr__(self) -> str:
        return f"GPU({self.index}, {self.uuid}, {self.name})"


def get_gpus(root: str = KFD_NODES) -> List[GPU]:
    """GPU nodes (simd_count > 0) in KFD order, which is the HIP device order."""
    if not os.path.isdir(root):
        return []
    out = []
    for n in sorted((int(x) for x in os.listdir(root) if x.isdigit())):
        props = {}
        try:
            for line in open(os.path.join(root, str(n), "properties")):
                k, _, v = line.partition(" ")
                props[k] = v.strip()
        except OSError:
            continue
        if int(props.get("simd_count", "0")) <= 0:
            continue
        try:
            name = open(os.path.join(root, str(n), "name")).read().strip()
        except OSError:
            name = "AMD Instinct"
        uid = int(props.get("unique_id", "0"))
        out.append(GPU(len(out), f"GPU-{uid:016x}", name, n))
    return out


def get_gpu_uuids_and_validate(use_gpu: bool, slot_ids: Optional[List[int]] = None) -> List[str]:
    """UUIDs of the GPUs this trial may use; checks the slot count against the visible devices
    (reference ``gpu.py:67``)."""
    if not use_gpu:
        return []
    gpus = get_gpus()
    visible = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if visible:
        idx = [int(x) for x in visible.split(",") if x.strip()]
        gpus = [g for g in gpus if g.index in idx]
    if slot_ids is not None and len(gpus) < len(slot_ids):
        raise RuntimeError(f"trial was assigned {len(slot_ids)} slots but only {len(gpus)} GPUs are visible")
    return [g.uuid for g in gpus]


def utilization() -> List[Dict[str, Any]]:
    """Per-GPU busy % and VRAM use from sysfs (``amdgpu`` driver), for the harness profiler."""
    out = []
    base = "/sys/class/drm"
    if not os.path.isdir(base):
        return out
    for card in sorted(os.listdir(base)):
        dev = os.path.join(base, card, "device")
        busy = os.path.join(dev, "gpu_busy_percent")
        if not card.startswith("card") or "-" in card or not os.path.exists(busy):
            continue
        rec = {"card": card}
        for key, fname in (("gpu_busy_percent", "gpu_busy_percent"), ("vram_used", "mem_info_vram_used"),
                           ("vram_total", "mem_info_vram_total")):
            try:
                rec[key] = int(open(os.path.join(dev, fname)).read().strip())
            except (OSError, ValueError):
                pass
        out.append(rec)
    return out


def amd_smi_json() -> Optional[Any]:
    exe = shutil.which("amd-smi")
    if not exe:
        return None
    try:
        return json.loads(subprocess.run([exe, "metric", "--json"], capture_output=True, text=True, timeout=10).stdout)
    except (subprocess.SubprocessError, ValueError):
        return None
