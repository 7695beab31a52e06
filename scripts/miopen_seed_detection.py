"""Seed the shipped MIOpen find-db + kernel cache (determined_1_amd/ops/miopen_db/) with every conv
problem the detection examples hit after shape bucketing, so a fresh box runs them without MIOpen
find / kernel builds in the training loop (measured: Faster R-CNN 0.65 images/s with a find on every
new batch shape vs 77.7 at one fixed shape, profiles/r2_fasterrcnn_shape_diagnosis.jsonl).

  DETR (pad_multiple 128, images 480-640 px): padded batches (H, W) in {512, 640}^2.
  Faster R-CNN (800 px short side, <= 1333 long, size_divisible 128, PennFudan-sized 300-500 px
  originals): one side of every resized image is 800 (-> 896) and the other 800..1333, so a batch
  of two pads to (H, W) in {896, 1024, 1152, 1280, 1408}^2 (a portrait and a landscape image).

Each padded shape is one training batch (forward + backward) of the real trial, at O0 (fp32, the
reference precision) and O2 (bf16).

    python scripts/miopen_seed_detection.py [--models detr,fasterrcnn] [--amps O0,O2] [--harvest DIR]
"""
import argparse
import importlib.util
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

_spec = importlib.util.spec_from_file_location("_det_miopen_db", os.path.join(REPO, "determined_1_amd", "ops", "miopen_db.py"))
miopen_db = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(miopen_db)  # type: ignore
miopen_db.configure(os.environ)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from determined_1_amd import pytorch, workload  # noqa: E402
from determined_1_amd.experimental import load_model_def, make_controller  # noqa: E402

# resized long side -> size_divisible-128 bucket: 850 -> 896, 1000 -> 1024, 1100 -> 1152, 1250 -> 1280, 1333 -> 1408;
# an original short side of 300 px scales by 8/3, so these are the original long sides
FRCNN_LONG = [None, 375, 412, 469, 500]  # None: a 300x300 original (800 x 800 -> 896)


class Resized(torch.utils.data.Dataset):
    """Items of ``base`` resized to prescribed (h, w) (absolute xyxy boxes scaled along)."""

    def __init__(self, base, sizes, absolute_boxes: bool) -> None:
        self.base, self.sizes, self.absolute = base, sizes, absolute_boxes

    def __len__(self) -> int:
        return len(self.sizes)

    def __getitem__(self, i):
        img, t = self.base[i]
        h, w = self.sizes[i]
        sy, sx = h / img.shape[1], w / img.shape[2]
        img = F.interpolate(img[None], size=(h, w), mode="bilinear", align_corners=False)[0]
        t = dict(t)
        if self.absolute:
            t["boxes"] = t["boxes"] * torch.tensor([sx, sy, sx, sy])
            if "masks" in t:
                t["masks"] = F.interpolate(t["masks"][None].float(), size=(h, w), mode="nearest")[0].to(torch.uint8)
            t["area"] = (t["boxes"][:, 3] - t["boxes"][:, 1]) * (t["boxes"][:, 2] - t["boxes"][:, 0])
        else:
            t["orig_size"] = t["size"] = torch.tensor([h, w])
        return img, t


def frcnn_sizes():
    out = []
    for lh in FRCNN_LONG:
        for lw in FRCNN_LONG:
            out.append((300, 300) if lh is None else (lh, 300))  # portrait: padded H bucket
            out.append((300, 300) if lw is None else (300, lw))  # landscape: padded W bucket
    return out


# Mask R-CNN: COCO-shaped 480-640 px originals -> 800 px short side, long side 800..1067 -> buckets
# 896 / 1024 / 1152; an original short side of 480 scales by 5/3
MRCNN_LONG = [None, 600, 640]


def mrcnn_sizes():
    out = []
    for lh in MRCNN_LONG:
        for lw in MRCNN_LONG:
            out.append((480, 480) if lh is None else (lh, 480))
            out.append((480, 480) if lw is None else (480, lw))
    return out


def detr_sizes():
    out = []
    for h in (500, 600):
        for w in (500, 600):
            out += [(h, w), (h, w)]
    return out


def _example_module(ex: str, name: str):
    """``<ex>/<name>.py`` loaded by path (several examples ship a ``data.py``)."""
    spec = importlib.util.spec_from_file_location(f"_seed_{os.path.basename(ex)}_{name}", os.path.join(ex, name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # type: ignore
    return mod


def run(model: str, amp: str) -> None:
    if model == "detr":
        ex = os.path.join(REPO, "examples", "computer_vision", "detr_coco_pytorch")
        base_cls = load_model_def(ex).DETRTrial
        sizes = detr_sizes()

        class Seed(base_cls):  # type: ignore
            def build_training_data_loader(self):
                return pytorch.DataLoader(Resized(self._dataset(True), sizes, False), batch_size=2,
                                          collate_fn=self._collate, shuffle=False)

        import yaml

        hp = dict(yaml.safe_load(open(os.path.join(ex, "const_fake.yaml")))["hyperparameters"])
        hp.update(global_batch_size=2, num_workers=0, amp=amp, train_records=len(sizes))
    elif model in ("maskrcnn", "retinanet"):
        ex = os.path.join(REPO, "examples", "computer_vision", f"{model}_coco_pytorch")
        mod = load_model_def(ex)
        base_cls = mod.MaskRCNNTrial if model == "maskrcnn" else mod.RetinaNetTrial
        sizes = mrcnn_sizes()
        from determined_1_amd.models import detection as mdata  # SyntheticCocoInstances, list_collate

        class Seed(base_cls):  # type: ignore
            def build_training_data_loader(self):
                return pytorch.DataLoader(Resized(mdata.SyntheticCocoInstances(len(sizes), num_classes=self.num_classes),
                                                  sizes, True), batch_size=2, collate_fn=mdata.list_collate)

        import yaml

        hp = dict(yaml.safe_load(open(os.path.join(ex, "const.yaml")))["hyperparameters"])
        hp.update(global_batch_size=2, amp=amp)
    else:
        ex = os.path.join(REPO, "examples", "computer_vision", "fasterrcnn_coco_pytorch")
        base_cls = load_model_def(ex).ObjectDetectionTrial
        sizes = frcnn_sizes()
        fdata = _example_module(ex, "data")

        class Seed(base_cls):  # type: ignore
            def build_training_data_loader(self):
                return pytorch.DataLoader(Resized(fdata.SyntheticPedestrians(len(sizes)), sizes, True), batch_size=2,
                                          collate_fn=fdata.collate_fn)

        import yaml

        hp = dict(yaml.safe_load(open(os.path.join(ex, "const.yaml")))["hyperparameters"])
        hp.update(global_batch_size=2, amp=amp, num_images=64)
    nb = len(sizes) // 2
    cfg = {"hyperparameters": hp, "records_per_epoch": 10 ** 6,
           "searcher": {"name": "single", "metric": "loss", "max_length": {"batches": nb}}}
    stream = iter([(workload.train_workload(1, num_batches=nb), [], workload.ignore_response),
                   (workload.terminate_workload(1, total_batches_processed=nb), [], workload.ignore_response)])
    t0 = time.time()
    make_controller(Seed, cfg, stream, use_gpu=True).run()
    torch.cuda.synchronize()
    print(f"{model} {amp}: {nb} batch shapes seeded in {time.time() - t0:.1f} s", flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="detr,fasterrcnn,maskrcnn,retinanet")
    ap.add_argument("--amps", default="O0,O2")
    ap.add_argument("--harvest", default="", help="copy the db + kernel cache here (e.g. gpurun_out/miopen_db)")
    args = ap.parse_args()
    for m in args.models.split(","):
        for a in args.amps.split(","):
            run(m, a)
    if args.harvest:
        n = miopen_db.harvest(args.harvest, with_cache=True)
        print(f"harvested {n} files into {args.harvest}", flush=True)


if __name__ == "__main__":
    main()
