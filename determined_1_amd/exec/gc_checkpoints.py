"""Checkpoint GC job (reference ``exec/gc_checkpoints.py:15-91``): delete the checkpoints the
master selected with the experiment's retention policy.

    python -m determined_1_amd.exec.gc_checkpoints SPEC.json
SPEC: {"experiment_config": {...}, "checkpoints": [{"uuid": ..., "resources": {...}}, ...]}
"""
import json
import logging
import sys

from determined_1_amd import storage


def delete_checkpoints(checkpoint_storage: dict, checkpoints: list) -> int:
    mgr = storage.build(checkpoint_storage)
    n = 0
    for c in checkpoints:
        md = storage.StorageMetadata.from_json(c.get("checkpoint") or c)
        logging.info("deleting checkpoint %s", md.storage_id)
        mgr.delete(md)
        n += 1
    return n


def main(argv: list) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s [gc] %(message)s")
    with open(argv[1]) as f:
        spec = json.load(f)
    n = delete_checkpoints(spec["experiment_config"].get("checkpoint_storage", {}), spec["checkpoints"])
    logging.info("deleted %d checkpoints", n)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
