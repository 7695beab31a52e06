"""shared_fs checkpoint storage (reference ``storage/shared.py:9-60``).

Inside a reference container the host path is mounted at ``/determined_shared_fs``; trial
processes here run directly on the agent host, so the host path is used unless the container
mount point exists.
"""
import os
import pathlib
from typing import Any, Dict, Optional

from determined_1_amd import constants
from determined_1_amd.storage.base import StorageManager


def full_storage_path(host_path: str, storage_path: Optional[str] = None, container_path: Optional[str] = None) -> str:
    if storage_path is not None and os.path.isabs(storage_path):
        if not os.path.normpath(storage_path).startswith(os.path.normpath(host_path)):
            raise ValueError(f"storage_path {storage_path} must be under host_path {host_path}")
        rel = os.path.relpath(storage_path, host_path)
    else:
        rel = storage_path or ""
    base = container_path if container_path else host_path
    return os.path.normpath(os.path.join(base, rel)) if rel else os.path.normpath(base)


class SharedFSStorageManager(StorageManager):
    @classmethod
    def from_config(cls, cfg: Dict[str, Any], container_path: Optional[str] = None) -> "SharedFSStorageManager":
        host_path = cfg.get("host_path", "/tmp")
        if container_path is None and os.path.isdir(constants.SHARED_FS_CONTAINER_PATH):
            container_path = constants.SHARED_FS_CONTAINER_PATH
        return cls(full_storage_path(host_path, cfg.get("storage_path"), container_path))

    def __init__(self, base_path: str) -> None:
        super().__init__(base_path)
        pathlib.Path(base_path).mkdir(parents=True, exist_ok=True)
