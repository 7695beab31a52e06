"""Storage manager base class and checkpoint metadata (reference ``storage/base.py:11-147``)."""
import contextlib
import os
import pathlib
import shutil
import tempfile
import uuid
from typing import Any, Dict, Iterator, Optional, Tuple


class StorageMetadata:
    def __init__(self, storage_id: str, resources: Optional[Dict[str, int]] = None,
                 framework: Optional[str] = None, format: Optional[str] = None) -> None:  # noqa: A002
        self.storage_id = storage_id
        self.resources = resources or {}
        self.framework = framework
        self.format = format

    def __json__(self) -> Dict[str, Any]:
        return {"uuid": self.storage_id, "resources": self.resources, "framework": self.framework,
                "format": self.format}

    @staticmethod
    def from_json(record: Dict[str, Any]) -> "StorageMetadata":
        return StorageMetadata(record["uuid"], record.get("resources"), record.get("framework"), record.get("format"))

    def __repr__(self) -> str:
        return f"StorageMetadata(uuid={self.storage_id}, {len(self.resources)} files)"


def list_directory(root: pathlib.Path) -> Dict[str, int]:
    """``{relpath: size}``; directories appear as ``"dir/": 0`` (reference ``_list_directory``)."""
    root = pathlib.Path(root)
    out = {}
    for dirpath, dirnames, filenames in os.walk(root):
        rel = os.path.relpath(dirpath, root)
        for d in dirnames:
            out[os.path.join(rel, d).lstrip("./") + "/" if rel != "." else d + "/"] = 0
        for f in filenames:
            p = os.path.join(dirpath, f)
            key = f if rel == "." else os.path.join(rel, f)
            out[key] = os.path.getsize(p)
    return out


class StorageManager:
    """Checkpoints live in ``<base_path>/<uuid>``; remote managers stage through a temp dir."""

    def __init__(self, base_path: str) -> None:
        self._base_path = str(base_path)

    @property
    def base_path(self) -> str:
        return self._base_path

    def post_store_path(self, storage_id: str, storage_dir: pathlib.Path, metadata: StorageMetadata) -> None:
        """Hook after the checkpoint directory is written (remote stores upload here)."""

    @contextlib.contextmanager
    def store_path(self, storage_id: Optional[str] = None) -> Iterator[Tuple[str, pathlib.Path]]:
        storage_id = storage_id or str(uuid.uuid4())
        path = pathlib.Path(self._base_path).joinpath(storage_id)
        old = os.umask(0)
        try:
            path.mkdir(parents=True, exist_ok=True)
        finally:
            os.umask(old)
        yield storage_id, path
        md = StorageMetadata(storage_id, list_directory(path))
        self.post_store_path(storage_id, path, md)

    @contextlib.contextmanager
    def restore_path(self, metadata: StorageMetadata) -> Iterator[pathlib.Path]:
        yield pathlib.Path(self._base_path).joinpath(metadata.storage_id)

    def delete(self, metadata: StorageMetadata) -> None:
        shutil.rmtree(pathlib.Path(self._base_path).joinpath(metadata.storage_id), ignore_errors=True)


def validate_manager(manager: StorageManager) -> None:
    """Write / read back / delete a probe checkpoint (reference ``exec/harness.py:214-221``)."""
    with manager.store_path() as (storage_id, path):
        path.joinpath("VALIDATE.txt").write_text(storage_id)
    md = StorageMetadata(storage_id, {"VALIDATE.txt": len(storage_id)})
    with manager.restore_path(md) as p:
        got = pathlib.Path(p).joinpath("VALIDATE.txt").read_text()
        if got != storage_id:
            raise RuntimeError(f"checkpoint storage validation failed: wrote {storage_id}, read {got}")
    manager.delete(md)


def staging_dir() -> pathlib.Path:
    return pathlib.Path(tempfile.mkdtemp(prefix="det-ckpt-"))
