"""Model-definition packaging (reference ``common/determined_common/context.py:14-120``):
walk the directory, honour ``.detignore`` (gitignore syntax via ``pathspec``), enforce the
context size limit, return ``[{path, type, content(base64), mode, mtime}]``."""
import base64
import os
import pathlib
from typing import Any, Dict, List, Optional

from determined_1_amd import constants


def read_detignore(root: pathlib.Path) -> Optional[Any]:
    p = root.joinpath(".detignore")
    if not p.exists():
        return None
    import pathspec

    return pathspec.PathSpec.from_lines("gitwildmatch", p.read_text().splitlines())


def read_context(root: pathlib.Path, limit: int = constants.MAX_CONTEXT_SIZE) -> List[Dict[str, Any]]:
    root = pathlib.Path(root).resolve()
    if not root.is_dir():
        raise ValueError(f"model definition must be a directory: {root}")
    spec = read_detignore(root)
    items = []  # type: List[Dict[str, Any]]
    total = 0
    for dirpath, dirnames, filenames in os.walk(root):
        rel_dir = os.path.relpath(dirpath, root)
        dirnames[:] = sorted(d for d in dirnames if d not in ("__pycache__", ".git"))
        for d in dirnames:
            rel = os.path.normpath(os.path.join(rel_dir, d))
            if spec is not None and spec.match_file(rel + "/"):
                continue
            items.append({"path": rel + "/", "type": "dir", "content": "", "mode": 0o755})
        for f in sorted(filenames):
            rel = os.path.normpath(os.path.join(rel_dir, f))
            if spec is not None and spec.match_file(rel):
                continue
            if f.endswith(".pyc"):
                continue
            full = os.path.join(dirpath, f)
            data = pathlib.Path(full).read_bytes()
            total += len(data)
            if total > limit:
                raise ValueError(f"model definition exceeds the {limit // (1024 * 1024)} MiB limit; "
                                 "use a .detignore file to exclude large files")
            items.append({"path": rel, "type": "file", "content": base64.b64encode(data).decode(),
                          "mode": os.stat(full).st_mode & 0o777, "mtime": int(os.path.getmtime(full))})
    return items
