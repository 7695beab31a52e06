"""Persistent MIOpen find/perf database and kernel cache for the conv layers MIOpen still runs.

Problem: with ``torch.backends.cudnn.benchmark`` on, MIOpen "find" times every applicable solver
for every conv problem on first use and JIT-compiles the HIP/CK kernels it tries.  On a fresh
MI355X box there is no gfx950 system find-db in ``/opt/rocm/share/miopen/db``, so a ResNet-50 run
spent ~360 s of warmup tuning (BENCH_r01.json), and N ranks of one job would each tune the same
problems concurrently against one user db.

Fix (MI355X-first, no reference counterpart -- the reference runs cuDNN/Horovod images):
  * the user find-db / perf-db that a tuning run wrote is shipped IN-TREE under
    ``determined_1_amd/ops/miopen_db/`` (text files keyed by problem + ``gfx950_256``);
  * ``configure(env)`` points ``MIOPEN_USER_DB_PATH`` / ``MIOPEN_CUSTOM_CACHE_DIR`` at a writable
    per-user (and, in a multi-rank job, per-local-rank) copy under ``$TMPDIR`` seeded from the
    shipped files, before any process touches the GPU, so every rank (and every trial container)
    gets find results from the db instead of re-tuning; only the kernels MIOpen actually picked
    are compiled (or loaded from the seeded kernel cache).  Seeding is key-merging and stamped:
    entries the user already tuned are never overwritten, and a changed shipped db is merged in
    again on the next run;
  * ``harvest(dst)`` copies a run's db back so a tuning run can refresh the shipped copy.

This module deliberately imports nothing from torch or the package: launchers call it before
deciding which process owns which GPU.
"""
import hashlib
import os
import shutil
from typing import Dict, MutableMapping, Optional

SHIPPED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "miopen_db")


def _merge_text_db(src: str, dst: str) -> bool:
    """Merge a MIOpen text db (``key=value`` lines): keys already in ``dst`` keep their (user-tuned)
    value, keys only in ``src`` are appended.  Returns True if ``dst`` changed."""
    def entries(path: str) -> Dict[str, str]:
        out = {}  # type: Dict[str, str]
        with open(path, errors="replace") as f:
            for line in f:
                line = line.rstrip("\n")
                if "=" in line:
                    k, v = line.split("=", 1)
                    out[k] = v
        return out

    have = entries(dst) if os.path.exists(dst) else {}
    add = {k: v for k, v in entries(src).items() if k not in have}
    if not add and os.path.exists(dst):
        return False
    tmp = dst + ".tmp%d" % os.getpid()
    with open(tmp, "w") as f:
        for k, v in list(have.items()) + list(add.items()):
            f.write(f"{k}={v}\n")
    os.replace(tmp, dst)
    return True


def _copy_tree_missing(src: str, dst: str) -> int:
    """Seed ``dst`` from ``src``: text dbs are key-merged (never overwriting an entry ``dst``
    already holds), binary files (the kernel cache) are copied only when missing.  Returns the
    number of files written."""
    n = 0
    if not os.path.isdir(src):
        return 0
    for root, _, files in os.walk(src):
        rel = os.path.relpath(root, src)
        out = os.path.join(dst, rel) if rel != "." else dst
        os.makedirs(out, exist_ok=True)
        for f in files:
            if f.startswith(".") or f.endswith(".md"):
                continue
            s = os.path.join(root, f)
            d = os.path.join(out, f)
            try:
                if f.endswith(".txt"):
                    n += int(_merge_text_db(s, d))
                elif not os.path.exists(d):
                    tmp = d + ".tmp%d" % os.getpid()
                    shutil.copyfile(s, tmp)
                    os.replace(tmp, d)
                    n += 1
            except OSError:
                continue
    return n


def _shipped_stamp() -> str:
    """Identity of the shipped db (names, sizes, mtimes): a per-run copy is re-seeded when it changes."""
    h = hashlib.sha1()
    for root, _, files in sorted(os.walk(SHIPPED)):
        for f in sorted(files):
            st = os.stat(os.path.join(root, f))
            h.update(f"{os.path.relpath(os.path.join(root, f), SHIPPED)}:{st.st_size}:{int(st.st_mtime)}".encode())
    return h.hexdigest()


def run_root(env: Optional[MutableMapping[str, str]] = None) -> str:
    """Per-user root of the writable db copy; one sub-directory per local rank of a multi-rank job
    (ranks never write one db concurrently: MIOpen's text dbs are not multi-writer safe)."""
    e = os.environ if env is None else env
    base = e.get("DET_MIOPEN_DIR") or os.path.join(e.get("TMPDIR", "/tmp"), "det-miopen-%d" % os.getuid())
    if int(e.get("WORLD_SIZE", e.get("LOCAL_WORLD_SIZE", "1")) or 1) > 1 and "LOCAL_RANK" in e:
        base = os.path.join(base, "rank%s" % e["LOCAL_RANK"])
    return base


def configure(env: Optional[MutableMapping[str, str]] = None) -> Optional[str]:
    """Seed and select the MIOpen user db + kernel cache for processes started with ``env``.

    Respects an explicit ``MIOPEN_USER_DB_PATH`` (a user-chosen db is left alone) and
    ``DET_MIOPEN_DB=0`` (disable).  Returns the user-db directory in use."""
    e = os.environ if env is None else env
    if e.get("DET_MIOPEN_NAIVE", "0") != "1":
        # MIOpen's find times every applicable solver, including the GPU reference ("naive")
        # convolutions, which take 0.05-0.5 s per call at batch 512: rocprofv3 showed 114 s of
        # naive_conv_ab_nonpacked_{fwd,bwd,wrw} in the first ResNet-50 batch
        # (profiles/r2_resnet50_first_batch_find.txt).  They are never the fastest solver here.
        for d in ("FWD", "BWD", "WRW"):
            e.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_" + d, "0")
    if e.get("DET_MIOPEN_DB", "1") == "0":
        return e.get("MIOPEN_USER_DB_PATH")
    if e.get("MIOPEN_USER_DB_PATH"):
        return e["MIOPEN_USER_DB_PATH"]
    root = run_root(e)
    db = os.path.join(root, "db")
    cache = os.path.join(root, "cache")
    try:
        os.makedirs(db, exist_ok=True)
        os.makedirs(cache, exist_ok=True)
        stamp_path = os.path.join(root, ".seeded")
        stamp = _shipped_stamp()
        old = open(stamp_path).read() if os.path.exists(stamp_path) else ""
        if old != stamp:  # first use, or the shipped db changed: merge it in (user entries win)
            _copy_tree_missing(os.path.join(SHIPPED, "db"), db)
            _copy_tree_missing(os.path.join(SHIPPED, "cache"), cache)
            with open(stamp_path + ".tmp%d" % os.getpid(), "w") as f:
                f.write(stamp)
            os.replace(stamp_path + ".tmp%d" % os.getpid(), stamp_path)
    except OSError:
        return None
    e["MIOPEN_USER_DB_PATH"] = db
    e.setdefault("MIOPEN_CUSTOM_CACHE_DIR", cache)
    return db


def harvest(dst: str, env: Optional[MutableMapping[str, str]] = None, with_cache: bool = False) -> int:
    """Copy the active user db (and optionally the kernel cache) to ``dst`` (e.g. to refresh
    ``SHIPPED`` after a tuning run)."""
    e = os.environ if env is None else env
    n = 0
    db = e.get("MIOPEN_USER_DB_PATH")
    if db:
        n += _copy_tree_missing(db, os.path.join(dst, "db"))
    cache = e.get("MIOPEN_CUSTOM_CACHE_DIR")
    if with_cache and cache:
        n += _copy_tree_missing(cache, os.path.join(dst, "cache"))
    return n
