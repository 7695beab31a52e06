"""Build the gfx950 kernel library in-tree.

    python -m determined_1_amd.ops.build [--force]

Produces ``determined_1_amd/ops/libdetkernels.so`` with ``hipcc --offload-arch=gfx950``.  The .so
is git-ignored but travels to the GPU box with the repo snapshot.  Rebuilds only when a source
is newer than the library (or ``--force``).
"""
import argparse
import os
import pathlib
import shutil
import subprocess
import sys
from typing import List

HERE = pathlib.Path(__file__).resolve().parent
SRC_DIR = HERE / "csrc"
SOURCES = [SRC_DIR / "det_kernels.hip", SRC_DIR / "det_norm.hip", SRC_DIR / "det_transformer.hip", SRC_DIR / "det_attention.hip",
           SRC_DIR / "det_pool.hip", SRC_DIR / "det_conv.hip", SRC_DIR / "det_igemm.hip", SRC_DIR / "det_detect.hip",
           SRC_DIR / "det_stream.hip", SRC_DIR / "det_cnn.hip", SRC_DIR / "det_embed.hip", SRC_DIR / "det_blaslt.hip",
           SRC_DIR / "det_graph.hip", SRC_DIR / "det_gemm8.hip"]
OUT = HERE / "libdetkernels.so"
ARCH = os.environ.get("DET_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (expected /opt/rocm/bin/hipcc)")


def needs_build(out: pathlib.Path, sources: List[pathlib.Path]) -> bool:
    if not out.exists():
        return True
    mtime = out.stat().st_mtime
    return any(s.stat().st_mtime > mtime for s in sources if s.exists())


def build(force: bool = False, verbose: bool = False) -> pathlib.Path:
    """Compile each source to an object in parallel (one hipcc per .hip), then link the .so."""
    sources = [s for s in SOURCES if s.exists()]
    if not force and not needs_build(OUT, sources):
        return OUT
    from concurrent.futures import ThreadPoolExecutor

    objdir = HERE / "build"
    objdir.mkdir(exist_ok=True)
    flags = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC"]

    def compile_one(src: pathlib.Path) -> pathlib.Path:
        obj = objdir / (src.stem + ".o")
        if force or not obj.exists() or obj.stat().st_mtime < src.stat().st_mtime:
            cmd = [hipcc()] + flags + ["-c", str(src), "-o", str(obj)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
        return obj

    jobs = max(1, min(len(sources), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, sources))
    tmp = OUT.with_suffix(".so.tmp")
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp)] + [str(o) for o in objs] + ["-ldl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args()
    print(build(force=args.force, verbose=True))


if __name__ == "__main__":
    main()
