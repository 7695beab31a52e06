"""Build the native C++ control plane (``native/``) in-tree: ``make -C native``.

Outputs ``determined_1_amd/_native/{libdetcore.so,det-master,det-agent}``.
"""
import os
import pathlib
import subprocess
import sys

REPO = pathlib.Path(__file__).resolve().parent.parent
NATIVE = REPO / "native"


def build_native(force: bool = False, jobs: int = 8) -> None:
    if not (NATIVE / "Makefile").exists():
        raise RuntimeError(f"native sources not found at {NATIVE}")
    if force:
        subprocess.run(["make", "-C", str(NATIVE), "clean"], check=True, stdout=subprocess.DEVNULL)
    jobs = min(jobs, 16)
    subprocess.run(["make", "-C", str(NATIVE), f"-j{jobs}", "all"], check=True,
                   stdout=subprocess.DEVNULL if not os.environ.get("DET_BUILD_VERBOSE") else None)


if __name__ == "__main__":
    build_native(force="--force" in sys.argv)
    print("built", REPO / "determined_1_amd" / "_native")
