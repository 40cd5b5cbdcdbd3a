"""Build libgaplac_hip.so in-tree (gaplac_amd/_lib/) with hipcc for gfx950.

    python -m gaplac_amd.build [--force]

Cross-compiles without a GPU. The .so is git-ignored but travels to the GPU box with the
repo snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["gaplac_kernels.hip", "gaplac_api.hip", "gaplac_dist.hip"]
HEADERS = ["gaplac_internal.h", os.path.join("..", "..", "include", "gaplac.h")]
OUT = os.path.join(HERE, "_lib", "libgaplac_hip.so")
ARCH = os.environ.get("GAPLAC_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm 7.x expected under /opt/rocm)")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps)


def build_library(force: bool = False, verbose: bool = False, out: str | None = None, defines=()) -> str:
    """The in-tree library (default), or an A/B variant: out = another path, defines =
    extra -D switches (e.g. ("GAPLAC_EARLY_DEQ=0",)), loaded with GAPLAC_LIB_PATH."""
    target = out or OUT
    if out is None and not defines and not force and not _stale():
        return OUT
    os.makedirs(os.path.dirname(os.path.abspath(target)), exist_ok=True)
    tmp = target + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall"]
    cmd += [f"-D{d}" for d in defines]
    cmd += ["-o", tmp] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stderr[-4000:]}")
    os.replace(tmp, target)
    return target


if __name__ == "__main__":
    # python -m gaplac_amd.build [--force] [--out PATH] [-DNAME=VALUE ...]
    a = sys.argv[1:]
    out = a[a.index("--out") + 1] if "--out" in a else None
    print(build_library(force="--force" in a, verbose=True, out=out,
                        defines=[x[2:] for x in a if x.startswith("-D")]))
