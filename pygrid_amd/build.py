"""Build libpygrid_hip.so in-tree for gfx950 with hipcc (no torch in the link line).

Parity-relevant flags: ``-ffp-contract=off`` (the iterative plan's ``a*k + d`` must not become
an FMA), no fast-math, f32 denormals kept (hipcc default), correctly rounded f32 division
(hipcc default ``-fhip-fp32-correctly-rounded-divide-sqrt``).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "libpygrid_hip.so"
SOURCES = [CSRC / "pgh_kernels.hip", CSRC / "pgh_api.cpp", CSRC / "pgh_ingest.cpp", CSRC / "pgh_reduce.cpp",
           CSRC / "pgh_slots.cpp", CSRC / "pgh_group.cpp", CSRC / "pgh_state.cpp", CSRC / "pgh_b64.cpp"]
HEADERS = [CSRC / "pgh_kernels.h", CSRC / "pgh_state.h", CSRC / "pgh_internal.h", CSRC / "pgh_ctx.h",
           ROOT / "include" / "pgh_api.h"]
ARCH = os.environ.get("PGH_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (set HIPCC)")


def _stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return any(p.stat().st_mtime > t for p in SOURCES + HEADERS + [Path(__file__)])


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and not _stale():
        return LIB
    objs = []
    bdir = ROOT / "build" / "pgh"
    bdir.mkdir(parents=True, exist_ok=True)
    common = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-ffp-contract=off",
              f"-I{ROOT / 'include'}"]
    for src in SOURCES:
        obj = bdir / (src.name + ".o")
        cmd = [hipcc(), *common, "-c", str(src), "-o", str(obj)]
        if src.suffix == ".hip":
            cmd[1:1] = ["-x", "hip", f"--offload-arch={ARCH}", "--no-offload-compress"]
        else:
            cmd[1:1] = ["-D__HIP_PLATFORM_AMD__"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        objs.append(str(obj))
    tmp = LIB.with_suffix(".so.tmp")
    # -ldl: librccl.so.1 is dlopen'ed at the first multi-GPU collective (no link-time RCCL)
    cmd = [hipcc(), "-shared", "-fPIC", *objs, "-o", str(tmp), f"--offload-arch={ARCH}",
           "-Wl,-soname,libpygrid_hip.so", "-ldl",
           "-Wl,-z,now"]  # bind every symbol at load: the node's first cycle close pays no lazy PLT lookups
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
