"""Build the in-tree HIP shared library ``awebox_amd/libawegpu.so`` for gfx950.

Plain ``hipcc -shared -fPIC`` (no JIT cache): the .so lives next to this file so that it travels
with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libawegpu.so")
SOURCES = [os.path.join(CSRC, "awegpu.hip")]
HEADERS = [os.path.join(CSRC, f) for f in ("ap2_model.hpp", "ap2_tables.hpp", "scalar.hpp")] + [
    os.path.join(os.path.dirname(HERE), "include", "awegpu.h")]
ARCH = os.environ.get("AWE_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-Wno-unused-value",
         "-Wno-unused-result"]


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *FLAGS, *SOURCES, "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
