"""Build the in-tree HIP shared libraries for gfx950.

* ``awebox_amd/libawegpu.so`` -- the AP2 collocation evaluator (include/awegpu.h);
* ``awebox_amd/libawempc.so`` -- the 3-DOF tracking-MPC evaluator (include/awempc.h);
* ``awebox_amd/libawedual.so`` -- the dual-kite (multi-kite) evaluator (include/awedual.h);
* ``awebox_amd/libawelu.so`` -- batched LU of the structured KKT solve's interval blocks.

Plain ``hipcc -shared -fPIC`` (no JIT cache): the .so files live next to this file so that they
travel with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
LIB = os.path.join(HERE, "libawegpu.so")
LIB_MPC = os.path.join(HERE, "libawempc.so")
LIB_DUAL = os.path.join(HERE, "libawedual.so")
LIB_LU = os.path.join(HERE, "libawelu.so")
_COMMON = [os.path.join(CSRC, f) for f in ("ap2_model.hpp", "ap2_tables.hpp", "scalar.hpp")] + [
    os.path.join(INCLUDE, "awegpu.h")]
TARGETS = {
    LIB: ([os.path.join(CSRC, "awegpu.hip")], _COMMON),
    LIB_MPC: ([os.path.join(CSRC, "awempc.hip")],
              _COMMON + [os.path.join(CSRC, f) for f in ("kite3_model.hpp", "kite3_tables.hpp")]
              + [os.path.join(INCLUDE, "awempc.h")]),
    LIB_DUAL: ([os.path.join(CSRC, "awedual.hip")],
               _COMMON + [os.path.join(CSRC, f) for f in ("dual_model.hpp", "dual_tables.hpp")]
               + [os.path.join(INCLUDE, "awedual.h")]),
    LIB_LU: ([os.path.join(CSRC, "batched_lu.hip")], []),
}
ARCH = os.environ.get("AWE_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-Wno-unused-value",
         "-Wno-unused-result"]


def _stale(lib, deps) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(p) > t for p in deps)


def build_one(lib: str, force: bool = False, verbose: bool = False) -> str:
    sources, headers = TARGETS[lib]
    if not force and not _stale(lib, sources + headers):
        return lib
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *FLAGS, *sources, "-o", lib + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(lib + ".tmp", lib)
    return lib


def build(force: bool = False, verbose: bool = False) -> str:
    """Build every library; returns the AP2 library path (the headline evaluator)."""
    for lib in TARGETS:
        build_one(lib, force=force, verbose=verbose)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print("\n".join(TARGETS))
