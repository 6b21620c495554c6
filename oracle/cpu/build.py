"""Build the CPU port of the evaluator (oracle/cpu/libap2cpu.so) -- test/baseline infrastructure.

Plain g++ with OpenMP; x86-64-v3 (AVX2/FMA) code so that it runs on any current EPYC/Xeon host.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(HERE, "libap2cpu.so")
LIB_DUAL = os.path.join(HERE, "libdualcpu.so")
DUAL_SOURCES = [os.path.join(HERE, "dual_cpu.cpp")]
DUAL_HEADERS = [os.path.join(ROOT, "awebox_amd", "csrc", f) for f in
                ("dual_model.hpp", "dual_tables.hpp", "ap2_model.hpp", "ap2_tables.hpp", "scalar.hpp")] + [
    os.path.join(ROOT, "include", f) for f in ("awedual.h", "awegpu.h")]
SOURCES = [os.path.join(HERE, "ap2_cpu.cpp")]
HEADERS = [os.path.join(HERE, "dualn.hpp")] + [
    os.path.join(ROOT, "awebox_amd", "csrc", f) for f in ("ap2_model.hpp", "ap2_tables.hpp", "scalar.hpp")] + [
    os.path.join(ROOT, "include", "awegpu.h")]
FLAGS = ["-O3", "-march=x86-64-v3", "-fopenmp", "-fPIC", "-shared", "-std=c++17",
         "-I", os.path.join(ROOT, "awebox_amd", "csrc"), "-I", os.path.join(ROOT, "include")]


def _stale(lib=LIB, deps=None) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(p) > t for p in (deps or SOURCES + HEADERS))


def _compile(lib, sources, verbose):
    cmd = [os.environ.get("CXX", "g++"), *FLAGS, *sources, "-o", lib + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)


def build(force: bool = False, verbose: bool = False) -> str:
    """Both CPU ports: libap2cpu.so (AP2) and libdualcpu.so (dual kites); returns the AP2 path."""
    if force or _stale():
        _compile(LIB, SOURCES, verbose)
    if force or _stale(LIB_DUAL, DUAL_SOURCES + DUAL_HEADERS):
        _compile(LIB_DUAL, DUAL_SOURCES, verbose)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
