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
SOURCES = [os.path.join(HERE, "ap2_cpu.cpp")]
HEADERS = [os.path.join(HERE, "dualn.hpp")] + [
    os.path.join(ROOT, "awebox_amd", "csrc", f) for f in ("ap2_model.hpp", "ap2_tables.hpp", "scalar.hpp")] + [
    os.path.join(ROOT, "include", "awegpu.h")]
FLAGS = ["-O3", "-march=x86-64-v3", "-fopenmp", "-fPIC", "-shared", "-std=c++17",
         "-I", os.path.join(ROOT, "awebox_amd", "csrc"), "-I", os.path.join(ROOT, "include")]


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    cmd = [os.environ.get("CXX", "g++"), *FLAGS, *SOURCES, "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
