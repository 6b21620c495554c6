"""Build the in-tree HIP shared libraries for gfx950.

* ``awebox_amd/libawegpu.so`` -- the AP2 collocation evaluator (include/awegpu.h);
* ``awebox_amd/libawempc.so`` -- the 3-DOF tracking-MPC evaluator (include/awempc.h);
* ``awebox_amd/libawedual.so`` -- the dual-kite (multi-kite) evaluator (include/awedual.h);
* ``awebox_amd/libawelu.so`` -- batched LU of the structured KKT solve's interval blocks.

Plain ``hipcc -shared -fPIC`` (no JIT cache): the .so files live next to this file so that they
travel with the repository snapshot to the GPU box.

Before the libraries are compiled, ``generate()`` refreshes the generated node code: each node model
is traced and differentiated by its generator under ``csrc/gen/`` (g++, host) for the default
constants -- ``ap2_nodejac.gen.hpp`` / ``ap2_nodehess.gen.hpp`` (AP2 Jacobian and Hessian),
``kite3_nodejac.gen.hpp`` (tracking MPC), ``dual_nodejac.gen.hpp`` (dual kites) -- and the straight-line
code they write is what the instance-minor kernels run.
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
GEN_HEADER = os.path.join(CSRC, "ap2_nodejac.gen.hpp")
GEN_SOURCES = [os.path.join(CSRC, "gen", f) for f in ("ap2_jacgen.cpp", "sym.hpp")] + [
    os.path.join(CSRC, f) for f in ("ap2_model.hpp", "ap2_tables.hpp", "scalar.hpp")] + [
    os.path.join(INCLUDE, "awegpu.h"), os.path.join(HERE, "problem.py")]
# the node-Hessian code (forward-over-reverse, csrc/gen/ap2_hessgen.cpp)
HESS_HEADER = os.path.join(CSRC, "ap2_nodehess.gen.hpp")
HESS_SOURCES = [os.path.join(CSRC, "gen", "ap2_hessgen.cpp")] + GEN_SOURCES[1:]
# the tracking-MPC node-Jacobian code (csrc/gen/kite3_jacgen.cpp)
K3_HEADER = os.path.join(CSRC, "kite3_nodejac.gen.hpp")
K3_SOURCES = [os.path.join(CSRC, "gen", f) for f in ("kite3_jacgen.cpp", "sym.hpp")] + [
    os.path.join(CSRC, f) for f in ("kite3_model.hpp", "kite3_tables.hpp", "ap2_tables.hpp", "scalar.hpp")] + [
    os.path.join(INCLUDE, "awempc.h"), os.path.join(INCLUDE, "awegpu.h"), os.path.join(HERE, "kite3.py")]
# the dual-kite node-Jacobian code (csrc/gen/dual_jacgen.cpp)
DUAL_HEADER = os.path.join(CSRC, "dual_nodejac.gen.hpp")
DUAL_SOURCES = [os.path.join(CSRC, "gen", f) for f in ("dual_jacgen.cpp", "sym.hpp")] + [
    os.path.join(CSRC, f) for f in ("dual_model.hpp", "dual_tables.hpp", "ap2_model.hpp", "ap2_tables.hpp",
                                    "scalar.hpp")] + [
    os.path.join(INCLUDE, "awedual.h"), os.path.join(INCLUDE, "awegpu.h"), os.path.join(HERE, "dual.py")]
# (header, generator source, inputs hashed into the header's first line, default constants)
GENERATORS = [(GEN_HEADER, "ap2_jacgen.cpp", GEN_SOURCES, "ap2"), (HESS_HEADER, "ap2_hessgen.cpp", HESS_SOURCES, "ap2"),
              (K3_HEADER, "kite3_jacgen.cpp", K3_SOURCES, "kite3"), (DUAL_HEADER, "dual_jacgen.cpp", DUAL_SOURCES, "dual")]
# content hash of GEN_SOURCES recorded in the generated header's first line: the header is stale
# when the hash differs (file times do not survive a checkout or the copy to the GPU box)
_HASH_TAG = "// inputs-sha1: "
_COMMON = [os.path.join(CSRC, f) for f in ("ap2_model.hpp", "ap2_tables.hpp", "scalar.hpp")] + [
    os.path.join(INCLUDE, "awegpu.h")]
TARGETS = {
    LIB: ([os.path.join(CSRC, "awegpu.hip")], _COMMON + [GEN_HEADER, HESS_HEADER]),
    LIB_MPC: ([os.path.join(CSRC, "awempc.hip")],
              _COMMON + [os.path.join(CSRC, f) for f in ("kite3_model.hpp", "kite3_tables.hpp", "im_layout.hpp")]
              + [os.path.join(INCLUDE, "awempc.h"), K3_HEADER]),
    LIB_DUAL: ([os.path.join(CSRC, "awedual.hip"), os.path.join(CSRC, "awedual_gen.hip")],
               _COMMON + [os.path.join(CSRC, f) for f in ("dual_model.hpp", "dual_tables.hpp", "dual_hess_tables.hpp",
                                                          "awedual_gen.hpp", "im_layout.hpp")]
               + [os.path.join(INCLUDE, "awedual.h"), DUAL_HEADER]),
    LIB_LU: ([os.path.join(CSRC, "batched_lu.hip")], [os.path.join(INCLUDE, "awelu.h")]),
}
ARCH = os.environ.get("AWE_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-Wno-unused-value",
         "-Wno-unused-result"]


def _lib_hash(lib) -> str:
    """Content hash of everything a library is built from: its sources and headers (names and
    bytes), the compiler flags and the offload architecture."""
    import hashlib
    sources, headers = TARGETS[lib]
    h = hashlib.sha1(" ".join(FLAGS).encode() + b"\0")
    for p in sources + headers:
        with open(p, "rb") as fh:
            h.update(os.path.basename(p).encode() + b"\0" + fh.read())
    return h.hexdigest()


def _stamp(lib) -> str:
    return lib + ".sha1"


def _stale(lib) -> bool:
    """A library is stale unless the content hash recorded beside it at its build (``<lib>.sha1``)
    matches its inputs now.  File times are not used: they do not survive a checkout or the copy of
    the tree to the GPU box, and a library copied there with newer times than edited sources would
    pass a time check while being built from other code."""
    if not os.path.exists(lib) or not os.path.exists(_stamp(lib)):
        return True
    with open(_stamp(lib)) as fh:
        return fh.read().strip() != _lib_hash(lib)


def build_one(lib: str, force: bool = False, verbose: bool = False) -> str:
    sources, headers = TARGETS[lib]
    if not force and not _stale(lib):
        return lib
    want = _lib_hash(lib)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if len(sources) == 1:
        cmd = [hipcc, *FLAGS, *sources, "-o", lib + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True, cwd=CSRC)
    else:
        # several translation units: compiled side by side into objects, then linked
        import tempfile
        with tempfile.TemporaryDirectory() as tmp:
            objs = [os.path.join(tmp, os.path.splitext(os.path.basename(src))[0] + ".o") for src in sources]
            cflags = [f for f in FLAGS if f != "-shared"] + ["-c"]
            procs = []
            for src, obj in zip(sources, objs):
                cmd = [hipcc, *cflags, src, "-o", obj]
                if verbose:
                    print(" ".join(cmd), file=sys.stderr)
                procs.append((cmd, subprocess.Popen(cmd, cwd=CSRC)))
            for cmd, pr in procs:
                if pr.wait() != 0:
                    raise subprocess.CalledProcessError(pr.returncode, cmd)
            cmd = [hipcc, *FLAGS, *objs, "-o", lib + ".tmp"]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(lib + ".tmp", lib)
    with open(_stamp(lib) + ".tmp", "w") as fh:
        fh.write(want + "\n")
    os.replace(_stamp(lib) + ".tmp", _stamp(lib))
    return lib


def gen_inputs_hash(sources=None) -> str:
    import hashlib
    h = hashlib.sha1()
    for p in (GEN_SOURCES if sources is None else sources):
        with open(p, "rb") as fh:
            h.update(os.path.basename(p).encode() + b"\0" + fh.read())
    return h.hexdigest()


def _header_hash(header=GEN_HEADER) -> str | None:
    if not os.path.exists(header):
        return None
    with open(header) as fh:
        first = fh.readline()
    return first[len(_HASH_TAG):].strip() if first.startswith(_HASH_TAG) else None


def generate(force: bool = False, verbose: bool = False) -> str:
    """Regenerate the generated headers (csrc/ap2_nodejac.gen.hpp: node Jacobians;
    csrc/ap2_nodehess.gen.hpp: node Hessians) when the model, a generator or the default constants
    changed (content hash of the generator's inputs against the one recorded in the header); a file
    is rewritten only if its content differs, so an unchanged model does not trigger a rebuild.
    Without a host C++ compiler the committed headers are kept (tests/test_codegen.py checks them
    against the model wherever g++ exists)."""
    for header, gen, sources, model in GENERATORS:
        _generate_one(header, gen, sources, force, verbose, model)
    return GEN_HEADER


def _default_constants(model):
    if model == "kite3":
        from . import kite3
        return kite3.build_constants().consts
    if model == "dual":
        from . import dual
        return dual.build_constants().consts
    from . import problem as pb
    return pb.build_constants(pb.Ap2Config()).consts


def _generate_one(header, gen, sources, force, verbose, model="ap2"):
    import shutil
    want = gen_inputs_hash(sources)
    if not force and _header_hash(header) == want:
        return header
    cxx = os.environ.get("CXX", "g++")
    if shutil.which(cxx) is None:
        if os.path.exists(header):
            if verbose:
                print(f"{cxx} not found: keeping the committed {os.path.basename(header)}", file=sys.stderr)
            return header
        raise RuntimeError(f"{cxx} not found and no generated header to fall back to")
    import tempfile

    import numpy as np

    consts = _default_constants(model)
    with tempfile.TemporaryDirectory() as tmp:
        exe = os.path.join(tmp, os.path.splitext(gen)[0])
        cmd = [cxx, "-O1", "-std=c++17", os.path.join(CSRC, "gen", gen), "-o", exe]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        cfile = os.path.join(tmp, "consts.txt")
        np.savetxt(cfile, consts)
        out = os.path.join(tmp, "gen.hpp")
        r = subprocess.run([exe, cfile, out], check=True, capture_output=True, text=True)
        if verbose:
            print(r.stdout.strip(), file=sys.stderr)
        new = _HASH_TAG + want + "\n" + open(out).read()
    old = open(header).read() if os.path.exists(header) else None
    if new != old:
        with open(header + ".tmp", "w") as fh:
            fh.write(new)
        os.replace(header + ".tmp", header)
    return header


def build(force: bool = False, verbose: bool = False) -> str:
    """Build every library (side by side: the dual-kite library's generated node kernel alone takes
    ~9 minutes of hipcc); returns the AP2 library path (the headline evaluator)."""
    from concurrent.futures import ThreadPoolExecutor
    generate(force=force, verbose=verbose)
    with ThreadPoolExecutor(max_workers=len(TARGETS)) as pool:
        for fut in [pool.submit(build_one, lib, force, verbose) for lib in TARGETS]:
            fut.result()
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print("\n".join(TARGETS))
