"""Build libdeig.so (HIP, gfx950) in-tree with hipcc.

The shared library is built next to this file so it travels with the repo
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libdeig.so")
SOURCES = ["capi.hip", "syrk.hip", "syrk_split.hip", "syrk_u8.hip", "skinny.hip", "rr.hip", "oja.hip",
           "project.hip", "sweep.hip", "shift.hip"]
# Per-source extra flags.  sweep.hip: keep the split's scalar f32 subtractions
# unpacked (v_pk_add_f32 beside MFMAs costs issue cycles, MI355X_MICROARCH.md).
EXTRA_FLAGS = {"sweep.hip": ["-fno-slp-vectorize"], "syrk_split.hip": ["-fno-slp-vectorize"]}
HEADERS = ["deig_internal.hpp", os.path.join("..", "..", "include", "deig.h")]
# Test-only variant (tests/test_gpu_oja_timeout.py): oja.hip with a zero spin bound, so
# every resident hand-off times out and the DEIG_ETIMEOUT report can be exercised; the
# other objects are the shipped library's.
OJA_TIMEOUT_LIB = os.path.join(HERE, "libdeig_test_oja_timeout.so")
ARCH = os.environ.get("DEIG_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build libdeig.so)")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    return any(os.path.getmtime(p) > t for p in deps)


def build_library(force: bool = False, verbose: bool = True, defines=(), out: str | None = None) -> str:
    """Build libdeig.so (or, with ``defines`` such as ``-DDEIG_AB_SYRK_VARIANT=22``, an
    A/B variant into ``out`` - measurement tooling only; the shipped library reads
    no environment and has no knobs)."""
    lib = out or LIB
    if not force and not defines and lib == LIB and not _stale():
        return LIB
    objs = []
    tmpdir = os.path.join(HERE, "build" if not defines else "build_ab")
    os.makedirs(tmpdir, exist_ok=True)
    hipcc = _hipcc()
    procs = []
    for src in SOURCES:
        obj = os.path.join(tmpdir, src.replace(".hip", ".o"))
        objs.append(obj)
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
               "-Wno-unused-function", "-Wno-inline-asm"] + list(defines) + EXTRA_FLAGS.get(src, []) + \
            ["-c", os.path.join(CSRC, src), "-o", obj]
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + out.decode())
        if verbose and out.strip():
            sys.stderr.write(out.decode())
    tmp_lib = lib + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp_lib] + objs
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stdout.decode())
    os.replace(tmp_lib, lib)
    if verbose:
        sys.stderr.write(f"built {lib}\n")
    return lib


def build_oja_timeout_lib(verbose: bool = True) -> str:
    """The test-only variant OJA_TIMEOUT_LIB (oja.hip with -DDEIG_AB_OJA_SPIN_TICKS=0,
    linked with the shipped library's other objects; build_library first)."""
    tmpdir = os.path.join(HERE, "build")
    hipcc = _hipcc()
    obj = os.path.join(tmpdir, "oja_timeout.o")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
           "-Wno-inline-asm", "-DDEIG_AB_OJA_SPIN_TICKS=0", "-c", os.path.join(CSRC, "oja.hip"), "-o", obj]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + r.stdout.decode())
    objs = [obj if s == "oja.hip" else os.path.join(tmpdir, s.replace(".hip", ".o")) for s in SOURCES]
    tmp_lib = OJA_TIMEOUT_LIB + ".tmp"
    r = subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp_lib] + objs,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stdout.decode())
    os.replace(tmp_lib, OJA_TIMEOUT_LIB)
    if verbose:
        sys.stderr.write(f"built {OJA_TIMEOUT_LIB}\n")
    return OJA_TIMEOUT_LIB


if __name__ == "__main__":
    build_library(force="--force" in sys.argv)
