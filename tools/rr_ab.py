"""A/B of the one-workgroup Rayleigh-Ritz small solve (csrc/rr.hip): the r04
rr_small2_body (blocked Cholesky / L^-1, lower-triangle Jacobi with V in registers)
against the r03 rr_small_body (-DDEIG_AB_RR_V1), in ONE process on the same matrices.
Measurement tooling only (the shipped library has no knobs).

  python tools/rr_ab.py build            # here: tools/ab_libs/libdeig_rrv1.so
  python tools/rr_ab.py run [--reps R] [--other LIB]   # GPU box: per case solve ms (median), sweeps,
                                         # residual and the two solves' agreement
(rocprofv3 --kernel-trace --stats around `run` gives rr_small_kernel vs
rr_small2_kernel averages.)
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIBDIR = os.path.join(ROOT, "tools", "ab_libs")
V1 = os.path.join(LIBDIR, "libdeig_rrv1.so")


SCALARJ = os.path.join(LIBDIR, "libdeig_rrscalarj.so")


def build():
    from distributed_eigenspaces_amd import _build
    os.makedirs(LIBDIR, exist_ok=True)
    _build.build_library()
    objdir = os.path.join(_build.HERE, "build")
    hipcc = _build._hipcc()
    others = [os.path.join(objdir, s.replace(".hip", ".o")) for s in _build.SOURCES if s != "rr.hip"]
    for define, out in (("-DDEIG_AB_RR_V1", V1), ("-DDEIG_AB_RR_SCALARJ", SCALARJ)):
        obj = out + ".o"
        subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                        "-Wno-unused-function", "-Wno-inline-asm", define, "-c",
                        os.path.join(_build.CSRC, "rr.hip"), "-o", obj], check=True)
        subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", out, obj] + others,
                       check=True)
        os.remove(obj)
        print("built", out)


def _bind(path):
    from distributed_eigenspaces_amd import _lib
    L = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def run(reps, other=None):
    import torch

    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import _lib, synthetic
    dev = torch.device("cuda", 0)
    libs = {"v2": _bind(_lib.LIB_PATH), "v1": _bind(other or V1)}
    cases = [("c1", 6250, 3072, 10), ("c2", 1 << 16, 3072, 16), ("c3", 16384, 8192, 64),
             ("c5", 32768, 16384, 128)]
    for name, n, d, k in cases:
        U = synthetic.planted_basis(d, k, seed=0, device=dev)
        X = synthetic.spiked_samples(n, U, seed=1)
        S = de.sigma_hat(X)
        del X
        torch.cuda.synchronize()
        res = {}
        for tag in ("v2", "v1", "v2", "v1"):
            _lib._lib = libs[tag]
            ts = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r = de.topk_eigh(S, k, check_finite=False)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            res.setdefault(tag, []).extend(ts)
            res[tag + "_r"] = r
        a, b = res["v2_r"], res["v1_r"]
        Va, Vb = a.V.double(), b.V.double()
        pd = float(torch.linalg.matrix_norm(Va @ Va.t() - Vb @ Vb.t())) if d <= 8192 else float(
            (torch.linalg.svdvals(Va.t() @ Vb).clamp(max=1).pow(2).neg().add(1).clamp(min=0).sum()).sqrt() * 2 ** 0.5)
        out = {"case": name, "d": d, "k": k, "p": de.default_subspace(d, k),
               "v2_ms": statistics.median(res["v2"]), "v1_ms": statistics.median(res["v1"]),
               "v2_sweeps": a.sweeps, "v1_sweeps": b.sweeps, "v2_resid": a.resid, "v1_resid": b.resid,
               "P_dist_v2_v1": pd,
               "evals_rel_v2_v1": float(((a.evals - b.evals).abs() / b.evals.abs()).max())}
        print(json.dumps(out), flush=True)
        del S
        torch.cuda.empty_cache()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--other", default=None, help="B library for run (default: the r03 solve)")
    a = ap.parse_args()
    if a.cmd == "build":
        build()
    else:
        run(a.reps, a.other)
