"""A/B timing of covariance SYRK builds in ONE process (interleaved rounds, same
device, same data; cdna_hip_programming.md §5.4 rule 24).  Measurement tooling only:
the variants are separate builds of libdeig.so with -DDEIG_AB_SYRK_VARIANT=N (the
shipped library has no knobs).

  python tools/syrk_ab.py build 162 174            # here (CPU): tools/ab_libs/libdeig_v*.so
  python tools/syrk_ab.py run 162 174 [--n N --d D --rounds R]   # on the GPU box
  python tools/syrk_ab.py check 162 174 --n 131071 --d 8192       # vs float64, poisoned workspace
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIBDIR = os.path.join(ROOT, "tools", "ab_libs")


def lib_path(v):
    return os.path.join(LIBDIR, f"libdeig_v{v}.so")


def build(variants):
    """Only syrk_split.hip differs between variants: compile it per variant (in
    parallel) and link it with the main build's other objects."""
    import subprocess

    from distributed_eigenspaces_amd import _build
    os.makedirs(LIBDIR, exist_ok=True)
    _build.build_library()  # the main objects are current
    objdir = os.path.join(_build.HERE, "build")
    hipcc = _build._hipcc()
    flags = [f"--offload-arch={_build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
             "-Wno-unused-function", "-Wno-inline-asm"] + _build.EXTRA_FLAGS["syrk_split.hip"]
    procs = []
    for v in variants:
        obj = os.path.join(LIBDIR, f"syrk_split_v{v}.o")
        cmd = [hipcc] + flags + [f"-DDEIG_AB_SYRK_VARIANT={v}", "-c",
                                 os.path.join(_build.CSRC, "syrk_split.hip"), "-o", obj]
        procs.append((v, obj, subprocess.Popen(cmd)))
    for v, obj, p in procs:
        if p.wait() != 0:
            raise RuntimeError(f"variant {v} failed to compile")
        others = [os.path.join(objdir, s.replace(".hip", ".o")) for s in _build.SOURCES
                  if s != "syrk_split.hip"]
        subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", lib_path(v),
                        obj] + others, check=True)
        os.remove(obj)
        print("built", lib_path(v), flush=True)


def run(variants, n, d, rounds, reps):
    import torch

    from distributed_eigenspaces_amd import _lib, synthetic
    dev = torch.device("cuda", 0)
    libs = {}
    for v in variants:
        L = ctypes.CDLL(lib_path(v))
        for name in ("deig_syrk_f32_ex", "deig_syrk_workspace_ex", "deig_last_error"):
            res, args = _lib.SIGNATURES[name]
            getattr(L, name).restype = res
            getattr(L, name).argtypes = args
        libs[v] = L
    U = synthetic.planted_basis(d, 64, seed=0, device=dev)
    X = synthetic.spiked_samples(n, U, seed=1)
    nbytes = max(L.deig_syrk_workspace_ex(n, d, _lib.DEIG_SYRK_SPLIT3) for L in libs.values())
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    S = {v: torch.empty((d, d), dtype=torch.float32, device=dev) for v in variants}
    st = torch.cuda.current_stream(dev)

    def launch(v):
        rc = libs[v].deig_syrk_f32_ex(X.data_ptr(), n, d, d, ctypes.c_float(1.0 / n), S[v].data_ptr(),
                                      d, _lib.DEIG_SYRK_SPLIT3, ws.data_ptr(), nbytes, st.cuda_stream)
        if rc:
            raise RuntimeError(f"v{v}: {libs[v].deig_last_error()}")

    for v in variants:  # warm-up (clock, caches)
        launch(v)
    torch.cuda.synchronize()
    times = {v: [] for v in variants}
    for r in range(rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(reps):
                launch(v)
            e1.record(st)
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / reps)
        print(f"round {r}: " + "  ".join(f"v{v} {times[v][-1]:.2f} ms" for v in variants), flush=True)
    flop = 3.0 * n * d * (d + 1)
    base = variants[0]
    for v in variants:
        med = statistics.median(times[v])
        diff = (S[v] - S[base]).abs().max().item() / S[base].abs().max().item()
        print(f"v{v}: median {med:.2f} ms min {min(times[v]):.2f} ms = "
              f"{flop / med / 1e9:.1f} TF/s bf16 ({flop / med / 1e9 / 2500:.3f} of 2.5 PF); "
              f"max|S - S_v{base}|/max|S| = {diff:.2e}; symmetric {bool(torch.equal(S[v], S[v].t()))}",
              flush=True)


def check(variants, n, d):
    """Each variant on a NaN-poisoned workspace (every byte 0xff) vs float64, at a
    ragged n: a variant that leaves any part of its image unwritten reads NaN."""
    import torch

    from distributed_eigenspaces_amd import _lib, synthetic
    dev = torch.device("cuda", 0)
    U = synthetic.planted_basis(d, 64, seed=0, device=dev)
    X = synthetic.spiked_samples(n, U, seed=1)
    Xd = X.double()
    ref = (Xd.t() @ Xd) / n
    del Xd
    scale = ref.abs().max().item()
    dref = torch.diagonal(ref)
    for v in variants:
        L = ctypes.CDLL(lib_path(v))
        for name in ("deig_syrk_f32_ex", "deig_syrk_workspace_ex", "deig_last_error"):
            res, args = _lib.SIGNATURES[name]
            getattr(L, name).restype = res
            getattr(L, name).argtypes = args
        nbytes = L.deig_syrk_workspace_ex(n, d, _lib.DEIG_SYRK_SPLIT3)
        ws = torch.full((nbytes,), 255, dtype=torch.uint8, device=dev)
        S = torch.full((d, d), float("nan"), dtype=torch.float32, device=dev)
        st = torch.cuda.current_stream(dev)
        for rep in range(2):
            rc = L.deig_syrk_f32_ex(X.data_ptr(), n, d, d, ctypes.c_float(1.0 / n), S.data_ptr(), d,
                                    _lib.DEIG_SYRK_SPLIT3, ws.data_ptr(), nbytes, st.cuda_stream)
            if rc:
                raise RuntimeError(f"v{v}: {L.deig_last_error()}")
            torch.cuda.synchronize()
            err = ((S.double() - ref).abs().max().item()) / scale
            derr = ((torch.diagonal(S).double() - dref).abs().max().item()) / scale
            print(f"check v{v} n={n} d={d} launch {rep}: max|S - S64|/max|S64| = {err:.3e} "
                  f"(diagonal {derr:.3e}); finite {bool(torch.isfinite(S).all())}; "
                  f"symmetric {bool(torch.equal(S, S.t()))}", flush=True)
        del ws, S


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run", "check"])
    ap.add_argument("variants", nargs="+", type=int)
    ap.add_argument("--n", type=int, default=1 << 21)
    ap.add_argument("--d", type=int, default=8192)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    if a.cmd == "build":
        build(a.variants)
    elif a.cmd == "check":
        check(a.variants, a.n, a.d)
    else:
        run(a.variants, a.n, a.d, a.rounds, a.reps)


if __name__ == "__main__":
    main()
