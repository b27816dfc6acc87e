"""A/B timing of Oja builds in ONE process (interleaved rounds, same device, same
data).  Measurement tooling only: the variants are separate builds of libdeig.so
with -DDEIG_AB_OJA_VARIANT=N (oja.hip: knock-outs of the NN / TN passes and the
prefetch depth; the shipped library is variant 0).

  python tools/oja_ab.py build 0 1 2 4           # here (CPU): tools/ab_libs/libdeig_oja_v*.so
  python tools/oja_ab.py run 0 1 2 4 [--b B --d D --k K --nb NB --rounds R]   # GPU box
"""
import argparse
import ctypes
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIBDIR = os.path.join(ROOT, "tools", "ab_libs")


def lib_path(v):
    return os.path.join(LIBDIR, f"libdeig_oja_v{v}.so")


def build(variants):
    from distributed_eigenspaces_amd import _build
    os.makedirs(LIBDIR, exist_ok=True)
    _build.build_library()
    objdir = os.path.join(_build.HERE, "build")
    hipcc = _build._hipcc()
    flags = [f"--offload-arch={_build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
             "-Wno-unused-function", "-Wno-inline-asm"] + _build.EXTRA_FLAGS.get("oja.hip", [])
    procs = []
    for v in variants:
        obj = os.path.join(LIBDIR, f"oja_v{v}.o")
        cmd = [hipcc] + flags + [f"-DDEIG_AB_OJA_VARIANT={v}", "-c",
                                 os.path.join(_build.CSRC, "oja.hip"), "-o", obj]
        procs.append((v, obj, subprocess.Popen(cmd)))
    for v, obj, p in procs:
        if p.wait() != 0:
            raise RuntimeError(f"variant {v} failed to compile")
        others = [os.path.join(objdir, s.replace(".hip", ".o")) for s in _build.SOURCES
                  if s != "oja.hip"]
        subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", lib_path(v),
                        obj] + others, check=True)
        os.remove(obj)
        print("built", lib_path(v), flush=True)


def run(variants, b, d, k, nb, rounds, reps):
    import torch

    from distributed_eigenspaces_amd import _lib, synthetic
    dev = torch.device("cuda", 0)
    libs = {}
    for v in variants:
        L = ctypes.CDLL(lib_path(v))
        for name in ("deig_oja_steps_f32", "deig_oja_workspace", "deig_last_error"):
            res, args = _lib.SIGNATURES[name]
            getattr(L, name).restype = res
            getattr(L, name).argtypes = args
        libs[v] = L
    U = synthetic.planted_basis(d, k, seed=0, device=dev)
    X = synthetic.spiked_samples(nb * b, U, seed=1)
    V0 = torch.linalg.qr(torch.randn(d, k, device=dev, dtype=torch.float64))[0].float()
    nbytes = max(L.deig_oja_workspace(b, d, k) for L in libs.values())
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    V = {v: V0.t().contiguous().t() for v in variants}
    st = torch.cuda.current_stream(dev)

    def launch(v):
        V[v].copy_(V0)
        rc = libs[v].deig_oja_steps_f32(X.data_ptr(), nb, b, d, d, ctypes.c_float(0.3), V[v].data_ptr(),
                                        k, d, 8, ws.data_ptr(), nbytes, st.cuda_stream)
        if rc:
            raise RuntimeError(f"v{v}: {libs[v].deig_last_error()}")

    for v in variants:
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
            times[v].append(e0.elapsed_time(e1) * 1e3 / reps / nb)
        print(f"round {r}: " + "  ".join(f"v{v} {times[v][-1]:.2f}" for v in variants), flush=True)
    base = variants[0]
    algo = 8.0 * b * d
    for v in variants:
        med = statistics.median(times[v])
        diff = (V[v] - V[base]).abs().max().item()
        print(f"v{v}: median {med:.2f} us/batch (min {min(times[v]):.2f}) = "
              f"{algo / med / 1e3:.0f} GB/s algorithmic; max|V - V_v{base}| = {diff:.2e}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("variants", type=int, nargs="+")
    ap.add_argument("--b", type=int, default=4096)
    ap.add_argument("--d", type=int, default=3072)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--nb", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    if a.cmd == "build":
        build(a.variants)
    else:
        run(a.variants, a.b, a.d, a.k, a.nb, a.rounds, a.reps)


if __name__ == "__main__":
    main()
