"""A/B of tools/u8_lds_mirror.patch (the uint8 SYRK's direct epilogue with the mirror
store S[j][i] routed through an LDS transpose, float4 rows) against the shipped
direct epilogue, in ONE process on the c1 worker shard (6250 x 3072 bytes); both
must give the same bits.  Measurement tooling only.

  python tools/u8_mirror_ab.py build    # here: tools/ab_libs/libdeig_u8mirror.so
  python tools/u8_mirror_ab.py run      # GPU box
"""
import ctypes
import os
import shutil
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIBDIR = os.path.join(ROOT, "tools", "ab_libs")
PATCHED = os.path.join(LIBDIR, "libdeig_u8mirror.so")


def build():
    from distributed_eigenspaces_amd import _build
    os.makedirs(LIBDIR, exist_ok=True)
    _build.build_library()
    # patch a copy next to the sources (its includes are relative), compile, remove
    src = os.path.join(_build.CSRC, "_ab_syrk_u8_mirror.hip")
    shutil.copy(os.path.join(_build.CSRC, "syrk_u8.hip"), src)
    try:
        subprocess.run(["patch", "-s", src, os.path.join(ROOT, "tools", "u8_lds_mirror.patch")], check=True)
        hipcc = _build._hipcc()
        obj = os.path.join(LIBDIR, "syrk_u8_mirror.o")
        subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                        "-Wno-unused-function", "-Wno-inline-asm", "-c", src, "-o", obj], check=True)
    finally:
        os.remove(src)
    objdir = os.path.join(_build.HERE, "build")
    others = [os.path.join(objdir, s.replace(".hip", ".o")) for s in _build.SOURCES if s != "syrk_u8.hip"]
    subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", PATCHED, obj] + others,
                   check=True)
    os.remove(obj)
    print("built", PATCHED)


def run(rounds=5, reps=20):
    import torch

    from distributed_eigenspaces_amd import _lib
    dev = torch.device("cuda", 0)
    libs = {}
    for tag, path in (("shipped", _lib.LIB_PATH), ("mirror", PATCHED)):
        L = ctypes.CDLL(path)
        for name, (res, args) in _lib.SIGNATURES.items():
            getattr(L, name).restype = res
            getattr(L, name).argtypes = args
        libs[tag] = L
    n, d = 6250, 3072
    g = torch.Generator(device="cpu").manual_seed(3)
    X = torch.randint(0, 256, (n, d), generator=g, dtype=torch.uint8).to(dev)
    st = torch.cuda.current_stream().cuda_stream
    outs, times = {}, {t: [] for t in libs}
    for rnd in range(rounds):
        for tag, L in libs.items():
            S = torch.empty((d, d), dtype=torch.float32, device=dev)
            nb = L.deig_syrk_u8_workspace(n, d, 0)
            ws = torch.empty(nb, dtype=torch.uint8, device=dev)
            call = lambda: L.deig_syrk_u8(X.data_ptr(), n, d, d, 0, ctypes.c_double(1.0 / n), S.data_ptr(), d,
                                          None, d, ws.data_ptr(), nb, st)
            assert call() == 0, _lib.last_error()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                call()
            e1.record()
            e1.synchronize()
            times[tag].append(e0.elapsed_time(e1) / reps * 1e3)
            outs[tag] = S
    same = bool(torch.equal(outs["shipped"], outs["mirror"]))
    for tag in libs:
        print(f"{tag}: median {statistics.median(times[tag]):.1f} us per covariance (c1 worker shard), "
              f"rounds {[round(t, 1) for t in times[tag]]}")
    print("bit-identical:", same)


if __name__ == "__main__":
    build() if sys.argv[1:] == ["build"] else run()
