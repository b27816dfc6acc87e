"""Build an A/B variant of libdeig.so: the sources that test the given -D macro are
recompiled with it, the rest linked from the in-tree build (measurement tooling; the
shipped library has no knobs).

  python tools/ab_build.py DEIG_AB_SYRK_PIPE=1 tools/ab_libs/libdeig_pipe1.so
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(macro, out):
    from distributed_eigenspaces_amd import _build
    _build.build_library()
    objdir = os.path.join(_build.HERE, "build")
    hipcc = _build._hipcc()
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    objs = []
    for s in _build.SOURCES:
        src = os.path.join(_build.CSRC, s)
        if macro.split("=")[0] in open(src).read():
            obj = f"{out}.{s}.o"
            subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                            "-Wno-unused-function", "-Wno-inline-asm", f"-D{macro}", "-c", src, "-o", obj],
                           check=True)
            objs.append(obj)
        else:
            objs.append(os.path.join(objdir, s.replace(".hip", ".o")))
    subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", out] + objs, check=True)
    for o in objs:
        if o.startswith(out):
            os.remove(o)
    print("built", out)


if __name__ == "__main__":
    build(sys.argv[1], sys.argv[2])
