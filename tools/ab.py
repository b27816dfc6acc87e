"""One A/B harness for libdeig measurement builds (measurement tooling: the shipped
library reads no environment and has no knobs; variants differ only by -D macros the
sources test, e.g. DEIG_AB_OJA_LATE_TRANSPOSE, DEIG_AB_SYRK_VARIANT, DEIG_AB_SWEEP_DEPTH).

Builds are interleaved in ONE process on the same inputs (the same binary runs 3-4 %
apart across boxes, so only interleaved runs compare), each reporting its median time
and whether it reproduces the first build's output bit for bit.  LIB "shipped" is the
in-tree distributed_eigenspaces_amd/libdeig.so.

  python tools/ab.py build "MACRO=V [-DOTHER=W]" tools/ab_libs/libdeig_x.so   # here (CPU)
  python tools/ab.py syrk  REPS N D LIB [LIB ...]          # split3 covariance, ms per op
  python tools/ab.py sweep REPS D P MODE LIB [LIB ...]     # solver sweep chain, us per sweep
                                                           # MODE half | bf16x3 | bf16x5 | bf16x6
  python tools/ab.py oja   REPS ORTH LIB [LIB ...]         # config-4 Oja, us per batch
  python tools/ab.py rr    [LIB ...]                       # RR small-solve phases (DEIG_DEBUG)
  python tools/ab.py tests TAG LIB [LIB ...] [-- PYTEST ARGS]   # GPU suite per build
"""
import ctypes
import os
import re
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


# ---------------------------------------------------------------- build
def build(macros, out):
    """Recompile the sources that test any of the given macros with them, link the
    rest from the in-tree build."""
    from distributed_eigenspaces_amd import _build
    _build.build_library()
    objdir = os.path.join(_build.HERE, "build")
    hipcc = _build._hipcc()
    defs = ["-D" + (m[2:] if m.startswith("-D") else m) for m in macros.split()]
    names = [d[2:].split("=")[0] for d in defs]
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    objs = []
    for s in _build.SOURCES:
        src = os.path.join(_build.CSRC, s)
        text = open(src).read()
        if any(n in text for n in names):
            obj = f"{out}.{s}.o"
            subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                            "-Wno-unused-function", "-Wno-inline-asm"] + defs +
                           _build.EXTRA_FLAGS.get(s, []) + ["-c", src, "-o", obj], check=True)
            objs.append(obj)
        else:
            objs.append(os.path.join(objdir, s.replace(".hip", ".o")))
    subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", out] + objs, check=True)
    for o in objs:
        if o.startswith(out):
            os.remove(o)
    print("built", out)


# ---------------------------------------------------------------- helpers
def load_libs(paths):
    from distributed_eigenspaces_amd import _lib
    libs = []
    for path in paths:
        L = ctypes.CDLL(_lib.LIB_PATH if path == "shipped" else path)
        for name, (res, args) in _lib.SIGNATURES.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        libs.append((path, L))
    return libs


def interleave(libs, reps, run):
    """run(path, L) -> (time, output); rounds alternate the build order."""
    times = {p: [] for p, _ in libs}
    outs = {}
    for r in range(reps + 1):
        for path, L in (libs if r % 2 == 0 else libs[::-1]):
            t, out = run(path, L)
            if r:
                times[path].append(t)
            outs[path] = out
    return times, outs


def report(times, same, unit, extra=lambda p, med: ""):
    for path, ts in times.items():
        st = sorted(ts)
        med = st[len(st) // 2]
        print(f"{path}: median {med:.2f} {unit} (min {st[0]:.2f}){extra(path, med)}; bit-identical to "
              f"first: {same(path)} {[round(t, 2) for t in ts]}", flush=True)


# ---------------------------------------------------------------- syrk
def ab_syrk(reps, n, d, paths):
    import torch
    from distributed_eigenspaces_amd import synthetic
    libs = load_libs(paths)
    dev = torch.device("cuda", 0)
    U = synthetic.planted_basis(d, 64, 0, dev)
    X = synthetic.spiked_samples(n, U, seed=1)
    nbytes = max(L.deig_syrk_workspace_ex(n, d, 1) for _, L in libs)
    ws = torch.empty(nbytes // 4 + 64, dtype=torch.float32, device=dev)
    S = {p: torch.empty(d, d, device=dev) for p, _ in libs}
    st = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run(path, L):
        torch.cuda.synchronize()
        e0.record(st)
        rc = L.deig_syrk_f32_ex(X.data_ptr(), n, d, X.stride(0), ctypes.c_float(1.0 / n),
                                S[path].data_ptr(), d, 1, ws.data_ptr(), nbytes, st.cuda_stream)
        e1.record(st)
        e1.synchronize()
        assert rc == 0, L.deig_last_error()
        return e0.elapsed_time(e1), S[path]

    times, outs = interleave(libs, reps, run)
    ref = outs[libs[0][0]]
    # float64 reference of 64 sampled columns of X^T X / n (chunked over the rows)
    cols = torch.randperm(d, generator=torch.Generator().manual_seed(3))[:64].to(dev)
    S64 = torch.zeros(d, 64, dtype=torch.float64, device=dev)
    for r0 in range(0, n, 1 << 17):
        Xc = X[r0:r0 + (1 << 17)].double()
        S64 += Xc.t() @ Xc[:, cols]
        del Xc
    S64 /= n
    scale = S64.abs().max().item()
    flop = 3.0 * n * d * (d + 1)
    report(times, lambda p: torch.equal(outs[p], ref), "ms",
           lambda p, med: f" = {flop / med / 1e9 / 2.5e3:.4f} of bf16 peak, max|S - S_f64| / max|S| on 64 "
                          f"columns {((outs[p][:, cols].double() - S64).abs().max().item()) / scale:.2e}")


# ---------------------------------------------------------------- sweep
def ab_sweep(reps, d, p, mode, paths):
    import torch
    from distributed_eigenspaces_amd import _lib
    libs = load_libs(paths)
    code = _lib.DEIG_SWEEP_BF16X6
    if mode != "bf16x6":
        code |= _lib.DEIG_SWEEP_ROUND_Q
    if mode in ("bf16x3", "half"):
        code |= _lib.DEIG_SWEEP_FAST
    if mode == "half":
        code |= _lib.DEIG_SWEEP_HALF
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    g = torch.Generator(device=dev).manual_seed(5)
    A = torch.randn((d, d), generator=g, device=dev)
    S = (A + A.t()) * (0.5 / d ** 0.5)
    del A
    Q0 = torch.randn((d, p), generator=g, device=dev)
    cs = torch.full((p,), 0.5, device=dev)
    steps = 20
    state = {}
    for path, L in libs:
        nbytes = L.deig_sym_apply_workspace(d, p, code)
        ws = torch.empty(nbytes // 4 + 64, dtype=torch.float32, device=dev)
        Q = Q0.clone()
        Y = torch.empty((d, p), device=dev)
        rc = L.deig_sym_apply_f32(S.data_ptr(), d, d, Q.data_ptr(), p, p, Y.data_ptr(), p,
                                  ctypes.c_float(1.0), code, ws.data_ptr(), nbytes, st.cuda_stream)
        assert rc == 0, L.deig_last_error()
        state[path] = (ws, nbytes, Y)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run(path, L):
        ws, nbytes, Y = state[path]
        Q = Q0.clone()
        torch.cuda.synchronize()
        e0.record(st)
        rc = L.deig_sym_power_f32(S.data_ptr(), d, d, Q.data_ptr(), p, p, Y.data_ptr(), p, cs.data_ptr(),
                                  steps, code | _lib.DEIG_SWEEP_PREPARED, ws.data_ptr(), nbytes,
                                  st.cuda_stream)
        e1.record(st)
        e1.synchronize()
        assert rc == 0, L.deig_last_error()
        return e0.elapsed_time(e1) / steps * 1e3, (Y.clone(), Q)

    times, outs = interleave(libs, reps, run)
    ref = outs[libs[0][0]]
    report(times, lambda q: torch.equal(outs[q][0], ref[0]) and torch.equal(outs[q][1], ref[1]),
           f"us/sweep (d={d} p={p} {mode})",
           lambda q, med: f" = {4.0 * d * d / med / 1e3 / 8000:.3f} of 8 TB/s")


# ---------------------------------------------------------------- oja
def ab_oja(reps, orth, paths):
    import torch
    libs = load_libs(paths)
    b, d, k, nb = 4096, 3072, 32, 64
    dev = torch.device("cuda", 0)
    X = torch.randn(nb * b, d, device=dev)
    V0 = torch.linalg.qr(torch.randn(d, k, device=dev, dtype=torch.float64))[0].float()
    nbytes = max(L.deig_oja_workspace(b, d, k) for _, L in libs)
    ws = torch.zeros(nbytes // 4 + 64, dtype=torch.float32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run(path, L):
        V = V0.t().contiguous().t()
        torch.cuda.synchronize()
        e0.record()
        rc = L.deig_oja_steps_f32(X.data_ptr(), nb, b, d, X.stride(0), ctypes.c_float(0.02), V.data_ptr(),
                                  k, V.stride(1), orth, ws.data_ptr(), nbytes, None)
        e1.record()
        e1.synchronize()
        assert rc == 0
        return e0.elapsed_time(e1) / nb * 1e3, V

    times, outs = interleave(libs, reps, run)
    ref = outs[libs[0][0]]
    report(times, lambda p: torch.equal(outs[p], ref) and bool(torch.isfinite(outs[p]).all()),
           "us/batch (config 4: 64 x 4096 x 3072, k = 32)")


# ---------------------------------------------------------------- rr phases
RR_CHILD = r'''
import hashlib, os, sys
sys.path.insert(0, os.environ["DEIG_ROOT"])
import torch
import distributed_eigenspaces_amd as de
from distributed_eigenspaces_amd import synthetic
dev = torch.device("cuda", 0)
for name, n, d, k in (("c1", 6250, 3072, 10), ("c3", 16384, 8192, 64), ("c5", 32768, 16384, 128)):
    U = synthetic.planted_basis(d, k, seed=0, device=dev)
    X = synthetic.spiked_samples(n, U, seed=1)
    S = de.sigma_hat(X); del X
    torch.cuda.synchronize()
    print(f"=== {name}", file=sys.stderr, flush=True)
    r = de.topk_eigh(S, k, check_finite=False)
    torch.cuda.synchronize()
    h = hashlib.sha1(r.V.cpu().numpy().tobytes() + r.evals.cpu().numpy().tobytes()).hexdigest()[:12]
    print(f"=== {name} done sweeps {r.sweeps} resid {r.resid:.3e} conv {r.converged} out {h}", file=sys.stderr,
          flush=True)
    del S
    torch.cuda.empty_cache()
'''


def ab_rr(paths):
    """Per-phase time of the one-workgroup Rayleigh-Ritz solve (DEIG_DEBUG=1 trace) on the
    c1 / c3 / c5 worker shapes, one child process per build (DEIG_LIB_PATH)."""
    for lib in [None] + list(paths):
        env = dict(os.environ, DEIG_DEBUG="1", DEIG_ROOT=ROOT)
        if lib and lib != "shipped":
            env["DEIG_LIB_PATH"] = lib
        p = subprocess.run([sys.executable, "-c", RR_CHILD], env=env, capture_output=True, text=True,
                           timeout=600)
        case, res = None, {}
        for line in p.stderr.splitlines():
            m = re.match(r"=== (\S+)( done.*)?", line)
            if m:
                case = m.group(1)
                if m.group(2):
                    res.setdefault(case, {})["result"] = m.group(2).strip()
                continue
            m = re.search(r"p=(\d+) sweep (\d+) resid (\S+).*jacobi_sweeps (\d+) rotations (\d+) small-solve us: "
                          r"chol (\S+) linv (\S+) congr (\S+) jacobi (\S+) tail (\S+)", line)
            if m and case:
                res.setdefault(case, {}).setdefault("rr", []).append([float(x) for x in m.groups()])
        if p.returncode:
            print(p.stderr[-3000:])
        print(f"##### {lib or 'shipped'}")
        for c, r in res.items():
            rr = r.get("rr", [])
            if not rr:
                print(c, r.get("result"))
                continue
            cols = list(zip(*rr))
            print(f"{c:6s} p={int(cols[0][0])} RRs {len(rr)} {r.get('result', '')}; median us: chol "
                  f"{statistics.median(cols[5]):.1f} linv {statistics.median(cols[6]):.1f} congr "
                  f"{statistics.median(cols[7]):.1f} jacobi {statistics.median(cols[8]):.1f} tail "
                  f"{statistics.median(cols[9]):.1f}; jacobi us per sweep "
                  f"{sum(cols[8]) / max(sum(cols[3]), 1):.1f} over {int(sum(cols[3]))} sweeps")


# ---------------------------------------------------------------- tests
def ab_tests(tag, args):
    """The GPU suite against each build (DEIG_LIB_PATH), one pytest process per build,
    time-limited; stops at the first failing build."""
    if "--" in args:
        i = args.index("--")
        libs, extra = args[:i], args[i + 1:]
    else:
        libs, extra = args, []
    out = os.path.join(ROOT, "gpurun_out", tag)
    os.makedirs(out, exist_ok=True)
    for lib in libs:
        env = dict(os.environ)
        if lib != "shipped":
            env["DEIG_LIB_PATH"] = os.path.abspath(lib)
        log = os.path.join(out, os.path.basename(lib) + ".log")
        with open(log, "w") as f:
            rc = subprocess.run(["timeout", "-k", "10", "1000", sys.executable, "-u", "-m", "pytest", "-m", "gpu",
                                 "-q", "--timeout", "300", "--timeout-method", "thread"] + extra,
                                cwd=ROOT, env=env, stdout=f, stderr=subprocess.STDOUT).returncode
        print(lib, "rc", rc, open(log).read().splitlines()[-1] if os.path.getsize(log) else "")
        if rc:
            sys.exit(rc)


def main(argv):
    cmd, a = argv[0], argv[1:]
    if cmd == "build":
        build(a[0], a[1])
    elif cmd == "syrk":
        ab_syrk(int(a[0]), int(a[1]), int(a[2]), a[3:])
    elif cmd == "sweep":
        ab_sweep(int(a[0]), int(a[1]), int(a[2]), a[3], a[4:])
    elif cmd == "oja":
        ab_oja(int(a[0]), int(a[1]), a[2:])
    elif cmd == "rr":
        ab_rr(a)
    elif cmd == "tests":
        ab_tests(a[0], a[1:])
    else:
        raise SystemExit(__doc__)


if __name__ == "__main__":
    main(sys.argv[1:])
