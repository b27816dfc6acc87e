"""Per-phase time of the small Rayleigh-Ritz solve (DEIG_DEBUG=1 trace: chol / linv /
congruence / jacobi / tail microseconds per RR step) for the shipped library and an
A/B build, on the c1 / c3 / c5 worker shapes and the k = 160 projector average of
tests/test_gpu_general_solver.py.  Measurement tooling: one child process per library
(DEIG_LIB_PATH), summaries per (case, library).

  python tools/rr_phases_ab.py [other.so]        # GPU box
"""
import os
import re
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys
sys.path.insert(0, os.environ["DEIG_ROOT"])
import numpy as np, torch
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
    print(f"=== {name} done sweeps {r.sweeps} resid {r.resid:.3e} conv {r.converged}", file=sys.stderr, flush=True)
    del S
    torch.cuda.empty_cache()
d, k, m = 1024, 160, 4
g = torch.Generator(device="cpu").manual_seed(3)
Q = torch.linalg.qr(torch.randn(d, k + 8, generator=g, dtype=torch.float64))[0]
common, shared, private = Q[:, :k - 8], Q[:, k - 8:k], Q[:, k:]
bases = []
for i in range(m):
    B = torch.cat([common, shared if i < 3 else private], dim=1)
    R = torch.linalg.qr(torch.randn(k, k, generator=g, dtype=torch.float64))[0]
    bases.append((B @ R).float().to(dev))
print("=== projavg160", file=sys.stderr, flush=True)
r = de.linalg.projavg_topk(de.linalg.stack_bases(bases), k, 1.0 / m)
print(f"=== projavg160 done sweeps {r.sweeps} resid {r.resid:.3e} conv {r.converged}", file=sys.stderr, flush=True)
'''


def run(lib):
    env = dict(os.environ, DEIG_DEBUG="1", DEIG_ROOT=ROOT)
    if lib:
        env["DEIG_LIB_PATH"] = lib
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
    case, out = None, {}
    for line in p.stderr.splitlines():
        m = re.match(r"=== (\S+)( done.*)?", line)
        if m:
            case = m.group(1)
            if m.group(2):
                out.setdefault(case, {})["result"] = m.group(2).strip()
            continue
        m = re.search(r"p=(\d+) sweep (\d+) resid (\S+).*jacobi_sweeps (\d+) rotations (\d+) small-solve us: "
                      r"chol (\S+) linv (\S+) congr (\S+) jacobi (\S+) tail (\S+)", line)
        if m and case:
            rec = out.setdefault(case, {}).setdefault("rr", [])
            rec.append([float(x) for x in m.groups()])
    if p.returncode:
        print(p.stderr[-3000:])
    return out


def main():
    libs = [None] + sys.argv[1:]
    for lib in libs:
        res = run(lib)
        print(f"##### {lib or 'shipped'}")
        for case, r in res.items():
            rr = r.get("rr", [])
            if not rr:
                print(case, r.get("result"))
                continue
            cols = list(zip(*rr))
            js = cols[3]
            print(f"{case:12s} p={int(cols[0][0])} RRs {len(rr)} {r.get('result', '')}")
            print(f"    median us: chol {statistics.median(cols[5]):.1f} linv {statistics.median(cols[6]):.1f} "
                  f"congr {statistics.median(cols[7]):.1f} jacobi {statistics.median(cols[8]):.1f} "
                  f"tail {statistics.median(cols[9]):.1f}; jacobi us per sweep "
                  f"{sum(cols[8]) / max(sum(js), 1):.1f} over {int(sum(js))} sweeps, rotations {int(sum(cols[4]))}")
            print("    resid trace:", " ".join(f"{x:.1e}" for x in cols[2]))


if __name__ == "__main__":
    main()
