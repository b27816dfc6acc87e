"""DEIG_DEBUG trace of the k = 160 projector average of tests/test_gpu_general_solver.py
(test_projector_average_k_above_128) for the shipped library and an A/B build: every
RR line (residual, Chebyshev degree, Jacobi sweeps / rotations, phase times).

  python tools/diag_projavg160.py [other.so ...]     # GPU box
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys
sys.path.insert(0, os.environ["DEIG_ROOT"])
import torch
import distributed_eigenspaces_amd as de
dev = torch.device("cuda", 0)
d, k, m = 1024, 160, 4
g = torch.Generator(device="cpu").manual_seed(3)
Q = torch.linalg.qr(torch.randn(d, k + 8, generator=g, dtype=torch.float64))[0]
common, shared, private = Q[:, :k - 8], Q[:, k - 8:k], Q[:, k:]
bases = []
for i in range(m):
    B = torch.cat([common, shared if i < 3 else private], dim=1)
    R = torch.linalg.qr(torch.randn(k, k, generator=g, dtype=torch.float64))[0]
    bases.append((B @ R).float().to(dev))
r = de.linalg.projavg_topk(de.linalg.stack_bases(bases), k, 1.0 / m)
print(f"=== done sweeps {r.sweeps} resid {r.resid:.3e} conv {r.converged}", file=sys.stderr, flush=True)
'''


def main():
    for lib in [None] + sys.argv[1:]:
        env = dict(os.environ, DEIG_DEBUG="1", DEIG_ROOT=ROOT)
        if lib:
            env["DEIG_LIB_PATH"] = lib
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        print(f"##### {lib or 'shipped'} rc {p.returncode}")
        for line in p.stderr.splitlines():
            if line.startswith("[deig]") or line.startswith("==="):
                print(line)


if __name__ == "__main__":
    main()
