"""Phase timing of the one-workgroup Rayleigh-Ritz kernel (DEIG_DEBUG=1 prints
chol / linv / congruence / jacobi / tail microseconds per RR step) on the c1
worker shape (6250 x 3072 bytes, k = 10), the c2 shape (k = 16) and, with "big" as
the first argument, the c3 (d = 8192, k = 64) and c5 (d = 16384, k = 128) widths."""
import os
import sys

os.environ["DEIG_DEBUG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_eigenspaces_amd as de  # noqa: E402
from distributed_eigenspaces_amd import synthetic  # noqa: E402

dev = torch.device("cuda", 0)
shapes = (("c1", 6250, 3072, 10, True), ("c2", 1 << 16, 3072, 16, False))
if len(sys.argv) > 1 and sys.argv[1] == "big":
    shapes = (("c3", 1 << 16, 8192, 64, False), ("c5", 1 << 16, 16384, 128, False))
for name, n, d, k, u8 in shapes:
    U = synthetic.planted_basis(d, k, seed=0, device=dev)
    X = synthetic.spiked_bytes(n, U, seed=1) if u8 else synthetic.spiked_samples(n, U, seed=1)
    S = de.sigma_hat(X)
    torch.cuda.synchronize()
    print(f"=== {name}", file=sys.stderr, flush=True)
    r = de.topk_eigh(S, k)
    print(f"=== {name} sweeps {r.sweeps} resid {r.resid:.2e}", file=sys.stderr, flush=True)
