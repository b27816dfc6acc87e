"""Wall time of the spiked d = 3072, k = 16 solve of tests/test_gpu_solver_robust.py::test_chebyshev_keeps_spiked_sweep_counts under three Chebyshev thresholds (measurement tooling)."""
import sys, time, statistics, json
sys.path.insert(0, '.')
import numpy as np, torch
import distributed_eigenspaces_amd as de
from distributed_eigenspaces_amd import _lib
from tests.test_gpu_solver_robust import _matrix
dev = torch.device('cuda', 0)
rng = np.random.default_rng(2)
d, k = 3072, 16
lams = np.concatenate([np.linspace(9, 5, k), np.sort(rng.uniform(0.7, 1.4, d - k))[::-1]])
S = torch.from_numpy(_matrix(lams, seed=7)).to(dev)
for ca in (0.01, 0.1, 0.5):
    o = _lib.solver_opts(cheb_above=ca)
    ts = []
    for _ in range(7):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        r = de.topk_eigh(S, k, opts=o); torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"cheb_above": ca, "ms": statistics.median(ts), "sweeps": r.sweeps, "resid": r.resid}))
