"""Debug probe: the world-2 streaming-Oja aggregation, in one process."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import distributed_eigenspaces_amd as de
from tests.test_gpu_distributed import _oja_data
world, nb, b, d, k, agg = 2, 6, 1024, 256, 6, 3
batches, V0 = _oja_data(world, nb, b, d, k)
Vs = []
for r in range(world):
    V = torch.from_numpy(V0).float().cuda().t().contiguous().t()
    X = torch.from_numpy(np.concatenate(batches[r][:agg])).cuda()
    de.oja_steps(X, V, 0.3, b, 8)
    print("rank", r, "finite", bool(torch.isfinite(V).all()), "VtV", (V.t() @ V).diagonal().cpu().numpy(), flush=True)
    Vs.append(V)
Wt = de.stack_bases(Vs)
print("Wt finite", bool(torch.isfinite(Wt).all()), Wt.shape, flush=True)
for q0 in (Vs[0], None):
    try:
        r = de.projavg_topk(Wt, k, 1.0 / world, q0=q0)
        print("ok", r.sweeps, r.resid, r.evals.cpu().numpy(), flush=True)
    except Exception as e:
        print("ERR", e, flush=True)
