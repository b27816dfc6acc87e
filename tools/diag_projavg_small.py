"""Debug probe: projavg_topk on a few small stacks (rank-deficient operator: mk < p)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, warnings
import distributed_eigenspaces_amd as de
dev = torch.device("cuda", 0)
for d, k, m in [(256, 6, 1), (256, 6, 2), (256, 6, 3), (512, 10, 2)]:
    rng = np.random.default_rng(0)
    U = np.linalg.qr(rng.standard_normal((d, k)))[0]
    Vs = [np.linalg.qr(U + 0.05 * rng.standard_normal((d, k)))[0] for _ in range(m)]
    Wt = de.stack_bases([torch.from_numpy(v).float().to(dev) for v in Vs])
    with warnings.catch_warnings(record=True):
        try:
            r = de.projavg_topk(Wt, k, 1.0 / m, q0=torch.from_numpy(Vs[0]).float().to(dev))
            print(d, k, m, "ok", r.sweeps, r.resid, r.evals.cpu().numpy(), flush=True)
        except Exception as e:
            print(d, k, m, "ERR", e, flush=True)
