"""Eigensolver diagnostics on the golden shards (prints sweeps / residual / distance)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, warnings
warnings.simplefilter("ignore")
import distributed_eigenspaces_amd as de
from oracle import ref_cpu
from tests.conftest import load_golden, golden_names
dev = torch.device("cuda", 0)
for name in golden_names():
    g = load_golden(name); X32 = g["X"].astype(np.float32); k = int(g["k"])
    for i, (lo, hi) in enumerate(g["ranges"]):
        S = de.sigma_hat(torch.from_numpy(X32[lo:hi]).to(dev))
        Sr = ref_cpu.sigma_hat(X32[lo:hi].astype(np.float64))
        serr = np.abs(S.cpu().numpy() - Sr).max() / np.abs(Sr).max()
        for tol, ms, p in [(1e-6, 300, None), (1e-9, 60, None), (1e-9, 300, 32)]:
            r = de.topk_eigh(S, k, tol=tol, max_sweeps=ms, p=p)
            dist = ref_cpu.projector_distance(r.V.cpu().numpy(), g["worker_V"][i])
            evr = np.max(np.abs(r.evals.cpu().numpy() - g["worker_evals"][i]) / np.abs(g["worker_evals"][i]))
            print(f"{name} shard {i} serr={serr:.1e} tol={tol} ms={ms} p={p}: sweeps={r.sweeps} resid={r.resid:.2e} conv={r.converged} dist={dist:.2e} ev={evr:.1e}", flush=True)
