"""Quick kernel timing probe (HIP events on the launch stream)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import distributed_eigenspaces_amd as de
from distributed_eigenspaces_amd import synthetic

dev = torch.device("cuda", 0)
d = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
n = int(sys.argv[2]) if len(sys.argv) > 2 else (1 << 18)
k = int(sys.argv[3]) if len(sys.argv) > 3 else 64
U = synthetic.planted_basis(d, k, 0, dev)
t0 = time.time()
X = synthetic.spiked_samples(n, U, seed=1)
torch.cuda.synchronize(); print(f"gen {n}x{d}: {time.time()-t0:.2f}s", flush=True)
S = de.sigma_hat(X); torch.cuda.synchronize()
st = torch.cuda.current_stream()
for rep in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st); de.sigma_hat(X, out=S); e1.record(st); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    fl = n * d * (d + 1)
    print(f"syrk n={n} d={d}: {ms:.2f} ms  {fl/ms/1e9:.1f} TFLOP/s  ({fl/ms/1e9/157.3*100:.1f}% of 157.3)", flush=True)
for rep in range(2):
    t0 = time.time(); r = de.topk_eigh(S, k, check_finite=False); torch.cuda.synchronize()
    dt = time.time() - t0
    Uc = U.double(); Vc = r.V.double()
    s = torch.linalg.svdvals(Uc.t() @ Vc).min().item()
    print(f"topk d={d} k={k}: {dt*1e3:.1f} ms sweeps={r.sweeps} resid={r.resid:.2e} conv={r.converged} cos_min_vs_planted={s:.6f} evals[-3:]={r.evals[-3:].tolist()}", flush=True)
Wt = de.stack_bases([r.V] * 4)
t0 = time.time(); rs = de.projavg_topk(Wt, k, 0.25, q0=r.V); torch.cuda.synchronize()
print(f"projavg m=4: {(time.time()-t0)*1e3:.1f} ms sweeps={rs.sweeps} resid={rs.resid:.2e}", flush=True)
