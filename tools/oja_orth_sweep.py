"""Config 4's re-orthonormalisation interval: for orth_every in {8, 16, 32, 64} run the
64 Oja batches of one aggregation span (4096 x 3072, k = 32, eta = 0.02) through
linalg.oja_steps and report the projector distance to ref_cpu.oja_epoch (float64,
orthonormalised after every batch), ||V^T V - I|| and the time per batch (HIP events).
usage: python tools/oja_orth_sweep.py [nb]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import distributed_eigenspaces_amd as de  # noqa: E402
from distributed_eigenspaces_amd import synthetic  # noqa: E402
from oracle import ref_cpu  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 64
b, d, k, eta = 4096, 3072, 32, 0.02
dev = torch.device("cuda", 0)
U = synthetic.planted_basis(d, k, seed=0, device=dev)
X = synthetic.spiked_samples(nb * b, U, seed=3)
g = torch.Generator(device="cpu").manual_seed(5)
V0 = torch.linalg.qr(torch.randn(d, k, generator=g, dtype=torch.float64))[0]
Vr = ref_cpu.oja_epoch(X.double().cpu().numpy(), V0.numpy(), eta, b)
for orth in (8, 16, 32, 64):
    V = V0.float().to(dev).t().contiguous().t()
    de.oja_steps(X, V, eta, b, orth_every=orth)
    Vg = V.cpu().double().numpy()
    pd = ref_cpu.projector_distance(Vg, Vr)
    on = np.abs(Vg.T @ Vg - np.eye(k)).max()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = []
    for _ in range(5):
        V = V0.float().to(dev).t().contiguous().t()
        e0.record()
        de.oja_steps(X, V, eta, b, orth_every=orth)
        e1.record()
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    print(f"orth_every {orth:3d}: ||P - P_oracle||_F {pd:.2e}  max|V^T V - I| {on:.1e}  "
          f"{1e3 * np.median(ms) / nb:.2f} us per batch (median of 5, {nb} batches)", flush=True)
