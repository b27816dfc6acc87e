"""Interleaved A/B of the Oja paths at config 4 (64 batches of 4096 x 3072, k = 32,
orth_every 8): DEIG_OJA_RESIDENT vs DEIG_OJA_TWO_PASS, HIP events, plus their
subspace distance.  usage: python tools/oja_resident_ab.py [reps] [d] [k] [orth]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_eigenspaces_amd as de  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
d = int(sys.argv[2]) if len(sys.argv) > 2 else 3072
k = int(sys.argv[3]) if len(sys.argv) > 3 else 32
orth = int(sys.argv[4]) if len(sys.argv) > 4 else 8
b, nb = 4096, 64
dev = torch.device("cuda", 0)
X = torch.randn(nb * b, d, device=dev)
V0 = torch.linalg.qr(torch.randn(d, k, device=dev, dtype=torch.float64))[0].float()
res = {}
for algo in ("resident", "two_pass"):
    V = V0.t().contiguous().t()
    de.oja_steps(X, V, 0.02, b, orth_every=orth, algo=algo)
    res[algo] = V.double()
torch.cuda.synchronize()
Pa, Pb = res["resident"] @ res["resident"].t(), res["two_pass"] @ res["two_pass"].t()
print(f"projector distance resident vs two_pass: {torch.linalg.norm(Pa - Pb).item():.3e}")
times = {a: [] for a in res}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(reps):
    for algo in ("resident", "two_pass") if r % 2 == 0 else ("two_pass", "resident"):
        V = V0.t().contiguous().t()
        torch.cuda.synchronize()
        e0.record()
        de.oja_steps(X, V, 0.02, b, orth_every=orth, algo=algo)
        e1.record()
        e1.synchronize()
        times[algo].append(e0.elapsed_time(e1) / nb * 1e3)
for algo, ts in times.items():
    ts = sorted(ts)
    us = ts[len(ts) // 2]
    print(f"{algo}: median {us:.2f} us/batch (min {ts[0]:.2f}) = "
          f"{8.0 * b * d / us / 1e3:.0f} GB/s algorithmic (8 b d bytes), {[round(t, 2) for t in times[algo]]}")
