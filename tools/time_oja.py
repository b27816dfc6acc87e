"""Time the Oja batch kernels: oja_steps over 64 batches of 4096 x 3072, k = 32
(config 4), HIP events; orth_every = 64 so the batch kernels dominate.
usage: python tools/time_oja.py [b d k nb]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_eigenspaces_amd as de  # noqa: E402

b, d, k, nb = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (4096, 3072, 32, 64)))
dev = torch.device("cuda", 0)
X = torch.randn(nb * b, d, device=dev)
V0 = torch.linalg.qr(torch.randn(d, k, device=dev, dtype=torch.float64))[0].float()
V = V0.t().contiguous().t()
for _ in range(2):
    de.oja_steps(X, V, 0.02, b, orth_every=nb)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 5
e0.record()
for _ in range(reps):
    de.oja_steps(X, V, 0.02, b, orth_every=nb)
e1.record()
e1.synchronize()
us = e0.elapsed_time(e1) / reps / nb * 1e3
print(f"probe={os.environ.get('DEIG_OJA_PROBE', '0')} slices={os.environ.get('DEIG_OJA_TN_SLICES', 'auto')} "
      f"kernel={os.environ.get('DEIG_OJA_KERNEL', '2')}: {us:.2f} us/batch = {8.0 * b * d / us / 1e6:.0f} GB/s")
