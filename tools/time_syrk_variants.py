"""A/B the split3 SYRK ring shapes (DEIG_SYRK_VARIANT) in one process on the
config-3 shard; also checks every variant gives bit-identical Sigma_hat (same
accumulation order), a cheap race screen.

usage: python tools/time_syrk_variants.py [n] [d] [variants...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_eigenspaces_amd as de  # noqa: E402
from distributed_eigenspaces_amd import synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 21)
d = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
variants = [int(v) for v in sys.argv[3:]] or [22, 13, 14, 15]
dev = torch.device("cuda", 0)
U = synthetic.planted_basis(d, 64, 0, dev)
X = synthetic.spiked_samples(n, U, seed=1)
ref = None
for rep in range(2):
    for v in variants:
        os.environ["DEIG_SYRK_VARIANT"] = str(v)
        S = de.sigma_hat(X, algo="split3")
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            de.sigma_hat(X, out=S, algo="split3")
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        if ref is None:
            ref = S.clone()
        same = bool(torch.equal(S, ref))
        tf = 3 * n * d * (d + 1) / (min(ts) * 1e-3) / 1e12
        print(f"variant {v}: {min(ts):8.2f} ms (median {sorted(ts)[1]:8.2f})  {tf:7.1f} bf16-MFMA TF/s  "
              f"bit-identical={same}", flush=True)
