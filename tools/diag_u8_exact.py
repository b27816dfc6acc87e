"""Which side of an inexact u8 covariance comparison is off: the GPU image/direct
paths vs an exact int64 CPU product on a column subset (one rounding for /n)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import distributed_eigenspaces_amd as de

for n, d in [(65536, 2052), (65537, 2052), (200000, 256)]:
    rng = np.random.default_rng(n + d)
    Xh = rng.integers(0, 256, (n, d), dtype=np.uint8)
    Xh[:, 0] = 255
    Xh[:, 1] = 0
    Xh[::2, d - 1] = 255
    X = torch.from_numpy(Xh).cuda()
    S64 = de.linalg.sigma_hat_u8(X, dtype=torch.float64).cpu().numpy()
    Xf = X.double()
    ref_gpu = ((Xf.t() @ Xf) / n).cpu().numpy()
    cols = np.r_[0:48, d - 16:d]
    Xi = Xh[:, cols].astype(np.int64)
    exact = (Xi.T @ Xi).astype(np.float64) / n  # int64 sums < 2^53: one rounding
    sub = S64[np.ix_(cols, cols)]
    subg = ref_gpu[np.ix_(cols, cols)]
    print(f"n={n} d={d}: kernel vs exact-int64 diff entries {int((sub != exact).sum())}, "
          f"torch-f64 vs exact {int((subg != exact).sum())}, kernel vs torch full "
          f"{int((S64 != ref_gpu).sum())} (max rel {np.max(np.abs(S64 - ref_gpu) / np.abs(ref_gpu).clip(1e-30)):.2e})",
          flush=True)
