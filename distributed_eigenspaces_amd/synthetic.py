"""Synthetic spiked-covariance data, generated on the GPU.

Sigma = I_d + U diag(theta) U^T with U (d x k) orthonormal from a seed and
theta_j linearly spaced theta_hi -> theta_lo.  Rows are x = g + U (h * sqrt(theta))
with g ~ N(0, I_d), h ~ N(0, I_k), so E[x x^T] = Sigma and the top-k eigenvectors
of the (uncentered) second moment are U, eigenvalues 1 + theta.

Used by bench.py and the GPU tests (the CIFAR files are not shipped with the
reference).  Generation is chunked so 64 GiB shards fit beside their output.
"""
from __future__ import annotations

import numpy as np
import torch

__all__ = ["planted_basis", "spiked_theta", "spiked_samples"]


def planted_basis(d: int, k: int, seed: int = 0, device=None) -> torch.Tensor:
    g = torch.Generator(device="cpu").manual_seed(int(seed))
    A = torch.randn(d, k, generator=g, dtype=torch.float64)
    U, _ = torch.linalg.qr(A)
    return U.to(dtype=torch.float32, device=device)


def spiked_theta(k: int, theta_hi: float = 8.0, theta_lo: float = 4.0) -> np.ndarray:
    return np.linspace(theta_hi, theta_lo, k)


def spiked_samples(n: int, U: torch.Tensor, seed: int = 1, theta_hi: float = 8.0,
                   theta_lo: float = 4.0, out: torch.Tensor | None = None,
                   chunk_rows: int = 1 << 18) -> torch.Tensor:
    """n spiked rows on U's device (float32, row-major)."""
    d, k = U.shape
    dev = U.device
    X = out if out is not None else torch.empty((n, d), dtype=torch.float32, device=dev)
    sq = torch.from_numpy(np.sqrt(spiked_theta(k, theta_hi, theta_lo))).to(dev, torch.float32)
    Ut = (U * sq[None, :]).t().contiguous()  # k x d
    gen = torch.Generator(device=dev)
    for c, lo in enumerate(range(0, n, chunk_rows)):
        hi = min(n, lo + chunk_rows)
        gen.manual_seed(int(seed) * 1_000_003 + c)
        blk = X[lo:hi]
        torch.randn(blk.shape, generator=gen, device=dev, dtype=torch.float32, out=blk)
        h = torch.randn((hi - lo, k), generator=gen, device=dev, dtype=torch.float32)
        blk.addmm_(h, Ut)
    return X
