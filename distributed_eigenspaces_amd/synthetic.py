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

__all__ = ["planted_basis", "spiked_theta", "spiked_samples", "spiked_bytes"]


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


def spiked_bytes(n: int, U: torch.Tensor, seed: int = 1, scale: float = 20.0,
                 channels: int = 0) -> torch.Tensor:
    """CIFAR-like uint8 samples on U's device: clip(round(128 + scale * x)) of
    spiked_samples rows x (CIFAR is not shipped with the reference).

    channels = 0: (n, d) raw bytes.  channels = 3: (n, H, W, 3) interleaved pixels
    (load_data.py:18-33 layout, H = W = sqrt(d)) whose channel c is x plus
    independent N(0, 1/4) noise, so the reference's grayscale (distributed.py:171)
    keeps U as the planted subspace.  The uncentered covariance of such bytes has
    the mean direction as its dominant eigenvector, as CIFAR's does."""
    d = U.shape[0]
    xf = spiked_samples(n, U, seed)
    if not channels:
        return xf.mul_(scale).add_(128.0).round_().clamp_(0, 255).to(torch.uint8)
    side = int(round(d ** 0.5))
    if side * side != d:
        raise ValueError(f"spiked_bytes: d = {d} is not a square image")
    out = torch.empty((n, d, channels), dtype=torch.uint8, device=U.device)
    gen = torch.Generator(device=U.device).manual_seed(int(seed) * 7919 + 17)
    for c in range(channels):
        noise = torch.randn((n, d), generator=gen, device=U.device, dtype=torch.float32)
        out[:, :, c] = noise.mul_(0.5).add_(xf).mul_(scale).add_(128.0).round_().clamp_(0, 255)
    return out.view(n, side, side, channels)
