"""Inputs of the golden fixtures (test infrastructure): the spiked-covariance
generator both tests/golden/gen_golden.py (which runs the reference on it) and the
tests (which regenerate the inputs of seeded fixtures too large to store) use."""
import hashlib

import numpy as np


def spiked_int_data(n, d, k, seed, theta_hi=8.0, theta_lo=4.0, grid=8):
    """Spiked-covariance rows X = G + H diag(sqrt(theta)) U^T rounded to 1/grid.

    Values are exactly representable in fp32 (and in int16 after * grid) so the
    same numbers feed the float64 reference and the fp32 GPU path.
    """
    rng = np.random.default_rng(seed)
    U, _ = np.linalg.qr(rng.standard_normal((d, k)))
    theta = np.linspace(theta_hi, theta_lo, k)
    X = rng.standard_normal((n, d)) + (rng.standard_normal((n, k)) * np.sqrt(theta)) @ U.T
    Xq = np.clip(np.round(X * grid), -32767, 32767).astype(np.int16)
    return Xq, U


def xq_digest(Xq):
    """sha256 of the int16 sample bytes (a seeded fixture pins its regenerated input)."""
    return hashlib.sha256(np.ascontiguousarray(Xq).tobytes()).hexdigest()
