"""Drop-in for the functions of ``Online Distributed PCA.ipynb`` plus the online
(multi-step) estimator, on the GPU hot path.

Citations are raw line numbers of the notebook JSON (``NB:<n>``) and
``assets/algorithm.png`` (the algorithm figure, lines 1-7).

* ``make_batches(data, batch_size)``      NB:149-153
* ``top_k_eigenvectors(matrix, k)``       NB:219-226 (== distributed.py:22-29)
* ``compute_segma_hat(x)``                NB:235-246 name, distributed.py:59-70 maths
  (the notebook's own body builds an n x n Gram and fails for n != d)
* ``online_distributed_pca(...)``         NB:277-316 ("notebook" schedule) or the
  figure's schedule; Sigma_tilde is never formed: it is kept as the stack of
  weighted server bases sqrt(w_t) V_bar_t^T and solved with the implicit
  projector-average operator.
* ``project(X, matrix_w)``                NB:345 (``lambda X: X @ matrix_w``)
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import linalg
from .distributed import compute_sigma_hat, top_k_eigenvectors  # noqa: F401  (re-export)

__all__ = ["make_batches", "top_k_eigenvectors", "compute_segma_hat", "online_distributed_pca",
           "OnlineDistributedPCA", "project", "one_shot_distributed_pca"]


def make_batches(data, batch_size):
    """NB:149-153: fixed-size row batches, the last one partial."""
    chunks = (data.shape[0] - 1) // batch_size + 1
    return [data[i * batch_size:(i + 1) * batch_size] for i in range(chunks)]


def compute_segma_hat(x):
    """Sigma_hat = X^T X / n (distributed.py:59-70 semantics, the notebook's name)."""
    return compute_sigma_hat(x)


def _worker_basis(x, k: int) -> torch.Tensor:
    """One worker: GPU Sigma_hat then top-k; returns V (d x k, column-major, device).
    float64 batches (the notebook's data.mean(axis=3) values, NB:54) take the
    mean-shifted float64 covariance; uint8 the exact one; float32 the fp32 SYRK."""
    if not isinstance(x, torch.Tensor):
        x = torch.as_tensor(np.asarray(x))
    if x.dtype == torch.uint8:
        S = linalg.sigma_hat(x, dtype=torch.float64)
    else:
        S = linalg.sigma_hat(linalg.require_device_tensor(x, "batch", keep_f64=True))
    return linalg.topk_eigh(S, k, check_finite=False).V


def _server(bases, k: int, m: int) -> torch.Tensor:
    """top_k((1/m) sum V V^T) without forming it (NB:300-306; figure line 5)."""
    Wt = linalg.stack_bases(bases)
    return linalg.projavg_topk(Wt, k, 1.0 / m, q0=bases[0]).V


class OnlineDistributedPCA:
    """Online estimator: Sigma_tilde(t) = Sigma_tilde(t-1) + w_t V_bar_t V_bar_t^T.

    The accumulated matrix is held implicitly as rows sqrt(w_t) V_bar_t^T
    (d x (t k) floats instead of d x d), and ``result()`` is its top-k.
    """

    def __init__(self, k: int, m: int):
        self.k, self.m = int(k), int(m)
        self.rows = []   # sqrt(w_t) * V_bar_t^T, each k x d
        self.vbars = []

    def step(self, shards, weight: float) -> torch.Tensor:
        bases = [_worker_basis(x, self.k) for x in shards]
        vbar = _server(bases, self.k, self.m)
        self.vbars.append(vbar)
        self.rows.append(math.sqrt(weight) * vbar.t())
        return vbar

    def result(self) -> linalg.EigResult:
        Wt = torch.cat(self.rows, dim=0).contiguous()
        return linalg.projavg_topk(Wt, self.k, 1.0, q0=self.vbars[-1])


def online_distributed_pca(batches=None, m: int = 10, T: int = 10, k: int = 2,
                           schedule: str = "notebook", batch_fn=None):
    """Online distributed PCA.  Returns (matrix_w d x k ascending, eigenvalues).

    schedule="notebook" reproduces NB:277-316 as saved: t = 1..T-1 (NB:288),
    worker l always reads batches[l] (NB:293), the average uses the first m
    bases (NB:302), weight 1/(t+1) (NB:307).
    schedule="figure" follows assets/algorithm.png: t = 1..T, worker l reads
    batch_fn(t, l) (1-based), weight 1/T.
    Output type follows the input: numpy in -> numpy float64 out.
    """
    est = OnlineDistributedPCA(k, m)
    if schedule == "notebook":
        if batches is None:
            raise ValueError("schedule='notebook' needs batches")
        numpy_out = isinstance(batches[0], np.ndarray)
        for t in range(1, T):
            est.step([batches[l] for l in range(m)], 1.0 / (t + 1))
    elif schedule == "figure":
        if batch_fn is None:
            raise ValueError("schedule='figure' needs batch_fn(t, l)")
        numpy_out = isinstance(batch_fn(1, 1), np.ndarray)
        for t in range(1, T + 1):
            est.step([batch_fn(t, l) for l in range(1, m + 1)], 1.0 / T)
    else:
        raise ValueError(f"unknown schedule {schedule!r}")
    res = est.result()
    if numpy_out:
        return (np.asfortranarray(res.V.double().cpu().numpy()),
                res.evals.double().cpu().numpy())
    return res.V, res.evals


def one_shot_distributed_pca(data, k: int, batches_number: int):
    """distributed.py master/slave pipeline in one call: contiguous shards of N // M
    rows (remainder dropped, :99-104), worker top-k, implicit server solve."""
    x = linalg.require_device_tensor(data, "data", keep_f64=True)
    step = x.shape[0] // batches_number
    bases = [_worker_basis(x[i * step:(i + 1) * step], k) for i in range(batches_number)]
    Wt = linalg.stack_bases(bases)
    return linalg.projavg_topk(Wt, k, 1.0 / batches_number, q0=bases[0])


def project(X, matrix_w):
    """NB:345 ``online_distributed_PCA = lambda X: X @ matrix_w``."""
    if isinstance(X, np.ndarray) and isinstance(matrix_w, np.ndarray):
        xw = linalg.project(linalg.require_device_tensor(X), linalg.require_device_tensor(matrix_w))
        return xw.double().cpu().numpy()
    return linalg.project(linalg.require_device_tensor(X), linalg.require_device_tensor(matrix_w))
