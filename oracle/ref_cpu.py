"""CPU oracle: float64 NumPy/SciPy restatement of the reference's hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / CPU baseline.  The product (``distributed_eigenspaces_amd``) never
imports it and has no CPU fallback.

Pinning: every function below is checked against golden vectors produced by
running the reference itself in the survey container
(``tests/golden/gen_golden.py``; ``tests/test_oracle_golden.py``).  The reference
has no tests or fixtures of its own, so these generated vectors
are the only pin.  Exceptions, marked "parity unpinned" below: the figure
schedule of the online estimator (``assets/algorithm.png`` is an image, not
code) and Oja (not in the reference at all).

Citations are ``file:line`` in TimeEscaper/distributed_eigenspaces; ``NB:<n>`` is
raw line n of ``Online Distributed PCA.ipynb``.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg

__all__ = [
    "sigma_hat", "top_k_eigh", "top_k_eigenvectors", "split_batches",
    "dispatch_order", "projector_average", "server_topk", "make_batches",
    "online_notebook", "online_figure", "one_shot", "oja_epoch", "oja_stream",
    "projector_distance", "sin_theta", "align_signs",
]


def sigma_hat(x: np.ndarray) -> np.ndarray:
    """Sigma_hat = X^T X / n, uncentered, float64.

    ``SlaveNode.compute_sigma_hat_`` distributed.py:59-70: ``n, d = x.shape`` (:66),
    ``np.zeros((d, d))`` (:67), ``+= np.dot(x.T, x)`` (:68), ``/= n`` (:69).
    """
    x = np.asarray(x, dtype=np.float64)
    n, d = x.shape
    s = np.zeros((d, d))
    s += np.dot(x.T, x)
    s /= n
    return s


def top_k_eigh(matrix: np.ndarray, k: int):
    """(eigenvalues[k], eigenvectors[d, k]) of the top-k, ascending order.

    ``Node.top_k_eigenvectors`` distributed.py:22-29 (``eigh(matrix,
    eigvals=(N-k, N-1))``; NB:219-226 twin).  ``eigvals=`` was removed in scipy
    1.14; ``subset_by_index`` is the same ``?syevr`` driver and inclusive range.
    The reference returns only ``[1]``; the eigenvalues ``[0]`` are the side
    output the north star asks for.
    """
    n = matrix.shape[0]
    w, v = scipy.linalg.eigh(matrix, subset_by_index=(n - k, n - 1))
    return w, v


def top_k_eigenvectors(matrix: np.ndarray, k: int) -> np.ndarray:
    """distributed.py:22-29 exactly: eigenvectors only, ascending, Fortran order."""
    return top_k_eigh(matrix, k)[1]


def split_batches(n_rows: int, batches_number: int):
    """Master's shard split, distributed.py:99-104: step = N // M, remainder dropped."""
    step = n_rows // batches_number
    return [(i * step, (i + 1) * step) for i in range(batches_number)]


def dispatch_order(batches_number: int, window: int = 5):
    """Order in which the master hands out shards (distributed.py:108-111, :132-134).

    ``batches.pop()`` = LIFO; five requests are sent up front (:108).  With a FIFO
    broker and one slave, shards complete in the order they are sent, so the
    arrival order at the master is the dispatch order.  M < 5 raises IndexError in
    the reference (:111 pops an empty list).
    """
    if batches_number < window:
        raise IndexError("pop from empty list")
    idx = list(range(batches_number))
    return [idx.pop() for _ in range(batches_number)]


def projector_average(Vs, batches_number: int) -> np.ndarray:
    """Sigma_tilde = (1/M) sum_i V_i V_i^T in list order (distributed.py:126-130)."""
    d = Vs[0].shape[0]
    s = np.zeros((d, d))
    for v in Vs:
        s += v @ v.T
    s /= batches_number
    return s


def server_topk(Vs, k: int, batches_number: int | None = None):
    """Server solve: top_k of the projector average (NB:300-306; figure line 5)."""
    m = len(Vs) if batches_number is None else batches_number
    return top_k_eigh(projector_average(Vs, m), k)


def make_batches(data, batch_size: int):
    """Notebook ``make_batches`` (NB:149-153): fixed size, last batch partial."""
    chunks = (data.shape[0] - 1) // batch_size + 1
    return [data[i * batch_size:(i + 1) * batch_size] for i in range(chunks)]


def one_shot(data, k: int, batches_number: int):
    """distributed.py master/slave pipeline + NB:306 server solve, float64.

    Returns (worker_evals, worker_V, server_evals, server_V).  Shards follow
    :99-104; the average is taken in shard order (arrival order only reorders a
    float64 sum; golden vectors pin the LIFO order separately).
    """
    ws, vs = [], []
    for lo, hi in split_batches(data.shape[0], batches_number):
        w, v = top_k_eigh(sigma_hat(data[lo:hi]), k)
        ws.append(w); vs.append(v)
    sw, sv = server_topk(vs, k, batches_number)
    return ws, vs, sw, sv


def online_notebook(batches, m: int = 10, T: int = 10, k: int = 2):
    """Notebook online loop as saved (NB:277-316), with distributed.py Sigma_hat.

    Quirks kept on purpose: t runs 1..T-1 (NB:288); every step
    reads ``batches[l]`` for l < m and ignores t (NB:293); the average sums only
    the first m entries of the growing list (NB:302); weight 1/(t+1) (NB:307).
    Returns (matrix_w, final eigenvalues, segma_e).
    """
    d = batches[0].shape[1]
    v_hat_list = []
    segma_e = np.zeros((d, d))
    for t in range(1, T):
        for l in range(m):
            v_hat_list.append(top_k_eigenvectors(sigma_hat(batches[l]), k))
        segma_bar = np.zeros((d, d))
        for l in range(m):
            segma_bar += v_hat_list[l] @ v_hat_list[l].T
        segma_bar /= m
        v_dash = top_k_eigenvectors(segma_bar, k)
        segma_e = segma_e + (1 / (t + 1)) * v_dash @ v_dash.T
    w, matrix_w = top_k_eigh(segma_e, k)
    return matrix_w, w, segma_e


def online_figure(batch_fn, m: int, T: int, k: int):
    """Figure schedule (assets/algorithm.png lines 1-7): parity unpinned (image only).

    ``batch_fn(t, l)`` returns X^(l)(t) for t = 1..T, l = 1..m; weight T^-1.
    Returns (final eigenvalues, V_K(T), list of V_bar(t)).
    """
    d = batch_fn(1, 1).shape[1]
    sig = np.zeros((d, d))
    vbars = []
    for t in range(1, T + 1):
        vs = [top_k_eigenvectors(sigma_hat(batch_fn(t, l)), k) for l in range(1, m + 1)]
        _, vbar = server_topk(vs, k, m)
        vbars.append(vbar)
        sig = sig + (1.0 / T) * vbar @ vbar.T
    w, v = top_k_eigh(sig, k)
    return w, v, vbars


def oja_epoch(X, V0, eta: float, batch: int):
    """Mini-batch Oja: V <- orth(V + eta * X_b^T (X_b V) / b).  Parity unpinned:
    not in the reference (named only by BASELINE.json north_star / config 4)."""
    V = np.array(V0, dtype=np.float64)
    for lo in range(0, X.shape[0], batch):
        xb = np.asarray(X[lo:lo + batch], dtype=np.float64)
        V = V + eta * (xb.T @ (xb @ V)) / xb.shape[0]
        V, _ = np.linalg.qr(V)
    return V


def oja_stream(rank_batches, V0, eta: float, agg_every: int):
    """Streaming Oja on R ranks with periodic aggregation (parity unpinned: not in
    the reference; restates distributed_eigenspaces_amd.streaming.StreamingOja).

    ``rank_batches[r]`` is rank r's list of row batches (all lists equally long).
    Every rank starts from V0; after every ``agg_every`` batches all ranks adopt the
    server solve of their bases (``server_topk``: top-k of (1/R) sum V_r V_r^T,
    distributed.py:126-130 + NB:306).  Returns the rank-0 basis at the end."""
    R = len(rank_batches)
    k = np.asarray(V0).shape[1]
    Vs = [np.array(V0, dtype=np.float64) for _ in range(R)]
    for i in range(len(rank_batches[0])):
        for r in range(R):
            xb = np.asarray(rank_batches[r][i], dtype=np.float64)
            v = Vs[r] + eta * (xb.T @ (xb @ Vs[r])) / xb.shape[0]
            Vs[r], _ = np.linalg.qr(v)
        if agg_every > 0 and (i + 1) % agg_every == 0:
            _, vbar = server_topk(Vs, k, R)
            Vs = [vbar.copy() for _ in range(R)]
    return Vs[0]


def projector_distance(A, B) -> float:
    """||A A^T - B B^T||_F without forming d x d (exact for any A, B, in float64):
    ||A A^T - B B^T||_F^2 = ||A^T A||_F^2 + ||B^T B||_F^2 - 2 ||A^T B||_F^2.
    Sign- and rotation-invariant; also charges column-norm errors (not only angles)."""
    A = np.asarray(A, dtype=np.float64)
    B = np.asarray(B, dtype=np.float64)
    aa, bb, ab = A.T @ A, B.T @ B, A.T @ B
    val = np.sum(aa * aa) + np.sum(bb * bb) - 2.0 * np.sum(ab * ab)
    return float(np.sqrt(max(val, 0.0)))


def align_signs(V, ref):
    """Flip the sign of each column of V to match ref (eigenvectors are sign-ambiguous)."""
    V = np.array(V, dtype=np.float64)
    s = np.sign(np.sum(V * np.asarray(ref, dtype=np.float64), axis=0))
    s[s == 0] = 1.0
    return V * s


def sin_theta(A, B) -> float:
    """||sin Theta(A, B)||_2 of two orthonormal bases."""
    s = np.linalg.svd(np.asarray(A, np.float64).T @ np.asarray(B, np.float64), compute_uv=False)
    return float(np.sqrt(max(0.0, 1.0 - float(np.min(s)) ** 2)))
