"""deig_backend - the file a maintainer of TimeEscaper/distributed_eigenspaces would add
next to its ``distributed.py`` to run the hot path on an MI355X through ``libdeig.so``.

It imports only ``ctypes`` and ``numpy`` (plus the standard library): device memory
comes from the HIP runtime (``libamdhip64.so``) through ctypes, the arithmetic from
libdeig's C ABI (``include/deig.h``).  Every function keeps the reference's data flow
- numpy float64 in, numpy float64 out - and binds the entry points that hold parity
on it:

* ``compute_sigma_hat(x)``  -> ``deig_syrk_shift`` (float64 X in, float64 Sigma out:
  the mean-shifted split3 SYRK, mean terms in double), or ``deig_syrk_u8`` (exact
  integer covariance) for uint8 samples.  Replaces ``SlaveNode.compute_sigma_hat_``,
  reference/distributed.py:59-70.
* ``top_k_eigenvectors(matrix, k)`` -> ``deig_topk_sym_ex`` with ``DEIG_F64`` (the
  solver reads the float64 Sigma in double; any d, any 1 <= k <= d).  Replaces
  ``Node.top_k_eigenvectors``, reference/distributed.py:22-29 (eigh(...)[1]:
  ascending, Fortran order); ``top_k_eigh`` also returns the eigenvalues.
* ``server_top_k(eigenspaces, k, batches_number)`` -> ``deig_projavg_topk_f32``: the
  top-k of (1 / batches_number) sum V V^T without forming it.  Replaces the master's
  ``sigma_tilde`` loop, reference/distributed.py:126-130, plus the notebook's server
  solve (Online Distributed PCA.ipynb raw line 306).

Wiring (reference side):

    # distributed.py
    import deig_backend
    class Node:
        def top_k_eigenvectors(self, matrix, k):
            return deig_backend.top_k_eigenvectors(matrix, k)
    class SlaveNode(Node):
        def compute_sigma_hat_(self, x):
            return deig_backend.compute_sigma_hat(x)
    # MasterNode.callback_, once every batch is in (:126-130):
    #     self.eigenspace = deig_backend.server_top_k(self.computed_eigens, self.rank,
    #                                                 self.batches_number)

``DEIG_LIB`` names libdeig.so (default: the in-tree build next to this directory).
Calls are synchronous (like numpy / scipy) and run on the default HIP stream of the
current device; return code 1 (DEIG_NOT_CONVERGED) becomes a RuntimeWarning, negative
codes a RuntimeError with deig_last_error().
"""
from __future__ import annotations

import ctypes
import os
import warnings

import numpy as np

__all__ = ["compute_sigma_hat", "top_k_eigenvectors", "top_k_eigh", "server_top_k"]

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("DEIG_LIB") or os.path.join(os.path.dirname(_HERE), "distributed_eigenspaces_amd",
                                                        "libdeig.so")

DEIG_OK, DEIG_NOT_CONVERGED = 0, 1
DEIG_F32, DEIG_F64 = 0, 1
DEIG_U8_RAW = 0
_H2D, _D2H = 1, 2  # hipMemcpyHostToDevice, hipMemcpyDeviceToHost

_i64, _sz, _vp, _int = ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int
_f32, _f64 = ctypes.c_float, ctypes.c_double
_pint, _pf32 = ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_float)

_hip = None
_L = None


def _load():
    """Bind the HIP runtime and libdeig.so (once)."""
    global _hip, _L
    if _L is not None:
        return
    hip = None
    for name in ("libamdhip64.so", "libamdhip64.so.7", "/opt/rocm/lib/libamdhip64.so"):
        try:
            hip = ctypes.CDLL(name)
            break
        except OSError:
            continue
    if hip is None:
        raise OSError("libamdhip64.so (the HIP runtime) not found")
    hip.hipMalloc.argtypes = [ctypes.POINTER(_vp), _sz]
    hip.hipFree.argtypes = [_vp]
    hip.hipMemcpy.argtypes = [_vp, _vp, _sz, _int]
    hip.hipMemset.argtypes = [_vp, _int, _sz]
    hip.hipDeviceSynchronize.argtypes = []
    hip.hipGetErrorString.restype = ctypes.c_char_p
    hip.hipGetErrorString.argtypes = [_int]
    L = ctypes.CDLL(_LIB_PATH)
    L.deig_last_error.restype = ctypes.c_char_p
    L.deig_syrk_shift.argtypes = [_vp, _int, _i64, _i64, _i64, _f64, _vp, _i64, _vp, _i64, _vp, _sz, _vp]
    L.deig_syrk_shift_workspace.restype = _sz
    L.deig_syrk_shift_workspace.argtypes = [_i64, _i64, _int]
    L.deig_syrk_u8.argtypes = [_vp, _i64, _i64, _i64, _int, _f64, _vp, _i64, _vp, _i64, _vp, _sz, _vp]
    L.deig_syrk_u8_workspace.restype = _sz
    L.deig_syrk_u8_workspace.argtypes = [_i64, _i64, _int]
    L.deig_topk_sym_ex.argtypes = [_vp, _int, _i64, _i64, _int, _int, _int, _f32, _vp, _int, _i64,
                                   _vp, _i64, _vp, _pint, _pf32, _vp, _vp, _sz, _vp]
    L.deig_topk_workspace_ex.restype = _sz
    L.deig_topk_workspace_ex.argtypes = [_i64, _int, _int, _int, _vp]
    L.deig_projavg_topk_f32.argtypes = [_vp, _i64, _i64, _i64, _f32, _int, _int, _int, _f32, _vp, _int,
                                        _i64, _vp, _i64, _vp, _pint, _pf32, _vp, _sz, _vp]
    L.deig_projavg_workspace.restype = _sz
    L.deig_projavg_workspace.argtypes = [_i64, _i64, _int, _int]
    _hip, _L = hip, L


def _hip_check(err, what):
    if err != 0:
        raise RuntimeError(f"{what}: {_hip.hipGetErrorString(err).decode()} ({err})")


def _check(rc, what):
    if rc == DEIG_OK:
        return
    msg = _L.deig_last_error().decode()
    if rc == DEIG_NOT_CONVERGED:
        warnings.warn(f"{what}: {msg}", RuntimeWarning, stacklevel=3)
        return
    raise RuntimeError(f"{what}: {msg} (code {rc})")


class _Device:
    """Device buffers of one call, freed on exit."""

    def __init__(self):
        self.ptrs = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        _hip.hipDeviceSynchronize()
        for p in self.ptrs:
            _hip.hipFree(p)

    def alloc(self, nbytes):
        p = _vp()
        _hip_check(_hip.hipMalloc(ctypes.byref(p), max(int(nbytes), 256)), "hipMalloc")
        self.ptrs.append(p)
        return p

    def upload(self, a: np.ndarray):
        a = np.ascontiguousarray(a)
        p = self.alloc(a.nbytes)
        _hip_check(_hip.hipMemcpy(p, a.ctypes.data_as(_vp), a.nbytes, _H2D), "hipMemcpy H2D")
        return p

    def download(self, p, shape, dtype):
        out = np.empty(shape, dtype=dtype)
        _hip_check(_hip.hipDeviceSynchronize(), "hipDeviceSynchronize")
        _hip_check(_hip.hipMemcpy(out.ctypes.data_as(_vp), p, out.nbytes, _D2H), "hipMemcpy D2H")
        return out


def compute_sigma_hat(x) -> np.ndarray:
    """``SlaveNode.compute_sigma_hat_`` (distributed.py:59-70): X^T X / n, uncentered,
    as a (d, d) float64 array (bit-exactly symmetric).  Float samples go through
    deig_syrk_shift in float64; uint8 samples through the exact deig_syrk_u8.

    uint8 input DELIBERATELY diverges from the reference: its ``np.dot(x.T, x)`` on a
    uint8 array accumulates in uint8 and wraps modulo 256 before the float64 add
    (distributed.py:67-69), while this returns the exact Sigma_hat of the byte values
    (what the reference computes on the float64 grey values it actually feeds in,
    distributed.py:169-173); ``x.astype(np.float64)`` gives the same value here."""
    _load()
    x = np.asarray(x)
    if x.ndim != 2:
        raise ValueError(f"x must be 2-D (n, d), got shape {x.shape}")
    n, d = x.shape
    if n == 0:
        return np.full((d, d), np.nan)  # numpy: zeros / 0
    with _Device() as dv:
        S = dv.alloc(d * d * 8)
        if x.dtype == np.uint8 and d % 4 == 0:
            X = dv.upload(x)
            nb = _L.deig_syrk_u8_workspace(n, d, DEIG_U8_RAW)
            ws = dv.alloc(nb)
            rc = _L.deig_syrk_u8(X, n, d, d, DEIG_U8_RAW, 1.0 / n, None, d, S, d, ws, nb, None)
            _check(rc, "deig_syrk_u8")
        else:
            X = dv.upload(np.asarray(x, dtype=np.float64))
            nb = _L.deig_syrk_shift_workspace(n, d, DEIG_F64)
            ws = dv.alloc(nb)
            rc = _L.deig_syrk_shift(X, DEIG_F64, n, d, d, 1.0 / n, S, d, None, d, ws, nb, None)
            _check(rc, "deig_syrk_shift")
        return dv.download(S, (d, d), np.float64)


def top_k_eigh(matrix, k: int, tol: float = 1e-6, max_sweeps: int = 300):
    """(eigenvalues ascending (k,), eigenvectors (d, k) Fortran-ordered, ascending) of a
    symmetric matrix - scipy.linalg.eigh(matrix, subset_by_index=(d-k, d-1)) as the
    reference calls it (distributed.py:29), read in float64 by the solver."""
    _load()
    S_h = np.ascontiguousarray(matrix, dtype=np.float64)
    if S_h.ndim != 2 or S_h.shape[0] != S_h.shape[1]:
        raise ValueError(f"expected a square matrix, got shape {S_h.shape}")
    d = S_h.shape[0]
    k = int(k)
    if not 1 <= k <= d:
        raise ValueError(f"k={k} out of range [1, {d}]")
    if not np.isfinite(S_h).all():
        raise ValueError("array must not contain infs or NaNs")
    with _Device() as dv:
        S = dv.upload(S_h)
        V = dv.alloc(d * k * 4)
        ev = dv.alloc(k * 4)
        nb = _L.deig_topk_workspace_ex(d, k, 0, DEIG_F64, None)
        ws = dv.alloc(nb)
        sw, rs = ctypes.c_int(0), ctypes.c_float(0)
        rc = _L.deig_topk_sym_ex(S, DEIG_F64, d, d, k, 0, int(max_sweeps), float(tol), None, 0, d, V, d, ev,
                                 ctypes.byref(sw), ctypes.byref(rs), None, ws, nb, None)
        _check(rc, "deig_topk_sym_ex")
        Vt = dv.download(V, (k, d), np.float32)  # column-major d x k == row-major k x d
        w = dv.download(ev, (k,), np.float32)
    return w.astype(np.float64), np.asfortranarray(Vt.T.astype(np.float64))


def top_k_eigenvectors(matrix, k: int) -> np.ndarray:
    """``Node.top_k_eigenvectors`` (distributed.py:22-29): eigh(...)[1]."""
    return top_k_eigh(matrix, k)[1]


def server_top_k(eigenspaces, k: int, batches_number: int, tol: float = 1e-6,
                 max_sweeps: int = 300) -> np.ndarray:
    """Top-k eigenvectors of (1 / batches_number) sum_i V_i V_i^T (the master's
    sigma_tilde, distributed.py:126-130, then the notebook's server solve, raw line
    306), never forming the d x d matrix; warm-started from the first basis."""
    _load()
    bases = [np.asarray(v, dtype=np.float64) for v in eigenspaces]
    if not bases:
        raise ValueError("no eigenspaces")
    d = bases[0].shape[0]
    k = int(k)
    dp = max(16, (d + 3) // 4 * 4)  # the implicit operator takes d % 4 == 0, d >= 16:
    Wt = np.zeros((sum(v.shape[1] for v in bases), dp), dtype=np.float32)  # zero columns add nothing
    r = 0
    for v in bases:
        Wt[r:r + v.shape[1], :d] = v.T
        r += v.shape[1]
    mk = Wt.shape[0]
    k0 = min(bases[0].shape[1], k)
    Q0 = np.zeros((k0, dp), dtype=np.float32)  # column-major dp x k0
    Q0[:, :d] = bases[0][:, :k0].T
    with _Device() as dv:
        W = dv.upload(Wt)
        Q = dv.upload(Q0)
        V = dv.alloc(dp * k * 4)
        ev = dv.alloc(k * 4)
        nb = _L.deig_projavg_workspace(dp, mk, k, 0)
        ws = dv.alloc(nb)
        sw, rs = ctypes.c_int(0), ctypes.c_float(0)
        rc = _L.deig_projavg_topk_f32(W, dp, mk, dp, 1.0 / batches_number, k, 0, int(max_sweeps), float(tol),
                                      Q, k0, dp, V, dp, ev, ctypes.byref(sw), ctypes.byref(rs), ws, nb, None)
        _check(rc, "deig_projavg_topk_f32")
        Vt = dv.download(V, (k, dp), np.float32)
    return np.asfortranarray(Vt[:, :d].T.astype(np.float64))
