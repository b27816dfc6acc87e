"""Device-level API of the hot path: PyTorch-ROCm tensors in, HIP kernels via the C ABI.

Buffers are torch tensors on ``cuda:<i>`` (HIP under ROCm); PyTorch is used only
for device memory, streams and collectives.  Every op launches on the current
torch stream of the tensor's device and returns without a host sync, except the
eigensolvers, which synchronise that stream between sweeps to test convergence
(the reference's scipy.linalg.eigh is synchronous too).

There is no CPU fallback: inputs must live on a ROCm device, and the ops raise
if ``libdeig.so`` is missing.
"""
from __future__ import annotations

import ctypes
import threading
import warnings
from dataclasses import dataclass

import torch

from . import _lib

__all__ = [
    "sigma_hat", "topk_eigh", "topk_eigh_batch", "projavg_topk", "oja_step", "default_subspace",
    "EigResult", "require_device_tensor", "project", "stack_bases", "gemm_skinny",
    "oja_steps", "oja_check", "sym_apply", "sym_power", "sigma_hat_u8", "sigma_hat_shift",
]

DEFAULT_TOL = 1e-6
DEFAULT_MAX_SWEEPS = 300
MAX_P = 128  # widest subspace of one solver block (kMaxP in csrc/capi.hip); k > 128
             # is solved in locked blocks of p - 16 pairs


class IndefiniteWarning(RuntimeWarning):
    """topk_eigh returned a negative eigenvalue: the input is not PSD."""


@dataclass
class EigResult:
    """Top-k eigenpairs, ascending order (LAPACK / scipy.linalg.eigh convention)."""

    evals: torch.Tensor   # (k,) float32
    V: torch.Tensor       # (d, k) float32, column-major (Fortran) strides (1, d)
    sweeps: int
    resid: float          # max_j ||A v_j - lambda_j v_j|| / |lambda_max|
    converged: bool


# ---------------------------------------------------------------- workspace cache
class _Workspace(threading.local):
    def __init__(self):
        self.bufs = {}


_ws = _Workspace()


def _workspace(device: torch.device, nbytes: int) -> torch.Tensor:
    """Per-thread, per-device, per-stream grow-only uint8 workspace."""
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    buf = _ws.bufs.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        _ws.bufs[key] = buf
    return buf


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device_tensor(t, name: str = "input", keep_f64: bool = False) -> torch.Tensor:
    """float32 tensor on a ROCm device (host arrays are copied over).  No CPU path.
    keep_f64: float64 input stays float64 (the reference's dtype; the covariance and
    the solver take it as is)."""
    if not torch.cuda.is_available():
        raise RuntimeError(
            f"{name}: distributed_eigenspaces_amd runs only on a ROCm GPU (MI355X); "
            "no GPU is visible and there is no CPU fallback")
    if not isinstance(t, torch.Tensor):
        t = torch.as_tensor(t)
    if t.device.type != "cuda":
        t = t.to(device=torch.device("cuda", torch.cuda.current_device()))
    if keep_f64 and t.dtype == torch.float64:
        return t
    if t.dtype != torch.float32:
        t = t.to(torch.float32)
    return t


def _rowmajor_4(t: torch.Tensor, name: str) -> torch.Tensor:
    """2-D row-major view with unit column stride, row stride % 4 == 0, 16-B aligned."""
    if t.dim() != 2:
        raise ValueError(f"{name} must be 2-D, got shape {tuple(t.shape)}")
    ok = (t.stride(1) == 1 and t.stride(0) % 4 == 0 and t.stride(0) >= t.shape[1]
          and t.data_ptr() % 16 == 0)
    if ok:
        return t
    d = t.shape[1]
    dp = (d + 3) // 4 * 4
    out = torch.zeros((t.shape[0], dp), dtype=torch.float32, device=t.device)
    out[:, :d] = t
    return out


def default_subspace(d: int, k: int) -> int:
    return int(_lib.lib().deig_default_subspace(int(d), int(k)))


# ---------------------------------------------------------------- covariance
def sigma_hat(x: torch.Tensor, alpha: float | None = None,
              out: torch.Tensor | None = None, algo: str = "auto",
              shift: bool | None = None, dtype: torch.dtype | None = None,
              accumulate: bool = False) -> torch.Tensor:
    """Sigma_hat = alpha * X^T X with alpha = 1/n by default (uncentered).

    GPU replacement for ``SlaveNode.compute_sigma_hat_`` (distributed.py:59-70).
    x: (n, d) on the GPU (host arrays are copied over):
      * float32 (default path): a (d, d) float32 tensor, bit-exactly symmetric.
        algo: "split3" (fp32 operands as bf16 hi/lo pairs on bf16 MFMA, fp32
        accumulation, see include/deig.h), "fp32" (f32 MFMA fma chain) or "auto"
        (split3 for n >= 1024 rows, fp32 below);
      * float64 (the reference's dtype, distributed.py:171) or ``shift=True``: the
        mean-shifted covariance (deig_syrk_shift: the SYRK runs on X - mu, the mean
        terms are added in double) returned as float64 - the small eigenvectors of an
        uncentered covariance keep float64 parity (csrc/shift.hip);
      * uint8 samples: the exact integer path (sigma_hat_u8; 2-D raw bytes or
        N x H x W x 3 pixels with the reference's grayscale fused in).
    dtype: result dtype (float32 / float64) for the shifted and uint8 paths.
    accumulate: ``out += alpha X^T X`` (float32 split3 path; a covariance streamed
    through in row blocks, DEIG_SYRK_ACCUMULATE).
    """
    if not isinstance(x, torch.Tensor):
        x = torch.as_tensor(x)
    if x.dtype == torch.uint8:
        return sigma_hat_u8(x, alpha=alpha, out=out, dtype=dtype or torch.float32)
    if shift is None:
        shift = x.dtype == torch.float64
    if shift:
        if accumulate:
            raise ValueError("accumulate is for the float32 split3 path (shift=False)")
        return sigma_hat_shift(x, alpha=alpha, out=out, dtype=dtype or torch.float64)
    if algo not in _lib.SYRK_ALGOS:
        raise ValueError(f"algo must be one of {sorted(_lib.SYRK_ALGOS)}, got {algo!r}")
    code = _lib.SYRK_ALGOS[algo]
    x = require_device_tensor(x, "sigma_hat")
    if accumulate:
        if out is None or algo == "fp32" or x.shape[1] % 4 or not out.is_contiguous():
            raise ValueError("accumulate needs out (contiguous d x d float32), d % 4 == 0 and "
                             "the split3 algorithm")
        code = _lib.DEIG_SYRK_SPLIT3 | _lib.DEIG_SYRK_ACCUMULATE
    if x.dim() != 2:
        raise ValueError(f"x must be 2-D (n, d), got {tuple(x.shape)}")
    n, d = x.shape
    if n == 0:
        # numpy: zeros / 0 -> NaN (with a RuntimeWarning); keep that behaviour
        return torch.full((d, d), float("nan"), dtype=torch.float32, device=x.device)
    a = (1.0 / n) if alpha is None else float(alpha)
    xx = _rowmajor_4(x, "x")
    dp = xx.shape[1]
    if out is not None and dp == d and out.shape == (d, d) and out.is_contiguous() \
            and out.dtype == torch.float32 and out.device == x.device and d % 4 == 0:
        S = out
    else:
        S = torch.empty((dp, dp), dtype=torch.float32, device=x.device)
    L = _lib.lib()
    with torch.cuda.device(x.device):
        nbytes = L.deig_syrk_workspace_ex(n, dp, code)
        ws = _workspace(x.device, nbytes) if nbytes else None
        rc = L.deig_syrk_f32_ex(xx.data_ptr(), n, dp, xx.stride(0), ctypes.c_float(a),
                                S.data_ptr(), S.stride(0), code,
                                ws.data_ptr() if ws is not None else None, nbytes,
                                _stream(x.device))
    _lib.check(rc, "deig_syrk_f32_ex")
    if dp != d:
        S = S[:d, :d].contiguous()
        if out is not None:
            out.copy_(S)
            return out
    return S


def sigma_hat_shift(x: torch.Tensor, alpha: float | None = None,
                    out: torch.Tensor | None = None,
                    dtype: torch.dtype = torch.float64) -> torch.Tensor:
    """Mean-shifted covariance alpha * X^T X (alpha = 1/n: distributed.py:59-70) of
    float32 / float64 samples (include/deig.h deig_syrk_shift): the SYRK runs on
    C = fl32(X - mu) and the mean terms are added in double, so its rounding is
    relative to the centred data instead of the dominant mean direction of an
    uncentered covariance.  Returns a (d, d) tensor of ``dtype`` (float64: the
    reference's), bit-exactly symmetric."""
    if not isinstance(x, torch.Tensor):
        x = torch.as_tensor(x)
    if x.dtype not in (torch.float32, torch.float64):
        x = x.to(torch.float64)
    x = require_device_tensor(x, "sigma_hat_shift", keep_f64=True)
    if x.dim() != 2:
        raise ValueError(f"x must be 2-D (n, d), got {tuple(x.shape)}")
    if dtype not in (torch.float32, torch.float64):
        raise ValueError("dtype must be torch.float32 or torch.float64")
    n, d = x.shape
    if n == 0:
        return torch.full((d, d), float("nan"), dtype=dtype, device=x.device)
    if x.stride(1) != 1 or x.stride(0) < d:
        x = x.contiguous()
    a = (1.0 / n) if alpha is None else float(alpha)
    xtype = _lib.DEIG_F64 if x.dtype == torch.float64 else _lib.DEIG_F32
    S = torch.empty((d, d), dtype=dtype, device=x.device)
    f64 = dtype == torch.float64
    L = _lib.lib()
    with torch.cuda.device(x.device):
        nbytes = L.deig_syrk_shift_workspace(n, d, xtype)
        ws = _workspace(x.device, nbytes)
        rc = L.deig_syrk_shift(x.data_ptr(), xtype, n, d, x.stride(0), ctypes.c_double(a),
                               S.data_ptr() if f64 else None, d, None if f64 else S.data_ptr(), d,
                               ws.data_ptr(), nbytes, _stream(x.device))
    _lib.check(rc, "deig_syrk_shift")
    if out is not None:
        out.copy_(S)
        return out
    return S


def sigma_hat_u8(x: torch.Tensor, mode: str = "auto", alpha: float | None = None,
                 out: torch.Tensor | None = None, dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """Exact Sigma_hat of uint8 samples on int8 MFMA (fused ingest).

    x: uint8 tensor on the GPU (host arrays are copied over), either
      * (n, d) raw bytes, mode "raw": V = x;
      * (n, H, W, 3) interleaved pixels (CIFAR layout, load_data.py:18-33), mode
        "gray": V = x.mean(axis=3).reshape(n, H*W) - the reference's preprocessing
        distributed.py:170-173 - fused into the covariance; or (n, 3m) rows with
        mode "gray" explicitly.
    Returns alpha * V^T V (alpha = 1/n: distributed.py:59-70) as a (d, d) tensor of
    ``dtype`` (float32: within one ulp of the exact result - a double quotient
    rounded to float; float64: exact to double rounding).  Every product and sum is an integer computation
    (include/deig.h deig_syrk_u8), so there is no accumulation error at all.
    """
    if not isinstance(x, torch.Tensor):
        x = torch.as_tensor(x)
    if x.dtype != torch.uint8:
        raise ValueError(f"sigma_hat_u8 needs uint8 samples, got {x.dtype}")
    if not torch.cuda.is_available():
        raise RuntimeError("sigma_hat_u8: needs a ROCm GPU; there is no CPU fallback")
    if x.device.type != "cuda":
        x = x.to(torch.device("cuda", torch.cuda.current_device()))
    if mode == "auto":
        mode = "gray" if x.dim() == 4 else "raw"
    if mode not in _lib.U8_MODES:
        raise ValueError(f"mode must be 'auto', 'raw' or 'gray', got {mode!r}")
    n = x.shape[0]
    if mode == "gray":
        if x.dim() == 4:
            if x.shape[3] != 3:
                raise ValueError(f"gray mode needs (n, H, W, 3) pixels, got {tuple(x.shape)}")
            x = x.reshape(n, -1)
        if x.dim() != 2 or x.shape[1] % 3:
            raise ValueError("gray mode needs rows of 3-byte pixels")
        d = x.shape[1] // 3
    else:
        if x.dim() != 2:
            raise ValueError(f"raw mode needs a 2-D (n, d) tensor, got {tuple(x.shape)}")
        d = x.shape[1]
    if n == 0:
        return torch.full((d, d), float("nan"), dtype=dtype, device=x.device)
    a = (1.0 / n) if alpha is None else float(alpha)
    width = 3 * d if mode == "gray" else d
    dp = (d + 3) // 4 * 4
    if x.stride(1) != 1 or x.stride(0) % 4 or x.data_ptr() % 4 or dp != d:
        wp = 3 * dp if mode == "gray" else dp
        xx = torch.zeros((n, (wp + 3) // 4 * 4), dtype=torch.uint8, device=x.device)
        xx[:, :width] = x[:, :width]
        x = xx
    if dtype not in (torch.float32, torch.float64):
        raise ValueError("dtype must be torch.float32 or torch.float64")
    direct = (out is not None and dp == d and out.dtype == dtype and out.device == x.device
              and out.shape == (d, d) and out.stride(1) == 1 and out.stride(0) >= d)
    S = out if direct else torch.empty((dp, dp), dtype=dtype, device=x.device)
    L = _lib.lib()
    with torch.cuda.device(x.device):
        nbytes = L.deig_syrk_u8_workspace(n, dp, _lib.U8_MODES[mode])
        ws = _workspace(x.device, nbytes)
        f32 = dtype == torch.float32
        lds = S.stride(0)
        rc = L.deig_syrk_u8(x.data_ptr(), n, dp, x.stride(0), _lib.U8_MODES[mode], ctypes.c_double(a),
                            S.data_ptr() if f32 else None, lds, None if f32 else S.data_ptr(), lds,
                            ws.data_ptr(), nbytes, _stream(x.device))
    _lib.check(rc, "deig_syrk_u8")
    if direct:  # written in place
        return out
    if dp != d:
        S = S[:d, :d].contiguous()
    if out is not None:
        out.copy_(S)
        return out
    return S


# ---------------------------------------------------------------- eigensolvers
def _pad_dim(d: int) -> int:
    return max(16, (d + 3) // 4 * 4)


def _finish(rc, V, evals, sweeps, resid, what):
    _lib.check(rc, what)
    conv = rc == _lib.DEIG_OK
    if not conv:
        warnings.warn(f"{what}: {_lib.last_error()}", _lib.NotConvergedWarning, stacklevel=3)
    return EigResult(evals=evals, V=V, sweeps=int(sweeps.value), resid=float(resid.value),
                     converged=conv)


def _colmajor(d: int, k: int, device) -> torch.Tensor:
    return torch.empty((k, d), dtype=torch.float32, device=device).t()


def _warm(q0, d, device):
    if q0 is None:
        return None, 0, d
    q = require_device_tensor(q0, "q0")
    if q.dim() == 1:
        q = q[:, None]
    if q.shape[0] != d:
        raise ValueError(f"q0 must have {d} rows")
    q = q.t().contiguous().t()  # column-major
    return q, q.shape[1], q.stride(1)


def _solver_matrix(S: torch.Tensor) -> torch.Tensor:
    """S as the solver reads it: unit column stride; when the library reads it in
    place (d % 4 == 0: include/deig.h deig_topk_sym_ex) also a row stride % 4 == 0 and
    16-byte alignment.  Other dimensions are staged by the library itself (a zero-padded
    copy in the workspace whose padding never enters the result), so no padding here."""
    d = S.shape[0]
    if S.stride(1) != 1 or S.stride(0) < d:
        S = S.contiguous()
    if d % 4 == 0 and (S.stride(0) % 4 or S.data_ptr() % 16):
        S = S.clone(memory_format=torch.contiguous_format)
    return S


def topk_eigh(S: torch.Tensor, k: int, *, p: int | None = None, tol: float = DEFAULT_TOL,
              max_sweeps: int = DEFAULT_MAX_SWEEPS, q0: torch.Tensor | None = None,
              check_finite: bool = True, opts: "_lib.SolverOpts | None" = None) -> EigResult:
    """Top-k eigenpairs of a symmetric matrix, ascending (GPU subspace iteration).

    GPU replacement for ``Node.top_k_eigenvectors`` (distributed.py:22-29:
    ``eigh(matrix, eigvals=(N-k, N-1))[1]``) that also returns the eigenvalues.
    Like scipy's ``?syevr`` call it takes any symmetric S of any size d and any
    1 <= k <= d (ValueError outside, like scipy's subset_by_index check): k > 128 runs
    in locked blocks of p - 16 pairs, an indefinite S is detected from the Ritz values
    and solved as S + sigma I, and a d the kernels cannot take as is (d % 4 != 0,
    d < 16, a subspace wider than d) is staged by the library in a padded copy whose
    padding directions never outrank S's own eigenpairs (include/deig.h
    deig_topk_sym_ex).  A float64 S (the reference's dtype) is read in double by the
    image and deflation passes.  Only the lower triangle matters mathematically, but
    the full matrix is read (the SYRK output is bit-exactly symmetric).  ``opts``:
    solver options (``_lib.solver_opts(...)``).
    """
    S = require_device_tensor(S, "topk_eigh", keep_f64=True)
    if S.dim() != 2 or S.shape[0] != S.shape[1]:
        raise ValueError(f"expected a square matrix, got {tuple(S.shape)}")
    d = S.shape[0]
    k = int(k)
    if not 1 <= k <= d:
        raise ValueError(f"k={k} out of range [1, {d}]")
    if check_finite and not bool(torch.isfinite(S).all()):
        raise ValueError("array must not contain infs or NaNs")
    S = _solver_matrix(S)
    q, k0, ldq = _warm(q0, d, S.device)
    pp = int(p) if p else 0
    stype = _lib.DEIG_F64 if S.dtype == torch.float64 else _lib.DEIG_F32
    o = opts if opts is not None else _lib.solver_opts()
    V = _colmajor(d, k, S.device)
    evals = torch.empty(k, dtype=torch.float32, device=S.device)
    sweeps, resid = ctypes.c_int(0), ctypes.c_float(0)
    L = _lib.lib()
    with torch.cuda.device(S.device):
        nbytes = L.deig_topk_workspace_ex(d, k, pp, stype, ctypes.byref(o))
        ws = _workspace(S.device, nbytes)
        rc = L.deig_topk_sym_ex(S.data_ptr(), stype, d, S.stride(0), k, pp, int(max_sweeps),
                                ctypes.c_float(tol), q.data_ptr() if q is not None else None,
                                k0, ldq, V.data_ptr(), d, evals.data_ptr(),
                                ctypes.byref(sweeps), ctypes.byref(resid), ctypes.byref(o),
                                ws.data_ptr(), nbytes, _stream(S.device))
    return _finish(rc, V, evals, sweeps, resid, "deig_topk_sym_ex")


def topk_eigh_batch(Ss, k: int, *, p: int | None = None, tol: float = DEFAULT_TOL,
                    max_sweeps: int = DEFAULT_MAX_SWEEPS, check_finite: bool = True,
                    opts: "_lib.SolverOpts | None" = None) -> list:
    """``topk_eigh`` of W same-shape symmetric matrices at once (the logical workers
    of one GPU, each SlaveNode's top_k_eigenvectors of distributed.py:22-29,
    :42-53): the same results as W ``topk_eigh`` calls, the W problems advanced in
    lockstep on the current stream (two interleaved groups on a second, joined
    stream from d = 2048) with each step's sweeps, Grams, small
    Rayleigh-Ritz solves and updates batched across them (include/deig.h
    deig_topk_sym_batch).  Returns a list of EigResult."""
    Ss = [require_device_tensor(S, "topk_eigh_batch", keep_f64=True) for S in Ss]
    if not Ss:
        return []
    S0 = Ss[0]
    if S0.dim() != 2 or S0.shape[0] != S0.shape[1]:
        raise ValueError(f"expected square matrices, got {tuple(S0.shape)}")
    d, dev, dt = S0.shape[0], S0.device, S0.dtype
    for S in Ss:
        if S.shape != S0.shape or S.device != dev or S.dtype != dt:
            raise ValueError("topk_eigh_batch: every matrix must have the same shape, dtype, device")
        if check_finite and not bool(torch.isfinite(S).all()):
            raise ValueError("array must not contain infs or NaNs")
    k = int(k)
    if not 1 <= k <= d:
        raise ValueError(f"k={k} out of range [1, {d}]")
    mats = [_solver_matrix(S) for S in Ss]
    lds = mats[0].stride(0)
    if any(S.stride(0) != lds for S in mats):
        mats = [S.contiguous() for S in mats]
        lds = d
    W = len(mats)
    pp = int(p) if p else 0
    stype = _lib.DEIG_F64 if dt == torch.float64 else _lib.DEIG_F32
    o = opts if opts is not None else _lib.solver_opts()
    Vs = [_colmajor(d, k, dev) for _ in range(W)]
    evs = [torch.empty(k, dtype=torch.float32, device=dev) for _ in range(W)]
    sweeps = (ctypes.c_int * W)()
    resid = (ctypes.c_float * W)()
    status = (ctypes.c_int * W)()
    vp = ctypes.c_void_p
    S_arr = (vp * W)(*[S.data_ptr() for S in mats])
    V_arr = (vp * W)(*[V.data_ptr() for V in Vs])
    E_arr = (vp * W)(*[e.data_ptr() for e in evs])
    cur = torch.cuda.current_stream(dev)
    L = _lib.lib()
    with torch.cuda.device(dev):
        nbytes = L.deig_topk_batch_workspace(W, d, k, pp, stype, ctypes.byref(o))
        ws = _workspace(dev, nbytes)
        rc = L.deig_topk_sym_batch_ex(W, S_arr, stype, d, lds, k, pp, int(max_sweeps),
                                      ctypes.c_float(tol), V_arr, d, E_arr, sweeps, resid, status,
                                      ctypes.byref(o), ws.data_ptr(), nbytes, cur.cuda_stream)
    _lib.check(rc, "deig_topk_sym_batch_ex")
    if rc != _lib.DEIG_OK:
        warnings.warn(f"deig_topk_sym_batch_ex: {_lib.last_error()}", _lib.NotConvergedWarning,
                      stacklevel=2)
    # each problem's own outcome (status[i]: what deig_topk_sym_ex would have returned)
    return [EigResult(evals=evs[i], V=Vs[i], sweeps=int(sweeps[i]), resid=float(resid[i]),
                      converged=int(status[i]) == _lib.DEIG_OK) for i in range(W)]


def stack_bases(bases) -> torch.Tensor:
    """[V_1, ..., V_m] (each d x k) -> Wt = [V_1^T; ...; V_m^T]  ((m k) x d row-major)."""
    rows = [require_device_tensor(v, "basis").t() for v in bases]
    return torch.cat(rows, dim=0).contiguous()


def projavg_topk(Wt: torch.Tensor, k: int, scale: float, *, p: int | None = None,
                 tol: float = DEFAULT_TOL, max_sweeps: int = DEFAULT_MAX_SWEEPS,
                 q0: torch.Tensor | None = None,
                 opts: "_lib.SolverOpts | None" = None) -> EigResult:
    """Top-k eigenpairs of scale * sum_i V_i V_i^T, never forming the d x d matrix.

    GPU replacement for MasterNode.callback_ (distributed.py:126-130:
    sigma_tilde = sum V V^T / batches_number) followed by the notebook's server
    solve (Online Distributed PCA.ipynb raw line 306).  Wt = stack_bases(...)
    is (m k) x d row-major; rows may carry per-basis weights (online variant).
    """
    Wt = require_device_tensor(Wt, "projavg_topk")
    if Wt.dim() != 2:
        raise ValueError("Wt must be 2-D ((m k) x d)")
    mk, d = Wt.shape
    k = int(k)
    if not 1 <= k <= d:
        raise ValueError(f"k={k} out of range [1, {d}]")
    dp = _pad_dim(d)
    if not p:
        dp = max(dp, default_subspace(max(dp, (min(k, MAX_P) + 15) // 16 * 16), k))
    if dp != d or Wt.stride(1) != 1 or Wt.stride(0) % 4 or Wt.data_ptr() % 16:
        Wp = torch.zeros((mk, dp), dtype=torch.float32, device=Wt.device)
        Wp[:, :d] = Wt
        Wt = Wp
    q, k0, ldq = _warm(q0, d, Wt.device)
    if q is not None and dp != d:
        qp = torch.zeros((dp, k0), dtype=torch.float32, device=Wt.device)
        qp[:d] = q
        q, ldq = qp.t().contiguous().t(), dp
    pp = int(p) if p else default_subspace(dp, k)
    o = opts if opts is not None else _lib.solver_opts()
    V = _colmajor(dp, k, Wt.device)
    evals = torch.empty(k, dtype=torch.float32, device=Wt.device)
    sweeps, resid = ctypes.c_int(0), ctypes.c_float(0)
    L = _lib.lib()
    with torch.cuda.device(Wt.device):
        nbytes = L.deig_projavg_workspace_ex(dp, mk, k, pp, ctypes.byref(o))
        ws = _workspace(Wt.device, nbytes)
        rc = L.deig_projavg_topk_ex(Wt.data_ptr(), dp, mk, Wt.stride(0), ctypes.c_float(scale),
                                    k, pp, int(max_sweeps), ctypes.c_float(tol),
                                    q.data_ptr() if q is not None else None, k0, ldq,
                                    V.data_ptr(), dp, evals.data_ptr(), ctypes.byref(sweeps),
                                    ctypes.byref(resid), ctypes.byref(o), ws.data_ptr(), nbytes,
                                    _stream(Wt.device))
    res = _finish(rc, V, evals, sweeps, resid, "deig_projavg_topk_ex")
    if dp != d:
        res.V = res.V[:d].t().contiguous().t()
    return res


# ---------------------------------------------------------------- Oja
def oja_step(Xb: torch.Tensor, V: torch.Tensor, eta: float) -> torch.Tensor:
    """In-place mini-batch Oja update V <- orth(V + eta/b Xb^T Xb V) (config 4).

    Not in the reference (parity unpinned).  V: (d, k) column-major float32
    (as returned by topk_eigh), k <= 64.  Returns V.
    """
    Xb = _rowmajor_4(require_device_tensor(Xb, "oja_step"), "Xb")
    b, d = Xb.shape
    if V.dim() != 2 or V.shape[0] != d or V.stride(0) != 1 or V.dtype != torch.float32 \
            or V.device != Xb.device:
        raise ValueError("V must be a (d, k) column-major float32 tensor on Xb's device")
    k = V.shape[1]
    L = _lib.lib()
    with torch.cuda.device(Xb.device):
        nbytes = L.deig_oja_workspace(b, d, k)
        ws = _workspace(Xb.device, nbytes)
        rc = L.deig_oja_step_f32(Xb.data_ptr(), b, d, Xb.stride(0), ctypes.c_float(eta),
                                 V.data_ptr(), k, V.stride(1), ws.data_ptr(), nbytes,
                                 _stream(Xb.device))
    _lib.check(rc, "deig_oja_step_f32")
    oja_check(Xb.device, b, d, k)
    return V


def oja_check(device, b: int, d: int, k: int) -> None:
    """Raise ``DeigTimeoutError`` if the last Oja call on this thread's workspace for
    (b, d, k) on ``device`` timed out in a resident hand-off (its basis is NaN);
    synchronises that device's current stream (include/deig.h deig_oja_error)."""
    L = _lib.lib()
    with torch.cuda.device(device):
        nbytes = L.deig_oja_workspace(b, d, k)
        ws = _workspace(device, nbytes)
        rc = L.deig_oja_error(ws.data_ptr(), nbytes, b, d, k, _stream(device))
    _lib.check(rc, "oja")


def oja_steps(X: torch.Tensor, V: torch.Tensor, eta: float, batch: int,
              orth_every: int = 8, algo: str = "auto", check: bool = True) -> torch.Tensor:
    """In-place Oja over the consecutive row batches X[i*batch:(i+1)*batch] (config 4).

    One C call for all batches (no host work in between); the basis is
    re-orthonormalised every ``orth_every`` batches and at the end, which gives the
    span of per-batch orthonormalisation (``oja_step`` in a loop) because the update
    is linear in V.  Rows beyond the last full batch are ignored.  ``algo``
    (include/deig.h DEIG_OJA_*): "auto", "two_pass" or "resident" (Xb read once per
    batch; batch = 4096, d a multiple of 512 up to 3072, k <= 32).  ``check`` (default):
    synchronise and raise ``DeigTimeoutError`` if a resident hand-off timed out (V is
    then NaN); ``check=False`` leaves the call asynchronous - then call ``oja_check``
    before any other op on this thread's stream (they share the workspace that holds
    the timeout word).  Returns V."""
    X = _rowmajor_4(require_device_tensor(X, "oja_steps"), "X")
    n, d = X.shape
    b = int(batch)
    nb = n // b if b > 0 else 0
    if nb < 1:
        raise ValueError(f"need at least one full batch of {batch} rows, got {n} rows")
    if V.dim() != 2 or V.shape[0] != d or V.stride(0) != 1 or V.dtype != torch.float32 \
            or V.device != X.device:
        raise ValueError("V must be a (d, k) column-major float32 tensor on X's device")
    k = V.shape[1]
    L = _lib.lib()
    with torch.cuda.device(X.device):
        nbytes = L.deig_oja_workspace(b, d, k)
        ws = _workspace(X.device, nbytes)
        rc = L.deig_oja_steps_ex(X.data_ptr(), nb, b, d, X.stride(0), ctypes.c_float(eta),
                                 V.data_ptr(), k, V.stride(1), int(orth_every),
                                 _lib.OJA_ALGOS[algo], ws.data_ptr(), nbytes, _stream(X.device))
    _lib.check(rc, "deig_oja_steps_ex")
    if check:
        oja_check(X.device, b, d, k)
    return V


# ---------------------------------------------------------------- sweep
def sym_apply(S: torch.Tensor, Q: torch.Tensor, algo: str = "auto", alpha: float = 1.0,
              out: torch.Tensor | None = None, prepared: bool = False,
              round_q: bool = False, fast: bool = False, half: bool = False,
              kernel_only: bool = False) -> torch.Tensor:
    """Y = alpha * S Q for symmetric S (d x d) and Q (d x p, p % 16 == 0, p <= 128):
    one subspace-iteration sweep of ``topk_eigh`` (include/deig.h DEIG_SWEEP_*):
    algo "bf16x6" (default via "auto") or "fp32".  ``prepared=True`` (bf16x6) reuses
    the sweep image of S left in this stream's workspace by the previous call with
    the same S and p (DEIG_SWEEP_PREPARED), as the solver does between sweeps.
    ``round_q=True`` (bf16x6, the solver's mode, DEIG_SWEEP_ROUND_Q): Q (contiguous,
    modified in place) is rounded to its two leading bf16 pieces and Y = alpha S Q'
    is formed from five bf16 products.  ``fast=True`` (implies round_q; the solver's
    early-sweep mode, DEIG_SWEEP_FAST): S is also taken as its two leading bf16
    pieces, three products, ~2^-16 relative.  ``half=True`` (implies fast; the
    solver's first sweeps, DEIG_SWEEP_HALF, p >= 64): S and Q as their leading bf16
    piece alone, one product, ~2^-9 relative.  ``kernel_only=True`` (measurement,
    DEIG_SWEEP_KERNEL_ONLY): only the sweep kernel runs, on the Q image the previous
    call in this stream's workspace left; ``out`` is not written."""
    fast = fast or half
    round_q = round_q or fast
    if algo not in _lib.SWEEP_ALGOS:
        raise ValueError(f"algo must be one of {sorted(_lib.SWEEP_ALGOS)}, got {algo!r}")
    S = require_device_tensor(S, "sym_apply")
    Q = require_device_tensor(Q, "Q")
    d = S.shape[0]
    if S.dim() != 2 or S.shape[1] != d or Q.dim() != 2 or Q.shape[0] != d:
        raise ValueError(f"shape mismatch: S {tuple(S.shape)}, Q {tuple(Q.shape)}")
    p = Q.shape[1]
    if d % 4 or S.stride(1) != 1 or S.stride(0) % 4 or S.data_ptr() % 16:
        raise ValueError("S must be row-major with d % 4 == 0 and a 16-byte aligned, %4 stride")
    if round_q:
        if algo == "fp32" or not Q.is_contiguous() or Q.dtype != torch.float32:
            raise ValueError("round_q needs algo bf16x6/auto and a contiguous float32 Q "
                             "(it is rounded in place)")
    Q = Q.contiguous()
    Y = out if out is not None else torch.empty((d, p), dtype=torch.float32, device=S.device)
    code = _lib.SWEEP_ALGOS[algo]
    if prepared and code != _lib.DEIG_SWEEP_FP32:
        code |= _lib.DEIG_SWEEP_PREPARED
    if round_q:
        code |= _lib.DEIG_SWEEP_ROUND_Q
    if fast:
        code |= _lib.DEIG_SWEEP_FAST
    if half:
        code |= _lib.DEIG_SWEEP_HALF
    if kernel_only:
        if code & 0xff == _lib.DEIG_SWEEP_FP32:
            raise ValueError("kernel_only needs algo bf16x6/auto")
        code |= _lib.DEIG_SWEEP_KERNEL_ONLY | _lib.DEIG_SWEEP_PREPARED
    L = _lib.lib()
    with torch.cuda.device(S.device):
        nbytes = L.deig_sym_apply_workspace(d, p, code)
        ws = _workspace(S.device, nbytes)
        rc = L.deig_sym_apply_f32(S.data_ptr(), d, S.stride(0), Q.data_ptr(), p, Q.stride(0),
                                  Y.data_ptr(), Y.stride(0), ctypes.c_float(alpha), code,
                                  ws.data_ptr(), nbytes, _stream(S.device))
    _lib.check(rc, "deig_sym_apply_f32")
    return Y


def sym_power(S: torch.Tensor, Q: torch.Tensor, cs: torch.Tensor, steps: int,
              out: torch.Tensor | None = None, prepared: bool = False,
              round_q: bool = False, fast: bool = False, half: bool = False) -> torch.Tensor:
    """``steps`` sweeps of the solver's power chain (include/deig.h
    deig_sym_power_f32): Y = S Q, then Q_j <- cs_j Y_j on the columns with
    cs_j > 0, each step fused into the sweep's split-K reduction with the next
    sweep's Q image, as between the Rayleigh-Ritz steps of ``topk_eigh``.  Q
    (contiguous float32, d x p) is updated in place; returns Y = S Q_{steps-1}.
    Flags as for ``sym_apply`` (bf16x6 only)."""
    fast = fast or half
    round_q = round_q or fast
    S = require_device_tensor(S, "sym_power")
    Q = require_device_tensor(Q, "Q")
    d = S.shape[0]
    if S.dim() != 2 or S.shape[1] != d or Q.dim() != 2 or Q.shape[0] != d:
        raise ValueError(f"shape mismatch: S {tuple(S.shape)}, Q {tuple(Q.shape)}")
    p = Q.shape[1]
    if d % 4 or S.stride(1) != 1 or S.stride(0) % 4 or S.data_ptr() % 16:
        raise ValueError("S must be row-major with d % 4 == 0 and a 16-byte aligned, %4 stride")
    if not Q.is_contiguous() or Q.dtype != torch.float32:
        raise ValueError("Q must be a contiguous float32 tensor (updated in place)")
    cs = cs.to(device=S.device, dtype=torch.float32).contiguous()
    if cs.numel() != p:
        raise ValueError(f"cs must hold p = {p} column scales")
    Y = out if out is not None else torch.empty((d, p), dtype=torch.float32, device=S.device)
    code = _lib.DEIG_SWEEP_BF16X6
    if prepared:
        code |= _lib.DEIG_SWEEP_PREPARED
    if round_q:
        code |= _lib.DEIG_SWEEP_ROUND_Q
    if fast:
        code |= _lib.DEIG_SWEEP_FAST
    if half:
        code |= _lib.DEIG_SWEEP_HALF
    L = _lib.lib()
    with torch.cuda.device(S.device):
        nbytes = L.deig_sym_apply_workspace(d, p, code)
        ws = _workspace(S.device, nbytes)
        rc = L.deig_sym_power_f32(S.data_ptr(), d, S.stride(0), Q.data_ptr(), p, Q.stride(0),
                                  Y.data_ptr(), Y.stride(0), cs.data_ptr(), int(steps), code,
                                  ws.data_ptr(), nbytes, _stream(S.device))
    _lib.check(rc, "deig_sym_power_f32")
    return Y


# ---------------------------------------------------------------- projection
def project(X: torch.Tensor, W: torch.Tensor) -> torch.Tensor:
    """Y = X W  (NB:345 ``X @ matrix_w``): X (n, d) row-major, W (d, k) any layout."""
    X = _rowmajor_4(require_device_tensor(X, "project"), "X")
    W = require_device_tensor(W, "matrix_w")
    n, dp = X.shape
    d, k = W.shape
    if d > dp or (dp != d and dp != (d + 3) // 4 * 4):
        raise ValueError(f"shape mismatch: X has {dp} columns, W has {d} rows")
    if dp != d:
        Wp = torch.zeros((dp, k), dtype=torch.float32, device=W.device)
        Wp[:d] = W
        W = Wp
    W = W.t().contiguous().t()  # column-major
    Y = torch.empty((n, k), dtype=torch.float32, device=X.device)
    L = _lib.lib()
    with torch.cuda.device(X.device):
        nbytes = L.deig_project_workspace(n, dp, k)
        ws = _workspace(X.device, nbytes)
        rc = L.deig_project_f32(X.data_ptr(), n, dp, X.stride(0), W.data_ptr(), k, W.stride(1),
                                Y.data_ptr(), Y.stride(0), ws.data_ptr(), nbytes,
                                _stream(X.device))
    _lib.check(rc, "deig_project_f32")
    return Y


# ---------------------------------------------------------------- building block
def gemm_skinny(A: torch.Tensor, B: torch.Tensor, trans_a: bool, alpha: float = 1.0,
                beta: float = 0.0, C: torch.Tensor | None = None) -> torch.Tensor:
    """C = alpha * op(A) @ B + beta * C on the solvers' skinny fp32-MFMA kernel.

    trans_a: A is (K, M) and op(A) = A^T; else A is (M, K).  B is (K, N) with
    N % 16 == 0 and N <= 256.  All row-major float32 on one device."""
    A = require_device_tensor(A, "A")
    B = require_device_tensor(B, "B")
    K, M = (A.shape if trans_a else (A.shape[1], A.shape[0]))
    N = B.shape[1]
    if B.shape[0] != K:
        raise ValueError("inner dimensions differ")
    if C is None:
        C = torch.zeros((M, N), dtype=torch.float32, device=A.device)
    L = _lib.lib()
    with torch.cuda.device(A.device):
        nbytes = L.deig_gemm_skinny_workspace(M, N, K)
        ws = _workspace(A.device, nbytes)
        rc = L.deig_gemm_skinny_f32(int(trans_a), A.data_ptr(), A.stride(0), B.data_ptr(),
                                    B.stride(0), C.data_ptr(), C.stride(0), M, N, K,
                                    ctypes.c_float(alpha), ctypes.c_float(beta), ws.data_ptr(),
                                    nbytes, _stream(A.device))
    _lib.check(rc, "deig_gemm_skinny_f32")
    return C
