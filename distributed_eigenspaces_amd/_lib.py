"""ctypes binding of libdeig.so (the C ABI declared in include/deig.h).

ctypes releases the GIL for the duration of each call, so several
``my_threading.Slave`` worker threads can drive the GPU concurrently.
There is no CPU fallback: if the library is missing the import of an op raises.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import re
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# DEIG_LIB_PATH: an A/B variant built by tools/ (_build.build_library(defines=...));
# the product default is the in-tree libdeig.so.
LIB_PATH = os.environ.get("DEIG_LIB_PATH") or os.path.join(HERE, "libdeig.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "deig.h")

DEIG_OK = 0
DEIG_NOT_CONVERGED = 1
DEIG_EINVAL = -1
DEIG_EHIP = -2
DEIG_EWORKSPACE = -3
DEIG_ETIMEOUT = -4
DEIG_SYRK_AUTO = 0
DEIG_SYRK_SPLIT3 = 1
DEIG_SYRK_FP32 = 2
DEIG_SYRK_ACCUMULATE = 0x100
SYRK_ALGOS = {"auto": DEIG_SYRK_AUTO, "split3": DEIG_SYRK_SPLIT3, "fp32": DEIG_SYRK_FP32}
DEIG_SWEEP_AUTO = 0
DEIG_SWEEP_BF16X6 = 1
DEIG_SWEEP_FP32 = 2
DEIG_SWEEP_PREPARED = 0x100
DEIG_SWEEP_ROUND_Q = 0x200
DEIG_SWEEP_FAST = 0x400
DEIG_SWEEP_HALF = 0x1000
DEIG_SWEEP_KERNEL_ONLY = 0x800
SWEEP_ALGOS = {"auto": DEIG_SWEEP_AUTO, "bf16x6": DEIG_SWEEP_BF16X6, "fp32": DEIG_SWEEP_FP32}
DEIG_U8_RAW = 0
DEIG_U8_GRAY3 = 1
U8_MODES = {"raw": DEIG_U8_RAW, "gray": DEIG_U8_GRAY3}
DEIG_F32 = 0
DEIG_F64 = 1
DEIG_OJA_AUTO = 0
DEIG_OJA_TWO_PASS = 1
DEIG_OJA_RESIDENT = 2
OJA_ALGOS = {"auto": DEIG_OJA_AUTO, "two_pass": DEIG_OJA_TWO_PASS, "resident": DEIG_OJA_RESIDENT}


class SolverOpts(ctypes.Structure):
    """``deig_solver_opts`` (include/deig.h); build with :func:`solver_opts`."""

    _fields_ = [
        ("size", ctypes.c_int),
        ("sweep_algo", ctypes.c_int),
        ("rr_every", ctypes.c_int),
        ("chebyshev", ctypes.c_int),
        ("cheb_above", ctypes.c_float),
        ("deflate", ctypes.c_int),
        ("deflate_early", ctypes.c_int),
        ("jacobi_early_sweeps", ctypes.c_int),
        ("jacobi_early_above", ctypes.c_float),
        ("fast_until", ctypes.c_float),
        ("round_until", ctypes.c_float),
        ("debug", ctypes.c_int),
        ("half_until", ctypes.c_float),
    ]

_c_i64 = ctypes.c_int64
_c_sz = ctypes.c_size_t
_vp = ctypes.c_void_p
_fp = ctypes.c_void_p  # device pointers are passed as integers

SIGNATURES = {
    "deig_version": (ctypes.c_int, []),
    "deig_shutdown": (None, []),
    "deig_oja_error": (ctypes.c_int, [_vp, _c_sz, _c_i64, _c_i64, ctypes.c_int, _vp]),
    "deig_last_error": (ctypes.c_char_p, []),
    "deig_syrk_f32": (ctypes.c_int, [_fp, _c_i64, _c_i64, _c_i64, ctypes.c_float, _fp, _c_i64,
                                     _vp, _c_sz, _vp]),
    "deig_syrk_workspace": (_c_sz, [_c_i64, _c_i64]),
    "deig_syrk_f32_ex": (ctypes.c_int, [_fp, _c_i64, _c_i64, _c_i64, ctypes.c_float, _fp,
                                        _c_i64, ctypes.c_int, _vp, _c_sz, _vp]),
    "deig_syrk_workspace_ex": (_c_sz, [_c_i64, _c_i64, ctypes.c_int]),
    "deig_syrk_u8": (ctypes.c_int, [_fp, _c_i64, _c_i64, _c_i64, ctypes.c_int, ctypes.c_double,
                                    _fp, _c_i64, _fp, _c_i64, _vp, _c_sz, _vp]),
    "deig_syrk_u8_workspace": (_c_sz, [_c_i64, _c_i64, ctypes.c_int]),
    "deig_default_subspace": (ctypes.c_int, [_c_i64, ctypes.c_int]),
    "deig_topk_sym_f32": (ctypes.c_int, [_fp, _c_i64, _c_i64, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_float, _fp, ctypes.c_int, _c_i64,
                                         _fp, _c_i64, _fp, ctypes.POINTER(ctypes.c_int),
                                         ctypes.POINTER(ctypes.c_float), _vp, _c_sz, _vp]),
    "deig_topk_workspace": (_c_sz, [_c_i64, ctypes.c_int, ctypes.c_int]),
    "deig_solver_opts_init": (None, [ctypes.POINTER(SolverOpts)]),
    "deig_topk_sym_ex": (ctypes.c_int, [_fp, ctypes.c_int, _c_i64, _c_i64, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_float, _fp, ctypes.c_int, _c_i64,
                                        _fp, _c_i64, _fp, ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_float), ctypes.POINTER(SolverOpts),
                                        _vp, _c_sz, _vp]),
    "deig_topk_workspace_ex": (_c_sz, [_c_i64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(SolverOpts)]),
    "deig_topk_batch_workspace": (_c_sz, [ctypes.c_int, _c_i64, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.POINTER(SolverOpts)]),
    "deig_topk_sym_batch": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp), ctypes.c_int, _c_i64,
                                           _c_i64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_float, ctypes.POINTER(_vp), _c_i64,
                                           ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_float),
                                           ctypes.POINTER(SolverOpts), _vp, _c_sz,
                                           ctypes.POINTER(_vp), _vp]),
    "deig_topk_sym_batch_ex": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp), ctypes.c_int, _c_i64,
                                              _c_i64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_float, ctypes.POINTER(_vp), _c_i64,
                                              ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_int),
                                              ctypes.POINTER(ctypes.c_float),
                                              ctypes.POINTER(ctypes.c_int),
                                              ctypes.POINTER(SolverOpts), _vp, _c_sz, _vp]),
    "deig_projavg_topk_ex": (ctypes.c_int, [_fp, _c_i64, _c_i64, _c_i64, ctypes.c_float,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_float, _fp, ctypes.c_int, _c_i64, _fp,
                                            _c_i64, _fp, ctypes.POINTER(ctypes.c_int),
                                            ctypes.POINTER(ctypes.c_float),
                                            ctypes.POINTER(SolverOpts), _vp, _c_sz, _vp]),
    "deig_projavg_workspace_ex": (_c_sz, [_c_i64, _c_i64, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(SolverOpts)]),
    "deig_syrk_shift": (ctypes.c_int, [_fp, ctypes.c_int, _c_i64, _c_i64, _c_i64, ctypes.c_double,
                                       _fp, _c_i64, _fp, _c_i64, _vp, _c_sz, _vp]),
    "deig_syrk_shift_workspace": (_c_sz, [_c_i64, _c_i64, ctypes.c_int]),
    "deig_projavg_topk_f32": (ctypes.c_int, [_fp, _c_i64, _c_i64, _c_i64, ctypes.c_float,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_float, _fp, ctypes.c_int, _c_i64, _fp,
                                             _c_i64, _fp, ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(ctypes.c_float), _vp, _c_sz, _vp]),
    "deig_projavg_workspace": (_c_sz, [_c_i64, _c_i64, ctypes.c_int, ctypes.c_int]),
    "deig_oja_step_f32": (ctypes.c_int, [_fp, _c_i64, _c_i64, _c_i64, ctypes.c_float, _fp,
                                         ctypes.c_int, _c_i64, _vp, _c_sz, _vp]),
    "deig_oja_workspace": (_c_sz, [_c_i64, _c_i64, ctypes.c_int]),
    "deig_oja_steps_f32": (ctypes.c_int, [_fp, _c_i64, _c_i64, _c_i64, _c_i64, ctypes.c_float,
                                          _fp, ctypes.c_int, _c_i64, ctypes.c_int, _vp, _c_sz,
                                          _vp]),
    "deig_oja_steps_ex": (ctypes.c_int, [_fp, _c_i64, _c_i64, _c_i64, _c_i64, ctypes.c_float,
                                         _fp, ctypes.c_int, _c_i64, ctypes.c_int, ctypes.c_int, _vp,
                                         _c_sz, _vp]),
    "deig_sym_apply_f32": (ctypes.c_int, [_fp, _c_i64, _c_i64, _fp, ctypes.c_int, _c_i64, _fp,
                                          _c_i64, ctypes.c_float, ctypes.c_int, _vp, _c_sz, _vp]),
    "deig_sym_power_f32": (ctypes.c_int, [_fp, _c_i64, _c_i64, _fp, ctypes.c_int, _c_i64, _fp,
                                          _c_i64, _fp, ctypes.c_int, ctypes.c_int, _vp, _c_sz,
                                          _vp]),
    "deig_sym_apply_workspace": (_c_sz, [_c_i64, ctypes.c_int, ctypes.c_int]),
    "deig_project_f32": (ctypes.c_int, [_fp, _c_i64, _c_i64, _c_i64, _fp, ctypes.c_int, _c_i64,
                                        _fp, _c_i64, _vp, _c_sz, _vp]),
    "deig_project_workspace": (_c_sz, [_c_i64, _c_i64, ctypes.c_int]),
    "deig_gemm_skinny_f32": (ctypes.c_int, [ctypes.c_int, _fp, _c_i64, _fp, _c_i64, _fp, _c_i64,
                                            _c_i64, _c_i64, _c_i64, ctypes.c_float,
                                            ctypes.c_float, _vp, _c_sz, _vp]),
    "deig_gemm_skinny_workspace": (_c_sz, [_c_i64, _c_i64, _c_i64]),
}

_lock = threading.Lock()
_lib = None


class DeigError(RuntimeError):
    """A libdeig call failed (HIP error or workspace problem)."""


class DeigTimeoutError(DeigError):
    """A resident Oja run's hand-off waited past its bound (DEIG_ETIMEOUT): the basis
    it wrote is NaN (CUs held by other work kept its grid from being co-resident)."""


class NotConvergedWarning(RuntimeWarning):
    """The eigensolver stopped at max_sweeps above its residual tolerance."""


def header_symbols(path: str = HEADER):
    """Function names declared in include/deig.h."""
    txt = open(path).read()
    return sorted(set(re.findall(r"\b(deig_[a-z0-9_]+)\s*\(", txt)))


def lib() -> ctypes.CDLL:
    """Load libdeig.so (once).  Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} is missing: build it with `python __graft_entry__.py build` "
                    "(hipcc, gfx950).  There is no CPU fallback.")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
            # free the library's pinned host blocks while the HIP runtime is alive:
            # Python's atexit runs before the C runtime's exit handlers (and the HIP
            # runtime's teardown), include/deig.h deig_shutdown
            atexit.register(_shutdown)
    return _lib


def _shutdown():
    if _lib is not None:
        try:
            _lib.deig_shutdown()
        except Exception:  # noqa: BLE001 - never raise from an exit handler
            pass


def solver_opts(**fields) -> SolverOpts:
    """Solver options: the library defaults (deig_solver_opts_init) with ``fields``
    overridden; DEIG_DEBUG=1 in the environment turns on the per-RR trace."""
    o = SolverOpts()
    lib().deig_solver_opts_init(ctypes.byref(o))
    if os.environ.get("DEIG_DEBUG", "") == "1":
        o.debug = 1
    for name, value in fields.items():
        if value is not None:
            setattr(o, name, value)
    return o


def last_error() -> str:
    msg = lib().deig_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> int:
    """Map a libdeig return code to Python exceptions (0 and NOT_CONVERGED pass)."""
    if rc in (DEIG_OK, DEIG_NOT_CONVERGED):
        return rc
    msg = f"{what}: {last_error()} (code {rc})"
    if rc == DEIG_EINVAL:
        raise ValueError(msg)
    if rc == DEIG_ETIMEOUT:
        raise DeigTimeoutError(msg)
    raise DeigError(msg)
