"""The C-ABI library loads and exports every symbol include/deig.h declares (CPU)."""
import ctypes

import pytest

from distributed_eigenspaces_amd import _lib


def test_header_symbols_exported():
    L = _lib.lib()
    syms = _lib.header_symbols()
    assert len(syms) >= 13
    for s in syms:
        assert hasattr(L, s), f"libdeig.so does not export {s}"
        assert s in _lib.SIGNATURES, f"no ctypes signature for {s}"


def test_header_constants_match_bindings():
    """Every #define DEIG_<NAME> <int> in include/deig.h has the same value in _lib."""
    import os
    import re
    hdr = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                       "deig.h")
    defs = dict(re.findall(r"^#define\s+(DEIG_[A-Z0-9_]+)\s+\(?(-?(?:0x[0-9a-fA-F]+|\d+))\)?\s*$",
                           open(hdr).read(), re.M))
    assert "DEIG_SWEEP_ROUND_Q" in defs and "DEIG_SWEEP_PREPARED" in defs
    assert "DEIG_SWEEP_FAST" in defs
    checked = 0
    for name, val in defs.items():
        if hasattr(_lib, name):
            assert getattr(_lib, name) == int(val, 0), f"{name}: header {val} != _lib"
            checked += 1
    assert checked >= 10


def test_version_and_error_string():
    L = _lib.lib()
    assert L.deig_version() == 0x000600
    assert isinstance(_lib.last_error(), str)


def test_workspace_queries():
    L = _lib.lib()
    # config-3 shard: d=8192 -> 528 tiles = 2 x 256 + 16 remainder tiles:
    # one flush slab + two remainder slabs of 256 x 256 fp32 per CU
    n, d = 1 << 21, 8192
    slabs = 3 * 256 * 256 * 256 * 4
    assert L.deig_syrk_workspace_ex(n, d, _lib.DEIG_SYRK_FP32) == slabs
    # split3 adds the bf16 hi/lo image of the shard (4 B per sample value, one chunk)
    # split3: one flush slab per CU + the 16 remainder tiles cut into 16 K-synchronous
    # segments (16 x 16 slabs), see syrk_split.hip remainder_segments()
    ws = L.deig_syrk_workspace_ex(n, d, _lib.DEIG_SYRK_SPLIT3)
    split_slabs = (256 + 16 * 16) * 256 * 256 * 4
    assert n * d * 4 + split_slabs <= ws <= n * d * 4 + split_slabs + (16 << 20)
    assert L.deig_syrk_workspace(n, d) == ws  # default = auto = split3 at n >= 1024
    assert L.deig_syrk_workspace(1000, 256) == L.deig_syrk_workspace_ex(1000, 256,
                                                                        _lib.DEIG_SYRK_FP32)
    assert L.deig_syrk_workspace(1000, 256) > 0
    for d, k in [(64, 4), (3072, 16), (8192, 64), (16384, 128)]:
        p = L.deig_default_subspace(d, k)
        assert p % 16 == 0 and k <= p <= 128
        assert L.deig_topk_workspace(d, k, 0) >= d * 2 * p * 4
        assert L.deig_projavg_workspace(d, 8 * k, k, 0) > 0
    assert L.deig_oja_workspace(4096, 3072, 32) > 3072 * 32 * 4
    assert L.deig_project_workspace(60000, 1024, 2) > 0


def test_invalid_arguments_rejected_before_any_gpu_work():
    L = _lib.lib()
    rc = L.deig_syrk_f32(None, 0, 64, 64, ctypes.c_float(1.0), None, 64, None, 0, None)
    assert rc == _lib.DEIG_EINVAL and "n must be" in _lib.last_error()
    rc = L.deig_syrk_f32(None, 10, 6, 8, ctypes.c_float(1.0), None, 8, None, 0, None)
    assert rc == _lib.DEIG_EINVAL
    with pytest.raises(ValueError):
        _lib.check(_lib.DEIG_EINVAL, "x")
    with pytest.raises(_lib.DeigError):
        _lib.check(_lib.DEIG_EHIP, "x")


def test_no_cpu_fallback():
    import torch

    import distributed_eigenspaces_amd as de
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        de.sigma_hat(torch.ones(4, 4))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        de.topk_eigh(torch.eye(16), 2)


def test_workspace_fused_split_variant():
    """d <= 2048 uses the fused split, which stages X itself: no image of the shard in
    the workspace; d > 2048 (config 2's 3072 since r04) runs the split pass and its
    image."""
    L = _lib.lib()
    n, d = 1 << 20, 2048
    ws = L.deig_syrk_workspace_ex(n, d, _lib.DEIG_SYRK_SPLIT3)
    assert 0 < ws < n * d * 4 // 10  # slabs only (the image would be n * d * 4)
    assert L.deig_syrk_workspace_ex(n, 3072, _lib.DEIG_SYRK_SPLIT3) >= n * 3072 * 4
    assert L.deig_syrk_workspace_ex(1 << 21, 8192, _lib.DEIG_SYRK_SPLIT3) >= (1 << 21) * 8192 * 4


def test_solver_opts_mirror_matches_header():
    """The ctypes mirror lists deig_solver_opts' fields in the header's order with the
    header's C types (a field added on one side only shifts every later one)."""
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "include", "deig.h")).read()
    body = re.search(r"typedef struct deig_solver_opts \{(.*?)\} deig_solver_opts;", hdr, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = re.findall(r"\b(int|float)\s+(\w+)\s*;", body)
    ctype = {"int": ctypes.c_int, "float": ctypes.c_float}
    assert [(n, ctype[t]) for t, n in fields] == list(_lib.SolverOpts._fields_)


def test_solver_opts_struct_and_defaults():
    """deig_solver_opts: the ctypes mirror has the C size (the library checks it) and
    the defaults the r02 environment knobs had."""
    o = _lib.solver_opts()
    assert o.size == ctypes.sizeof(_lib.SolverOpts)
    assert (o.chebyshev, o.deflate, o.deflate_early, o.rr_every) == (1, 1, 1, 0)
    assert o.cheb_above < 0 and abs(o.fast_until - 1e-3) < 1e-9  # cheb_above: per solve
    assert abs(o.round_until - 1e-4) < 1e-9 and o.jacobi_early_sweeps == -1
    assert abs(o.half_until - 1e-2) < 1e-9
    bad = _lib.SolverOpts()
    bad.size = 4
    V = ctypes.c_int(0)
    rc = _lib.lib().deig_topk_sym_ex(16, _lib.DEIG_F32, 64, 64, 2, 16, 10, ctypes.c_float(1e-6),
                                     None, 0, 0, 16, 64, 16, ctypes.byref(V), None,
                                     ctypes.byref(bad), 16, 1 << 20, None)
    assert rc == _lib.DEIG_EINVAL and "size" in _lib.last_error()


def test_library_reads_no_environment():
    """No A/B knobs in the shipped library: no getenv in csrc/, none imported by the .so."""
    import os
    import shutil
    import subprocess
    csrc = os.path.join(os.path.dirname(_lib.HERE), "distributed_eigenspaces_amd", "csrc")
    for root, _, files in os.walk(csrc):  # csrc/ab/ holds the A/B-only sources
        for f in files:
            assert "getenv" not in open(os.path.join(root, f)).read(), os.path.join(root, f)
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    if os.path.exists(nm):
        out = subprocess.run([nm, "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True,
                             text=True).stdout
        assert "getenv" not in out


def test_general_k_and_shift_workspaces():
    """k > 128 (block locking) and the mean-shifted covariance have workspace queries."""
    L = _lib.lib()
    assert L.deig_default_subspace(3072, 256) == 128
    assert L.deig_default_subspace(1024, 200) == 128
    o = _lib.solver_opts()
    w256 = L.deig_topk_workspace_ex(3072, 256, 0, _lib.DEIG_F64, ctypes.byref(o))
    assert w256 >= L.deig_topk_workspace(3072, 112, 128) > 0
    assert L.deig_projavg_workspace_ex(3072, 8 * 256, 256, 0, ctypes.byref(o)) > 0
    n, d = 7500, 1024
    ws = L.deig_syrk_shift_workspace(n, d, _lib.DEIG_F64)
    assert ws >= n * d * 4 + d * d * 4  # fp32 copy of X - mu and the centred image
