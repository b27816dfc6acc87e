"""Covariance of any n in one Sigma_hat: the split pass's row-chunk loop and
DEIG_SYRK_ACCUMULATE, against the float64 oracle of ALL rows.

The reference forms Sigma_hat = X^T X / n of a shard of any size in one call
(reference/distributed.py:66-69).  Here a shard larger than the caller's workspace
runs the split pass in row chunks that accumulate into S (csrc/syrk_split.hip
syrk_split_launch: beta = 1 for every chunk after the first, one diag_corr_kernel
per chunk adding that chunk's lo^2 diagonal term), and rows that arrive in blocks
(or exceed HBM: bench.py time_to_eigenspace_16M_rows_1gpu) are streamed through
``sigma_hat(..., accumulate=True)`` (DEIG_SYRK_ACCUMULATE) into one S.

Bars: max |S - S_ref| <= 2e-6 max |S_ref| (north_star SYRK bar, tests/test_gpu_kernels.py),
bit symmetry, and the MEAN relative diagonal error <= 5e-7: the lo*lo term the
split3 products drop is a -2^-18 ~ -3.8e-6 relative bias on the diagonal, so a
chunk whose diag_corr_kernel contribution is lost (or overwritten) moves that mean
by ~-3.8e-6 x its share of the rows, while the random fp32 rounding averages out.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import ref_cpu

pytestmark = pytest.mark.gpu

REL = 2e-6
DIAG_BIAS = 5e-7


def _samples(n, d, seed):
    rng = np.random.default_rng(seed)
    # a non-zero mean (uncentered covariance, like the reference's pixel data) and
    # values that are not bf16-exact, so every chunk's lo pieces matter
    return (rng.standard_normal((n, d)) * 3.0 + 1.0).astype(np.float32)


def _check(Sg, X32, what, Sr=None):
    Sg = Sg.astype(np.float64)
    if Sr is None:
        Sr = ref_cpu.sigma_hat(X32.astype(np.float64))
    err = np.abs(Sg - Sr).max() / np.abs(Sr).max()
    assert err <= REL, f"{what}: max rel err {err:.3e} > {REL:.0e}"
    bias = float(np.mean((np.diag(Sg) - np.diag(Sr)) / np.diag(Sr)))
    assert abs(bias) <= DIAG_BIAS, f"{what}: mean diagonal bias {bias:.3e} (lo^2 correction lost?)"
    assert np.array_equal(Sg, Sg.T), f"{what}: S must be bit-exactly symmetric"


def _syrk_raw(x, alpha, S, code, ws, nbytes):
    from distributed_eigenspaces_amd import _lib
    L = _lib.lib()
    n, d = x.shape
    return L.deig_syrk_f32_ex(x.data_ptr(), n, d, x.stride(0), ctypes.c_float(alpha), S.data_ptr(),
                              S.stride(0), code, ws.data_ptr() if ws is not None else None, nbytes,
                              torch.cuda.current_stream().cuda_stream)


@pytest.mark.parametrize("d", [8192, 8000])
def test_split_pass_chunk_loop(d, cuda):
    """d > 4096 (the split pass, the default there) with a workspace holding 4096
    rows of the split image: n = 16359 runs 4 chunks (4096, 4096, 4096, 4071 rows; the
    last one partial, n % 32 = 7) accumulating into S.  d = 8000 is ragged in the
    256-feature panel.  (n = 4071 in r04a: the one-chunk run itself landed at 3e-6,
    the split3 error is ~1/sqrt(n): the 2e-6 bar needs n >~ 8k rows.)"""
    from distributed_eigenspaces_amd import _lib
    L = _lib.lib()
    n, chunk = 16359, 4096
    X = _samples(n, d, seed=d)
    x = torch.from_numpy(X).to(cuda)
    S = torch.full((d, d), float("nan"), dtype=torch.float32, device=cuda)
    nbytes = L.deig_syrk_workspace_ex(chunk, d, _lib.DEIG_SYRK_SPLIT3)  # chunk rows of XP
    assert nbytes < L.deig_syrk_workspace_ex(n, d, _lib.DEIG_SYRK_SPLIT3), "one chunk would hold all rows"
    ws = torch.full((nbytes,), 0xFF, dtype=torch.uint8, device=cuda)  # NaN-poisoned workspace
    rc = _syrk_raw(x, 1.0 / n, S, _lib.DEIG_SYRK_SPLIT3, ws, nbytes)
    _lib.check(rc, "deig_syrk_f32_ex")
    torch.cuda.synchronize()
    Sr = ref_cpu.sigma_hat(X.astype(np.float64))
    _check(S.cpu().numpy(), X, f"split pass, {-(-n // chunk)} chunks, d={d}", Sr)
    # the same rows with the default workspace (one chunk): the same bar
    S1 = torch.empty_like(S)
    nb1 = L.deig_syrk_workspace_ex(n, d, _lib.DEIG_SYRK_SPLIT3)
    ws1 = torch.empty(nb1, dtype=torch.uint8, device=cuda)
    _lib.check(_syrk_raw(x, 1.0 / n, S1, _lib.DEIG_SYRK_SPLIT3, ws1, nb1), "deig_syrk_f32_ex")
    torch.cuda.synchronize()
    _check(S1.cpu().numpy(), X, f"split pass, one chunk, d={d}", Sr)
    # below the one-chunk minimum: an error, not a silent fallback
    assert _syrk_raw(x, 1.0 / n, S, _lib.DEIG_SYRK_SPLIT3, ws, 4096) == _lib.DEIG_EWORKSPACE


@pytest.mark.parametrize("d", [8192, 8000, 3072, 2048])
def test_accumulate_row_blocks(d, cuda):
    """Four ragged row blocks streamed through sigma_hat(..., accumulate=True) into
    one S with alpha = 1 / n_total: the covariance of all rows (d = 2048 runs the
    fused-split kernel with beta = 1, d > 2048 the split pass).  Variant 2: the first
    block without accumulate overwrites whatever S held."""
    import distributed_eigenspaces_amd as de
    sizes = [1000, 1031, 997, 1043]
    n = sum(sizes)
    X = _samples(n, d, seed=3 * d + 1)
    x = torch.from_numpy(X).to(cuda)
    bounds = np.cumsum([0] + sizes)
    S = torch.zeros((d, d), dtype=torch.float32, device=cuda)
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        de.sigma_hat(x[lo:hi], alpha=1.0 / n, out=S, accumulate=True)
    torch.cuda.synchronize()
    _check(S.cpu().numpy(), X, f"accumulate 4 blocks, d={d}")
    S2 = torch.full((d, d), 1e30, dtype=torch.float32, device=cuda)
    for i, (lo, hi) in enumerate(zip(bounds[:-1], bounds[1:])):
        de.sigma_hat(x[lo:hi], alpha=1.0 / n, out=S2, algo="split3", accumulate=i > 0)
    torch.cuda.synchronize()
    _check(S2.cpu().numpy(), X, f"overwrite + accumulate 3 blocks, d={d}")


def test_accumulate_rejects_unsupported(cuda):
    """accumulate is the split3 path's: fp32 algorithm, no out, or a float64 (shifted)
    input raise instead of silently overwriting."""
    import distributed_eigenspaces_amd as de
    x = torch.randn(64, 256, device=cuda)
    S = torch.zeros(256, 256, device=cuda)
    with pytest.raises(ValueError):
        de.sigma_hat(x, out=S, algo="fp32", accumulate=True)
    with pytest.raises(ValueError):
        de.sigma_hat(x, accumulate=True)
    with pytest.raises(ValueError):
        de.sigma_hat(x.double(), out=S, accumulate=True)


@pytest.mark.parametrize("d,rows", [(2048, 16384), (3072, 8192)])
def test_full_time_to_eigenspace_helper(d, rows, cuda):
    """bench.py's 16M-row helper (``time_to_eigenspace_16M_rows_1gpu``) at reduced
    size: 4 row blocks regenerated in place and streamed through ONE S (block 0
    overwrites, blocks 1-3 accumulate, each launch timed once).  S must be the
    covariance of ALL rows (r04's helper accumulated every block twice: S = 2
    Sigma_hat), and the top-k pairs the reference's (distributed.py:66-69 then
    :22-29) at the north_star bars.  d = 2048 runs the fused-split kernel, d = 3072
    the split pass."""
    import bench
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    k, blocks = 16, 4
    U = synthetic.planted_basis(d, k, seed=0, device=cuda)
    gen = bench.spiked_block_fn(synthetic, U)
    X = torch.empty((rows, d), dtype=torch.float32, device=cuda)
    parts = []
    for b in range(blocks):
        gen(b, X)
        parts.append(X.cpu().numpy().copy())
    Xall = np.concatenate(parts)
    out = bench.full_time_to_eigenspace(de, gen, X, U, blocks * rows, k,
                                        torch.cuda.current_stream(), keep_S=True)
    assert out["blocks"] == blocks and len(out["covariance_ms_per_block"]) == blocks
    assert out["sigma_hat_rel_err_vs_f64_sampled"] <= REL
    assert out["evals_rel_err_vs_f64_rayleigh_all_rows"] <= 1e-5
    Sr = ref_cpu.sigma_hat(Xall.astype(np.float64))
    _check(out["S"].cpu().numpy(), Xall, f"16M-row helper at d={d}, {blocks} x {rows} rows", Sr)
    w, V = ref_cpu.top_k_eigh(Sr, k)
    ev = np.array(out["evals"])
    assert np.max(np.abs(ev - w) / np.abs(w)) <= 1e-5
    assert ref_cpu.projector_distance(out["V"].cpu().numpy(), V) <= 1e-4
