"""Exact uint8 covariance (fused ingest) against the float64
oracle on the reference's own preprocessing: raw bytes, and the CIFAR grayscale
``data.mean(axis=3).reshape(n, -1)`` of distributed.py:170-173 followed by
distributed.py:59-70 (ref_cpu.sigma_hat).  The GPU sums are exact integers, so
the fp32 result must be the correctly rounded float64 value (<= 1 ulp apart from
the oracle's own float64 rounding) and the fp64 result must agree to ~1e-15."""
import numpy as np
import pytest
import torch

from oracle import ref_cpu

pytestmark = pytest.mark.gpu
ULP32 = 2.0 ** -23


def _check32(S, ref):
    S = S.cpu().numpy().astype(np.float64)
    rel = np.abs(S - ref) / np.maximum(np.abs(ref), 1e-30)
    assert rel.max() <= 1.01 * ULP32, rel.max()
    assert np.array_equal(S, S.T)


@pytest.mark.parametrize("n,d", [(1, 4), (63, 64), (65, 128), (1000, 100), (5000, 1024),
                                 (6250, 3072), (777, 260)])
def test_raw_bytes_exact(n, d, cuda):
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(n + d)
    X = rng.integers(0, 256, (n, d), dtype=np.uint8)
    S = de.linalg.sigma_hat_u8(torch.from_numpy(X).to(cuda))
    _check32(S, ref_cpu.sigma_hat(X.astype(np.float64)))


@pytest.mark.parametrize("n,hw", [(50, 32), (1000, 32), (333, 8), (4097, 16)])
def test_gray_pixels_exact(n, hw, cuda):
    """N x H x W x 3 (CIFAR layout) -> grayscale fused into the covariance."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(n * hw)
    img = rng.integers(0, 256, (n, hw, hw, 3), dtype=np.uint8)
    S = de.sigma_hat(torch.from_numpy(img).to(cuda))  # uint8 dispatch, 4-D -> gray
    ref = ref_cpu.sigma_hat(img.mean(axis=3).reshape(n, -1))
    _check32(S, ref)
    S64 = de.linalg.sigma_hat_u8(torch.from_numpy(img).to(cuda), dtype=torch.float64)
    np.testing.assert_allclose(S64.cpu().numpy(), ref, rtol=1e-14, atol=0)


def test_extremes_and_long_shard(cuda):
    """All-0 / all-255 columns (largest |y| and |t|) and 200k rows (> one int32
    segment of 65536 rows per item): still exact."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(3)
    n, d = 200_000, 256
    X = rng.integers(0, 256, (n, d), dtype=np.uint8)
    X[:, 0] = 255
    X[:, 1] = 0
    X[::2, 2] = 255
    S = de.linalg.sigma_hat_u8(torch.from_numpy(X).to(cuda), dtype=torch.float64)
    Xf = X.astype(np.float64)  # integer products and sums < 2^53: exact in float64
    ref = (Xf.T @ Xf) / n
    np.testing.assert_allclose(S.cpu().numpy(), ref, rtol=1e-15, atol=0)
    img = rng.integers(0, 256, (70_000, 4, 4, 3), dtype=np.uint8)
    img[:, 0, 0, :] = 255
    img[:, 0, 1, :] = 0
    S = de.linalg.sigma_hat_u8(torch.from_numpy(img).to(cuda), dtype=torch.float64)
    s = img.astype(np.float64).sum(axis=3).reshape(len(img), -1)
    ref = (s.T @ s) / (9.0 * len(img))
    np.testing.assert_allclose(S.cpu().numpy(), ref, rtol=1e-15, atol=0)


def test_strided_rows_and_alpha(cuda):
    """A column slice of a wider uint8 array (row stride != d) and alpha = 1."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(4)
    W = rng.integers(0, 256, (3000, 1040), dtype=np.uint8)
    Xt = torch.from_numpy(W).to(cuda)[:, :1024]
    S = de.linalg.sigma_hat_u8(Xt, alpha=1.0, dtype=torch.float64)
    Wf = W[:, :1024].astype(np.float64)
    ref = Wf.T @ Wf
    np.testing.assert_array_equal(S.cpu().numpy(), ref)


def test_compute_sigma_hat_dropin_uint8(cuda):
    """The drop-in compute_sigma_hat (distributed.py:59-70 surface) takes uint8 host
    arrays: numpy in -> float64 numpy out, the exact integer path underneath."""
    from distributed_eigenspaces_amd import distributed as dd
    rng = np.random.default_rng(5)
    X = rng.integers(0, 256, (2000, 512), dtype=np.uint8)
    S = dd.compute_sigma_hat(X)
    assert isinstance(S, np.ndarray) and S.dtype == np.float64
    ref = ref_cpu.sigma_hat(X.astype(np.float64))
    np.testing.assert_allclose(S, ref, rtol=1.01 * ULP32, atol=0)


@pytest.mark.parametrize("n,d", [(65536, 2052), (65537, 2052), (3000, 2048)])
def test_direct_epilogue_edges(n, d, cuda):
    """Raw shards whose whole K range fits one int32 item (n <= 65536) and whose
    tiles fill half the chip take the direct epilogue (S stored from the
    accumulators, no int64 image): the largest such n, one row more (image path),
    a ragged d (last tile partly past d) and extreme columns.  Reference: exact int64
    sums on a column subset that spans the first and last tiles (one rounding for
    /n), the full matrix within 1e-15 of a float64 GEMM (hipBLAS's float64 GEMM is
    not exact on integer data at these sizes: tools/diag_u8_exact.py, r03v)."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(n + d)
    Xh = rng.integers(0, 256, (n, d), dtype=np.uint8)
    Xh[:, 0] = 255
    Xh[:, 1] = 0
    Xh[::2, d - 1] = 255
    X = torch.from_numpy(Xh).to(cuda)
    S64 = de.linalg.sigma_hat_u8(X, dtype=torch.float64)
    S32 = de.linalg.sigma_hat_u8(X)
    cols = np.r_[0:40, 1000:1024, d - 40:d]
    Xi = Xh[:, cols].astype(np.int64)
    exact = (Xi.T @ Xi).astype(np.float64) / n
    np.testing.assert_array_equal(S64.cpu().numpy()[np.ix_(cols, cols)], exact)
    np.testing.assert_array_equal(S32.cpu().numpy()[np.ix_(cols, cols)], exact.astype(np.float32))
    assert torch.equal(S64, S64.t()) and torch.equal(S32, S32.t())
    Xf = X.double()
    torch.testing.assert_close(S64, (Xf.t() @ Xf) / n, rtol=1e-15, atol=0)
    # alpha = 1 (no /n) on a row-strided view of a wider array
    m = min(n, 3000)
    Wd = rng.integers(0, 256, (m, d + 12), dtype=np.uint8)
    S1 = de.linalg.sigma_hat_u8(torch.from_numpy(Wd).to(cuda)[:, :d], alpha=1.0, dtype=torch.float64)
    Wi = Wd[:, cols].astype(np.int64)
    np.testing.assert_array_equal(S1.cpu().numpy()[np.ix_(cols, cols)], (Wi.T @ Wi).astype(np.float64))
