"""The reference-side binding (integration/deig_backend.py, the file INTEGRATION.md tells
a maintainer of the reference to add) driven alone - ctypes + numpy, no package, no
torch - on the reference's own data flow, at the bars of the float64 flow
(tests/test_gpu_f64flow.py: ||P - P_ref||_F <= 5e-5, eigenvalues 5e-6 relative).

Matches reference/distributed.py:22-29 (top_k_eigenvectors), :59-70
(compute_sigma_hat_) and :126-130 + the notebook's server solve (NB:306), and the
reference's float64 grey values (distributed.py:169-173)."""
import numpy as np
import pytest

from oracle import ref_cpu
from tests.conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu
P_TOL, EV_TOL = 5e-5, 5e-6


@pytest.fixture(scope="module")
def stub(cuda):
    from integration import deig_backend
    return deig_backend


@pytest.mark.parametrize("name", golden_names(max_d=3072))
def test_stub_golden(name, stub):
    """Every shard of the reference-run fixtures: Sigma, worker basis and eigenvalues,
    and the server solve, through the stub's float64 entry points."""
    g = load_golden(name)
    X, k, m = g["X"], int(g["k"]), int(g["m"])
    Vs = []
    for i, (lo, hi) in enumerate(g["ranges"]):
        S = stub.compute_sigma_hat(X[lo:hi])
        assert S.dtype == np.float64 and np.array_equal(S, S.T)
        if "sigma_hat0" in g and (lo, hi) == tuple(int(v) for v in g["sigma_hat0_range"]):
            # (500-row shards: the shifted path's fp32 SYRK of the centred rows,
            # ~3e-7 of max|S| at these n)
            np.testing.assert_allclose(S, g["sigma_hat0"], rtol=0,
                                       atol=1e-6 * np.abs(g["sigma_hat0"]).max())
        w, V = stub.top_k_eigh(S, k)
        assert V.flags["F_CONTIGUOUS"] and V.shape == (X.shape[1], k)
        if i < len(g["worker_V"]):
            assert ref_cpu.projector_distance(V, g["worker_V"][i]) <= P_TOL, (name, i)
        np.testing.assert_allclose(w, g["worker_evals"][i], rtol=EV_TOL)
        Vs.append(V)
    if "server_V" in g and len(g["worker_V"]) == m:
        Vbar = stub.server_top_k([v for v in g["worker_V"]], k, m)
        assert ref_cpu.projector_distance(Vbar, g["server_V"]) <= 1e-4


def test_stub_gray_cifar_shard(stub):
    """7500 x 1024 float64 grey values (one of 8 shards of the reference's 60000 CIFAR
    images, distributed.py:169-173): lambda_1 / lambda_k ~ 1e4, the regime where only
    the float64 entry points hold the bars (the fp32 route measured 0.8-1.4e-4,
    DESIGN.md §3.1c)."""
    from tests.test_gpu_f64flow import gray
    n, k = 7500, 10
    X = gray(n, k, seed=31)
    S = stub.compute_sigma_hat(X)
    S_ref = ref_cpu.sigma_hat(X)
    np.testing.assert_allclose(S, S_ref, rtol=0, atol=2e-7 * np.abs(S_ref).max())
    w, V = stub.top_k_eigh(S, k)
    w_ref, V_ref = ref_cpu.top_k_eigh(S_ref, k)
    assert w_ref[-1] / w_ref[0] > 1e3
    assert ref_cpu.projector_distance(V, V_ref) <= P_TOL
    np.testing.assert_allclose(w, w_ref, rtol=EV_TOL)
    # the uint8 bytes themselves (the exact integer covariance) through the same stub
    from tests.test_gpu_cifar import spiked_bytes
    B = spiked_bytes(6250, 3072, k, seed=32)
    Sb = stub.compute_sigma_hat(B)
    np.testing.assert_allclose(Sb, ref_cpu.sigma_hat(B.astype(np.float64)), rtol=1e-15, atol=0)


def test_stub_ragged_and_indefinite(stub):
    """A d the kernels pad (d = 766) with an indefinite matrix: the stub passes it as
    is and gets the reference's eigh answer."""
    rng = np.random.default_rng(4)
    d, k = 766, 6
    U = np.linalg.qr(rng.standard_normal((d, d)))[0]
    lam = np.concatenate([np.linspace(3, 1, 3), -np.linspace(0.5, 1.0, 3), -np.linspace(2, 9, d - 6)])
    S = (U * lam) @ U.T
    S = (S + S.T) / 2
    w, V = stub.top_k_eigh(S, k)
    w_ref, V_ref = ref_cpu.top_k_eigh(S, k)
    assert ref_cpu.projector_distance(V, V_ref) <= 1e-4
    np.testing.assert_allclose(w, w_ref, rtol=1e-5, atol=1e-6)
