"""GPU parity at the BASELINE.json configs' own workload sizes.

Each test runs the HIP path on one config's shapes and compares it with a
float64 restatement of the reference computation on the same fp32 inputs:

* c2  (configs[1]): 2^20 x 3072 spiked shard, k = 16 - worker (distributed.py:59-70,
  :22-29) vs scipy eigh of the float64 covariance, and the m = 8 logical-worker
  variant through the estimator vs the float64 one-shot (distributed.py:99-104,
  :126-130, NB:306);
* c4  (configs[3]): Oja on 4096 x 3072 batches, k = 32 (parity unpinned w.r.t. the
  reference - no Oja there - so against ref_cpu.oja_epoch / oja_stream);
* c5  (configs[4]): one d = 16384, k = 128 worker and a 64-basis server solve,
  against float64 subspace iteration in torch (LAPACK eigh at d = 16384 does not fit
  a test's time budget): projector distance, eigenvalues and float64 residuals.

The float64 covariances are formed on the GPU with torch (test infrastructure:
the reference itself is float64 NumPy, distributed.py:66-69).
Bars: ||P - P_ref||_F <= 1e-4, eigenvalues <= 1e-5 relative (north_star).
"""
import numpy as np
import pytest
import torch

from oracle import ref_cpu

pytestmark = pytest.mark.gpu
P_TOL, EV_TOL = 1e-4, 1e-5


def _cov64(X: torch.Tensor, chunk: int = 1 << 16) -> torch.Tensor:
    """float64 X^T X / n on the GPU (distributed.py:66-69 in float64)."""
    n, d = X.shape
    S = torch.zeros((d, d), dtype=torch.float64, device=X.device)
    for lo in range(0, n, chunk):
        xc = X[lo:lo + chunk].double()
        S.addmm_(xc.t(), xc)
    return S / n


def _topk64_subspace(op, d: int, k: int, p: int, iters: int, device, seed: int = 0):
    """float64 block subspace iteration + Rayleigh-Ritz in torch: top-k eigenpairs
    (ascending) of the symmetric PSD operator ``op`` (test oracle only)."""
    g = torch.Generator(device=device).manual_seed(seed)
    Q = torch.linalg.qr(torch.randn((d, p), generator=g, device=device, dtype=torch.float64))[0]
    for _ in range(iters):
        Q = torch.linalg.qr(op(Q))[0]
    H = Q.t() @ op(Q)
    w, U = torch.linalg.eigh((H + H.t()) / 2)
    V = Q @ U
    return w[-k:], V[:, -k:]


def test_c2_worker_vs_float64_eigh(cuda):
    """configs[1]: d = 3072, n = 2^20, k = 16, one worker on one GPU."""
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    n, d, k = 1 << 20, 3072, 16
    U = synthetic.planted_basis(d, k, seed=0, device=cuda)
    X = synthetic.spiked_samples(n, U, seed=1)
    S = de.sigma_hat(X)
    S64 = _cov64(X)
    err = float((S.double() - S64).abs().max() / S64.abs().max())
    assert err < 2e-6, err
    r = de.topk_eigh(S, k)
    assert r.converged
    w, V = ref_cpu.top_k_eigh(S64.cpu().numpy(), k)
    assert ref_cpu.projector_distance(r.V.cpu().numpy(), V) <= P_TOL
    np.testing.assert_allclose(r.evals.cpu().numpy(), w, rtol=EV_TOL)


def test_c2_eight_logical_workers_vs_float64_one_shot(cuda):
    """configs[1], m = 8 logical workers on one GPU (distributed.py:99-104 split of
    the same 2^20 rows): estimator server result vs the float64 one-shot."""
    from distributed_eigenspaces_amd import synthetic
    from distributed_eigenspaces_amd.estimator import DistributedEigenspaceEstimator
    n, d, k, m = 1 << 20, 3072, 16, 8
    U = synthetic.planted_basis(d, k, seed=0, device=cuda)
    X = synthetic.spiked_samples(n, U, seed=2)
    res = DistributedEigenspaceEstimator(k, workers_per_rank=m, concurrent_workers=True).fit(X)
    Vs = []
    for lo, hi in ref_cpu.split_batches(n, m):
        _, v = ref_cpu.top_k_eigh(_cov64(X[lo:hi]).cpu().numpy(), k)
        Vs.append(v)
    for i, v in enumerate(Vs):  # every worker's basis (rows of the gathered stack)
        Vg = res.Wt[i * k:(i + 1) * k].t().double().cpu().numpy()
        assert ref_cpu.projector_distance(Vg, v) <= P_TOL, i
    sw, sv = ref_cpu.server_topk(Vs, k, m)
    assert ref_cpu.projector_distance(res.V.cpu().numpy(), sv) <= P_TOL
    np.testing.assert_allclose(res.evals.cpu().numpy(), sw, rtol=EV_TOL)


def test_c4_oja_config_shape_vs_oracle(cuda):
    """configs[3]: Oja steps on 4096 x 3072 batches, k = 32, the config's eta and
    orth_every; parity unpinned (no Oja in the reference): ref_cpu.oja_epoch."""
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    import bench
    b, d, k, nb, eta = 4096, 3072, 32, 32, 0.02
    U = synthetic.planted_basis(d, k, seed=0, device=cuda)
    X = synthetic.spiked_samples(nb * b, U, seed=3)
    g = torch.Generator(device="cpu").manual_seed(5)
    V0 = torch.linalg.qr(torch.randn(d, k, generator=g, dtype=torch.float64))[0]
    Vr = ref_cpu.oja_epoch(X.double().cpu().numpy(), V0.numpy(), eta, b)
    V = V0.float().to(cuda).t().contiguous().t()
    de.oja_steps(X, V, eta, b, orth_every=bench.CONFIGS["c4"]["orth_every"])
    Vg = V.cpu().numpy()
    np.testing.assert_allclose(Vg.T @ Vg, np.eye(k), atol=1e-5)
    assert ref_cpu.projector_distance(Vg, Vr) <= P_TOL


def test_c4_streaming_aggregation_config_shape(cuda):
    """configs[3] with periodic aggregation (every 8 batches here) on one rank ==
    ref_cpu.oja_stream with R = 1 (parity unpinned w.r.t. the reference)."""
    from distributed_eigenspaces_amd import synthetic
    from distributed_eigenspaces_amd.streaming import StreamingOja
    b, d, k, nb, eta, agg = 4096, 3072, 32, 16, 0.02, 8
    U = synthetic.planted_basis(d, k, seed=0, device=cuda)
    X = synthetic.spiked_samples(nb * b, U, seed=4)
    g = torch.Generator(device="cpu").manual_seed(6)
    V0 = torch.linalg.qr(torch.randn(d, k, generator=g, dtype=torch.float64))[0].float()
    est = StreamingOja(V0.to(cuda), eta=eta, agg_every=agg)
    est.partial_fit_block(X, b)
    assert est.aggregations == nb // agg
    batches = [X[i * b:(i + 1) * b].double().cpu().numpy() for i in range(nb)]
    ref = ref_cpu.oja_stream([batches], V0.double().numpy(), eta, agg)
    assert ref_cpu.projector_distance(est.V.cpu().numpy(), ref) <= P_TOL


def test_c5_worker_d16384_k128_vs_float64(cuda):
    """configs[4] worker: 65,536 rows x d = 16384, k = 128 (p = k = 128, no guard
    columns): against float64 subspace iteration on the float64 covariance of the
    same rows; float64 residuals and orthonormality."""
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    n, d, k = 65536, 16384, 128
    U = synthetic.planted_basis(d, k, seed=0, device=cuda)
    X = synthetic.spiked_samples(n, U, seed=5)
    S = de.sigma_hat(X)
    S64 = _cov64(X)
    del X
    r = de.topk_eigh(S, k, check_finite=False)
    assert r.converged
    V = r.V.double()
    ev = r.evals.double()
    np.testing.assert_allclose((V.t() @ V).cpu().numpy(), np.eye(k), atol=2e-5)
    R = S64 @ V - V * ev[None, :]
    assert float(R.norm(dim=0).max() / ev[-1]) < 1e-5
    w, Vr = _topk64_subspace(lambda Q: S64 @ Q, d, k, 192, 40, cuda)
    np.testing.assert_allclose(ev.cpu().numpy(), w.cpu().numpy(), rtol=EV_TOL)
    assert ref_cpu.projector_distance(V.cpu().numpy(), Vr.cpu().numpy()) <= P_TOL


def test_c5_server_64_bases_d16384_k128(cuda):
    """configs[4] server: 64 bases of d = 16384, k = 128 (Wt = 8192 x 16384, 537 MB),
    top-k of (1/64) sum V_i V_i^T without forming d x d (distributed.py:126-130,
    NB:306), against float64 subspace iteration on the same implicit operator."""
    import distributed_eigenspaces_amd as de
    d, k, m = 16384, 128, 64
    g = torch.Generator(device=cuda).manual_seed(7)
    U = torch.linalg.qr(torch.randn((d, k), generator=g, device=cuda, dtype=torch.float64))[0]
    bases = []
    for i in range(m):  # worker estimates = U rotated slightly off by independent noise
        E = torch.randn((d, k), generator=g, device=cuda, dtype=torch.float64) * 0.02
        bases.append(torch.linalg.qr(U + E)[0].float())
    Wt = de.stack_bases(bases)
    res = de.projavg_topk(Wt, k, 1.0 / m, q0=bases[0])
    assert res.converged
    W64 = Wt.double()
    op = lambda Q: W64.t() @ (W64 @ Q) / m  # noqa: E731
    V = res.V.double()
    ev = res.evals.double()
    R = op(V) - V * ev[None, :]
    assert float(R.norm(dim=0).max() / ev[-1]) < 1e-5
    w, Vr = _topk64_subspace(op, d, k, 160, 12, cuda)
    np.testing.assert_allclose(ev.cpu().numpy(), w.cpu().numpy(), rtol=EV_TOL)
    assert ref_cpu.projector_distance(V.cpu().numpy(), Vr.cpu().numpy()) <= P_TOL


def test_c3_server_leg_m8_golden(cuda):
    """configs[2]'s server leg on one GPU: the 8-basis projector average at d = 8192,
    k = 64 (distributed.py:126-130 + NB:306) from 8 logical workers' bases, against
    the reference's own run (tests/golden spiked_d8192_k64_m8_seeded: 8 shards of 8192
    rows through distributed.py's SlaveNode math, the master's sigma_tilde and the
    notebook's server solve).  End to end through the estimator (one rank, 8
    workers): shard 0's basis and every worker's eigenvalues, then the server basis
    and its eigenvalues."""
    from distributed_eigenspaces_amd.estimator import DistributedEigenspaceEstimator
    from tests.conftest import load_golden
    g = load_golden("spiked_d8192_k64_m8_seeded")
    k, m = int(g["k"]), int(g["m"])
    X = torch.from_numpy(np.array(g["Xq"])).to(cuda).float() / float(g["grid"])
    est = DistributedEigenspaceEstimator(k, workers_per_rank=m)
    r = est.fit(X)
    torch.cuda.synchronize()
    for i in range(m):
        np.testing.assert_allclose(r.worker_evals[i].double().cpu().numpy(), g["worker_evals"][i],
                                   rtol=EV_TOL)
    V0 = r.Wt[:k].t().double().cpu().numpy()
    assert ref_cpu.projector_distance(V0, g["worker_V"][0]) <= P_TOL
    dist = ref_cpu.projector_distance(r.V.cpu().numpy(), g["server_V"])
    assert dist <= P_TOL, dist
    np.testing.assert_allclose(r.evals.double().cpu().numpy(), g["server_evals"], rtol=EV_TOL)
