"""End-to-end GPU parity of the drop-in APIs against the reference's golden outputs
and the float64 oracle, plus full-size property tests.

Tolerances: ||P_gpu - P_ref||_F <= 1e-4, eigenvalues <= 1e-5 relative
(BASELINE.json north_star).  Oja has no reference: parity unpinned, judged by
sin(theta) against the one-shot oracle."""
import json

import numpy as np
import pytest
import torch

from oracle import ref_cpu
from tests.conftest import golden_keys, golden_names, load_golden

pytestmark = pytest.mark.gpu
P_TOL, EV_TOL = 1e-4, 1e-5


@pytest.mark.parametrize("name", [n for n in golden_names()
                                  if "request_ranges" in golden_keys(n)])
def test_protocol_end_to_end_golden(name, cuda):
    """SlaveNode/MasterNode over the in-process broker == the reference run."""
    from distributed_eigenspaces_amd import broker as br
    from distributed_eigenspaces_amd import distributed as dd
    g = load_golden(name)
    data = g["X"]  # float64 host array, like distributed.py:171
    b = br.InProcBroker("gpu-" + name)
    dd.SlaveNode(b, data)
    master = dd.MasterNode(b, int(g["k"]), int(g["m"]), data)
    master.start()
    resps = [json.loads(body) for q, body in b.delivered if q == "master"]
    np.testing.assert_array_equal(np.array([r["batch"] for r in resps]), g["ranges"])
    for i, r in enumerate(resps):
        V = np.array(r["eigenspace"])
        assert ref_cpu.projector_distance(V, g["worker_V"][i]) <= P_TOL
    assert ref_cpu.projector_distance(master.eigenspace, g["server_V"]) <= P_TOL
    np.testing.assert_allclose(master.eigenvalues, g["server_evals"], rtol=EV_TOL)
    assert master.eigenspace.flags["F_CONTIGUOUS"]


def test_node_api_numpy_in_numpy_out(cuda):
    from distributed_eigenspaces_amd import distributed as dd
    g = load_golden("spiked_d64_k4_m8")
    S = g["sigma_hat0"]
    V = dd.top_k_eigenvectors(S, 4)
    assert isinstance(V, np.ndarray) and V.dtype == np.float64 and V.flags["F_CONTIGUOUS"]
    assert ref_cpu.projector_distance(V, ref_cpu.top_k_eigenvectors(S, 4)) <= P_TOL
    lo, hi = g["sigma_hat0_range"]
    Sg = dd.compute_sigma_hat(g["X"][lo:hi])
    assert isinstance(Sg, np.ndarray) and Sg.shape == S.shape
    np.testing.assert_allclose(Sg, S, rtol=0, atol=2e-6 * np.abs(S).max())


def test_notebook_online_golden(cuda):
    from distributed_eigenspaces_amd import notebook as nb
    g = load_golden("notebook_online_d64")
    batches = nb.make_batches(g["X"], int(g["batch_size"]))
    mw, w = nb.online_distributed_pca(batches, int(g["m"]), int(g["T"]), int(g["k"]),
                                      schedule="notebook")
    assert ref_cpu.projector_distance(mw, g["matrix_w"]) <= P_TOL
    np.testing.assert_allclose(w, g["final_evals"], rtol=EV_TOL)


def test_figure_schedule_vs_oracle(cuda):
    """Figure schedule (assets/algorithm.png): parity pinned to the oracle only."""
    from distributed_eigenspaces_amd import notebook as nb
    g = load_golden("spiked_d256_k10_m8")
    X, k, m, T = g["X"], int(g["k"]), 4, 2
    n_t = X.shape[0] // (T * m)
    fn = lambda t, l: X[((t - 1) * m + (l - 1)) * n_t:((t - 1) * m + l) * n_t]  # noqa: E731
    V, w = nb.online_distributed_pca(m=m, T=T, k=k, schedule="figure", batch_fn=fn)
    wr, vr, _ = ref_cpu.online_figure(fn, m, T, k)
    assert ref_cpu.projector_distance(V, vr) <= P_TOL
    np.testing.assert_allclose(w, wr, rtol=EV_TOL)


def test_one_shot_and_projection(cuda):
    from distributed_eigenspaces_amd import notebook as nb
    g = load_golden("spiked_d256_k10_m8")
    X, k, m = g["X"], int(g["k"]), int(g["m"])
    r = nb.one_shot_distributed_pca(X.astype(np.float32), k, m)
    _, _, sw, sv = ref_cpu.one_shot(X, k, m)
    assert ref_cpu.projector_distance(r.V.cpu().numpy(), sv) <= P_TOL
    np.testing.assert_allclose(r.evals.cpu().numpy(), sw, rtol=EV_TOL)
    Y = nb.project(X, np.asfortranarray(sv))
    np.testing.assert_allclose(Y, X @ sv, rtol=0, atol=2e-5 * np.abs(X @ sv).max())


@pytest.mark.parametrize("n,d,k", [(1000, 256, 2), (3000, 1024, 16), (777, 64, 17)])
def test_project_shapes(n, d, k, cuda):
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, d)).astype(np.float32)
    W = np.asfortranarray(rng.standard_normal((d, k)).astype(np.float32))
    Y = de.linalg.project(torch.from_numpy(X).to(cuda), torch.from_numpy(W).to(cuda))
    ref = X.astype(np.float64) @ W.astype(np.float64)
    np.testing.assert_allclose(Y.cpu().numpy(), ref, rtol=0, atol=1e-5 * np.abs(ref).max())


def test_oja_matches_oracle_restatement(cuda):
    """Parity unpinned w.r.t. the reference (Oja is not in it): the GPU step is
    checked against the float64 restatement ref_cpu.oja_epoch on identical inputs,
    and the estimate approaches the one-shot top-k subspace."""
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    d, k, b, steps, eta = 512, 8, 2048, 16, 0.5
    U = synthetic.planted_basis(d, k, seed=3, device=cuda)
    X = synthetic.spiked_samples(steps * b, U, seed=4)
    V0 = torch.linalg.qr(torch.randn(d, k, device=cuda, dtype=torch.float64))[0]
    V = V0.float().t().contiguous().t()
    for i in range(steps):
        de.oja_step(X[i * b:(i + 1) * b], V, eta=eta)
    Xh = X.double().cpu().numpy()
    Vr = ref_cpu.oja_epoch(Xh, V0.cpu().numpy(), eta, b)
    Vg = V.cpu().numpy()
    np.testing.assert_allclose(Vg.T @ Vg, np.eye(k), atol=1e-5)  # orthonormal (CholQR2)
    assert ref_cpu.projector_distance(Vg, Vr) <= P_TOL
    _, vr = ref_cpu.top_k_eigh(ref_cpu.sigma_hat(Xh), k)
    assert ref_cpu.sin_theta(Vg, vr) < 0.3


def test_threaded_workers_overlap_safely(cuda):
    """my_threading.Slave workers on separate streams give the same bases."""
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd.my_threading import Slave
    g = load_golden("spiked_d256_k10_m8")
    X32 = torch.from_numpy(g["X"].astype(np.float32)).to(cuda)
    k = int(g["k"])
    out = [None] * len(g["ranges"])

    def work(i, lo, hi):
        s = torch.cuda.Stream(cuda)
        with torch.cuda.stream(s):
            S = de.sigma_hat(X32[lo:hi])
            out[i] = de.topk_eigh(S, k).V.cpu().numpy()
    ts = [Slave(work, i, int(lo), int(hi)) for i, (lo, hi) in enumerate(g["ranges"])]
    for t in ts:
        t.start()
    for t in ts:
        t.join(raise_error=True)
    for i, V in enumerate(out):
        assert ref_cpu.projector_distance(V, g["worker_V"][i]) <= P_TOL


def test_estimator_single_process(cuda):
    from distributed_eigenspaces_amd.estimator import DistributedEigenspaceEstimator
    g = load_golden("spiked_d256_k10_m8")
    X = torch.from_numpy(g["X"].astype(np.float32)).to(cuda)
    est = DistributedEigenspaceEstimator(int(g["k"]), workers_per_rank=int(g["m"]))
    r = est.fit(X)
    _, _, sw, sv = ref_cpu.one_shot(g["X"], int(g["k"]), int(g["m"]))
    assert ref_cpu.projector_distance(r.V.cpu().numpy(), sv) <= P_TOL
    np.testing.assert_allclose(r.evals.cpu().numpy(), sw, rtol=EV_TOL)


def test_estimator_concurrent_workers_match_serial(cuda):
    """concurrent_workers=True (each worker's solve in a Slave thread on its own
    stream, as bench.py runs config 5) gives the serial path's bases and the golden
    server result."""
    from distributed_eigenspaces_amd.estimator import DistributedEigenspaceEstimator
    g = load_golden("spiked_d256_k10_m8")
    X = torch.from_numpy(g["X"].astype(np.float32)).to(cuda)
    k, m = int(g["k"]), int(g["m"])
    rs = DistributedEigenspaceEstimator(k, workers_per_rank=m).fit(X)
    rc = DistributedEigenspaceEstimator(k, workers_per_rank=m, concurrent_workers=True).fit(X)
    torch.cuda.synchronize()
    assert rc.sweeps_worker == rs.sweeps_worker
    torch.testing.assert_close(rc.Wt, rs.Wt, rtol=0, atol=0)  # same kernels, same order
    _, _, sw, sv = ref_cpu.one_shot(g["X"], k, m)
    assert ref_cpu.projector_distance(rc.V.cpu().numpy(), sv) <= P_TOL
    np.testing.assert_allclose(rc.evals.cpu().numpy(), sw, rtol=EV_TOL)


def test_grayscale_ingest(cuda):
    from distributed_eigenspaces_amd import load_data
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (50, 32, 32, 3), dtype=np.uint8)
    g = load_data.grayscale_flatten(img).cpu().numpy()
    np.testing.assert_array_equal(g, img.mean(axis=3).reshape(50, -1).astype(np.float32))


# ---------------------------------------------------------------- full-size properties
def test_syrk_full_width_phases_and_remainder(cuda):
    """d = 8192: 528 tiles = 2 full phases over 256 CUs + 16 split-K remainder tiles.
    Checked on sampled entries against float64 dot products, and bit-symmetry."""
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    d, n, k = 8192, 40000, 64
    U = synthetic.planted_basis(d, k, seed=0, device=cuda)
    X = synthetic.spiked_samples(n, U, seed=9)
    S = de.sigma_hat(X)
    assert torch.equal(S, S.t())
    rng = np.random.default_rng(1)
    ii = torch.from_numpy(rng.integers(0, d, 512)).to(cuda)
    jj = torch.from_numpy(rng.integers(0, d, 512)).to(cuda)
    ref = (X[:, ii].double() * X[:, jj].double()).sum(0) / n
    got = S[ii, jj].double()
    scale = S.diagonal().abs().max().double()
    assert float((got - ref).abs().max() / scale) < 2e-6
    # diagonal = longest positive sums: two-level (flushed) fp32 accumulation
    dref = (X.double() ** 2).sum(0) / n
    assert float(((S.diagonal().double() - dref).abs() / dref).max()) < 5e-6
    # linearity: alpha = 1 on two halves sums to the whole (fp32 rounding of
    # 2 x 20000-row sums vs one 40000-row sum)
    S1 = de.sigma_hat(X[: n // 2], alpha=1.0)
    S2 = de.sigma_hat(X[n // 2:], alpha=1.0)
    assert float(((S1 + S2) / n - S).abs().max() / scale) < 1e-5


def test_full_size_worker_recovers_planted_subspace(cuda):
    """d = 8192, k = 64, 2^18 rows: the basis converges (small residual) and is close
    to the planted U (statistical error ~ sqrt(d / n))."""
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    d, n, k = 8192, 1 << 18, 64
    U = synthetic.planted_basis(d, k, seed=0, device=cuda)
    X = synthetic.spiked_samples(n, U, seed=2)
    S = de.sigma_hat(X)
    del X
    r = de.topk_eigh(S, k, check_finite=False)
    assert r.converged and r.resid < 1e-5
    s = torch.linalg.svdvals(U.double().t() @ r.V.double()).min().item()
    assert s > 0.99
    # eigenvalues ~ 1 + theta (8 -> 4) up to sampling error, ascending
    ev = r.evals.cpu().numpy()
    assert np.all(np.diff(ev) >= 0) and 4.5 < ev[0] < ev[-1] < 10.0
    # self-consistency: residual recomputed in float64 from S
    V = r.V.double()
    R = S.double() @ V - V * r.evals.double()[None, :]
    assert float(R.norm(dim=0).max() / ev[-1]) < 1e-5


def test_oja_steps_deferred_orthonormalisation_matches_oracle(cuda):
    """oja_steps (one C call, CholQR2 every orth_every batches) spans the same
    subspace as per-batch orthonormalisation (ref_cpu.oja_epoch); parity
    unpinned w.r.t. the reference (no Oja there)."""
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    d, k, b, steps, eta = 512, 8, 2048, 16, 0.5
    U = synthetic.planted_basis(d, k, seed=3, device=cuda)
    X = synthetic.spiked_samples(steps * b + 100, U, seed=4)  # + a partial batch (ignored)
    V0 = torch.linalg.qr(torch.randn(d, k, device=cuda, dtype=torch.float64))[0]
    Vr = ref_cpu.oja_epoch(X[:steps * b].double().cpu().numpy(), V0.cpu().numpy(), eta, b)
    for orth_every in (1, 3, 8):
        V = V0.float().t().contiguous().t()
        de.oja_steps(X, V, eta, b, orth_every=orth_every)
        Vg = V.cpu().numpy()
        np.testing.assert_allclose(Vg.T @ Vg, np.eye(k), atol=1e-5)
        assert ref_cpu.projector_distance(Vg, Vr) <= P_TOL, orth_every


def test_streaming_oja_single_rank_matches_oracle(cuda):
    """StreamingOja on one rank (aggregation = server solve of its own basis)
    == ref_cpu.oja_stream with R = 1; block and per-batch feeding agree."""
    from distributed_eigenspaces_amd import synthetic
    from distributed_eigenspaces_amd.streaming import StreamingOja
    d, k, b, nb, eta, agg = 256, 6, 1024, 10, 0.3, 4
    U = synthetic.planted_basis(d, k, seed=5, device=cuda)
    X = synthetic.spiked_samples(nb * b, U, seed=6)
    V0 = torch.linalg.qr(torch.randn(d, k, device=cuda, dtype=torch.float64))[0].float()
    a = StreamingOja(V0, eta=eta, agg_every=agg)
    for i in range(nb):
        a.partial_fit(X[i * b:(i + 1) * b])
    c = StreamingOja(V0, eta=eta, agg_every=agg)
    c.partial_fit_block(X, b)
    assert a.aggregations == c.aggregations == nb // agg
    batches = [X[i * b:(i + 1) * b].double().cpu().numpy() for i in range(nb)]
    ref = ref_cpu.oja_stream([batches], V0.double().cpu().numpy(), eta, agg)
    assert ref_cpu.projector_distance(a.V.cpu().numpy(), ref) <= P_TOL
    assert ref_cpu.projector_distance(c.V.cpu().numpy(), ref) <= P_TOL


def test_socket_two_process_protocol_gpu(tmp_path, cuda):
    """The multi-process CLI with the real GPU nodes: ``--mode master`` and ``--mode
    slave`` as separate processes over the socket broker (distributed.py:156-184),
    against the reference's golden run (arrival order and results)."""
    from tests.test_socket_broker import _run_pair
    g, r, _ = _run_pair(tmp_path, "spiked_d128_k2_m5_ragged", [], timeout=240)
    np.testing.assert_array_equal(r["ranges"], g["ranges"])
    for i in range(len(g["ranges"])):
        assert ref_cpu.projector_distance(r["worker_V"][i], g["worker_V"][i]) <= P_TOL
    assert ref_cpu.projector_distance(r["server_V"], g["server_V"]) <= P_TOL
    np.testing.assert_allclose(r["server_evals"], g["server_evals"], rtol=EV_TOL)


@pytest.mark.parametrize("d,b,k", [(500, 1000, 20), (260, 1040, 5), (96, 4100, 33)])
def test_oja_steps_ragged_shapes_poisoned_workspace(d, b, k, cuda):
    """Ragged Oja shapes - d and b not multiples of 32 (the last k-steps of both
    operand images partly past the data), k not a multiple of 16, a row stride
    > d - with the cached workspace filled with NaN bit patterns first: every
    image entry the kernels read must be written (zeros past the data)."""
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import linalg, synthetic
    nb, eta = 5, 0.4
    U = synthetic.planted_basis(d, k, seed=7, device=cuda)
    Xf = torch.zeros((nb * b, d + 12), dtype=torch.float32, device=cuda)
    Xf[:, :d] = synthetic.spiked_samples(nb * b, U, seed=8)
    X = Xf[:, :d]
    V0 = torch.linalg.qr(torch.randn(d, k, device=cuda, dtype=torch.float64))[0]
    linalg._workspace(X.device, 64 << 20).fill_(0xFF)
    V = V0.float().t().contiguous().t()
    de.oja_steps(X, V, eta, b, orth_every=2)
    Vg = V.cpu().numpy()
    assert np.isfinite(Vg).all()
    np.testing.assert_allclose(Vg.T @ Vg, np.eye(k), atol=1e-5)
    Vr = ref_cpu.oja_epoch(X.double().cpu().numpy(), V0.cpu().numpy(), eta, b)
    assert ref_cpu.projector_distance(Vg, Vr) <= P_TOL
