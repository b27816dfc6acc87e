"""GPU parity of the HIP kernels against the float64 oracle and the golden vectors.

Tolerances (BASELINE.json north_star):
  * projector  ||P_gpu - P_ref||_F <= 1e-4  (sign / rotation invariant)
  * eigenvalues  |l_gpu - l_ref| <= 1e-5 * |l_ref|
  * SYRK  max |S_gpu - S_ref| <= 2e-6 * max |S_ref|  (fp32 accumulation vs float64)
"""
import numpy as np
import pytest
import torch

from oracle import ref_cpu
from tests.conftest import golden_keys, golden_names, load_golden

pytestmark = pytest.mark.gpu

P_TOL = 1e-4
EV_TOL = 1e-5


def _split3_tol(n):
    # split3 per-product error <= ~3 * 2^-16 relative, zero-mean: the max
    # elementwise error over max|S| falls like 1/sqrt(n) (CPU emulation, d = 256:
    # 1.5e-5 at n = 1, 4e-6 at 8, 1.6e-6 at 64, 3.5e-7 at 4096; the max over
    # more entries (larger d) sits higher).  "auto" uses split3 only for n >= 1024.
    return 2e-6 if n >= 1024 else (5e-6 if n >= 64 else 2e-5)


def _syrk_check(X32, cuda, rel=2e-6, algo="auto"):
    import distributed_eigenspaces_amd as de
    x = torch.from_numpy(X32).to(cuda)
    S = de.sigma_hat(x, algo=algo)
    torch.cuda.synchronize()
    Sg = S.cpu().numpy().astype(np.float64)
    Sr = ref_cpu.sigma_hat(X32.astype(np.float64))
    err = np.abs(Sg - Sr).max() / max(np.abs(Sr).max(), 1e-300)
    assert err <= rel, f"SYRK[{algo}] rel err {err:.3e} (n={X32.shape[0]}, d={X32.shape[1]})"
    assert np.array_equal(Sg, Sg.T), "SYRK output must be bit-exactly symmetric"
    return Sg


SYRK_SHAPES = [(1, 4), (7, 12), (33, 64), (100, 256), (257, 260), (1000, 520), (4097, 1000),
               (64, 5632), (40, 7424), (2048, 3072)]


@pytest.mark.parametrize("algo", ["auto", "fp32", "split3"])
@pytest.mark.parametrize("n,d", SYRK_SHAPES)
def test_syrk_shapes(n, d, algo, cuda):
    rng = np.random.default_rng(n * 7919 + d)
    X = rng.standard_normal((n, d)).astype(np.float32)
    tol = _split3_tol(n) if algo == "split3" or (algo == "auto" and n >= 1024) else 2e-6
    _syrk_check(X, cuda, rel=tol, algo=algo)


def test_syrk_fused_split_strided_nan_padding(cuda):
    """Rows strided (ldx > d) with NaN in the padding columns and d not a multiple
    of the 256-feature panel: the fused split reads only features < d."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(5)
    n, d, ldx = 3000, 300, 312
    big = np.full((n, ldx), np.nan, dtype=np.float32)
    big[:, :d] = rng.standard_normal((n, d)).astype(np.float32)
    view = torch.from_numpy(big).to(cuda)[:, :d]
    S = de.sigma_hat(view, algo="split3").cpu().numpy().astype(np.float64)
    Sr = ref_cpu.sigma_hat(big[:, :d].astype(np.float64))
    assert np.isfinite(S).all()
    assert np.abs(S - Sr).max() <= 2e-6 * np.abs(Sr).max()


def test_syrk_split3_integer_data_exact_split(cuda):
    """CIFAR-like 0..255 integers are exact in bf16 (lo = 0): split3 == fp32 sums."""
    rng = np.random.default_rng(12)
    X = rng.integers(0, 256, size=(3000, 1024)).astype(np.float32)
    _syrk_check(X, cuda, rel=2e-6, algo="split3")


def test_syrk_strided_rows(cuda):
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(3)
    big = torch.from_numpy(rng.standard_normal((300, 136)).astype(np.float32)).to(cuda)
    view = big[:, :128]  # row stride 136, % 4 == 0 -> used in place
    S = de.sigma_hat(view).cpu().numpy().astype(np.float64)
    Sr = ref_cpu.sigma_hat(view.cpu().numpy().astype(np.float64))
    assert np.abs(S - Sr).max() <= 2e-6 * np.abs(Sr).max()


@pytest.mark.parametrize("algo", ["auto", "fp32", "split3"])
@pytest.mark.parametrize("name", golden_names())
def test_worker_path_golden(name, algo, cuda):
    """Sigma_hat + top-k of every shard vs the reference's own outputs."""
    import distributed_eigenspaces_amd as de
    g = load_golden(name)
    X32 = g["X"].astype(np.float32)
    k = int(g["k"])
    for i, (lo, hi) in enumerate(g["ranges"]):
        S = de.sigma_hat(torch.from_numpy(X32[lo:hi]).to(cuda), algo=algo)
        r = de.topk_eigh(S, k)
        V = r.V.cpu().numpy().astype(np.float64)
        ev = r.evals.cpu().numpy().astype(np.float64)
        if i < len(g["worker_V"]):  # m = 8 at d = 8192: shard 0's basis is stored
            dist = ref_cpu.projector_distance(V, g["worker_V"][i])
            assert dist <= P_TOL, f"{name} shard {i}: ||P-P_ref||_F = {dist:.3e}"
        np.testing.assert_allclose(ev, g["worker_evals"][i], rtol=EV_TOL, atol=0)
        assert r.V.stride() == (1, V.shape[0])  # Fortran order like LAPACK


@pytest.mark.parametrize("name", golden_names())
def test_server_golden(name, cuda):
    """Implicit projector-average top-k vs the reference master + NB:306 solve."""
    import distributed_eigenspaces_amd as de
    if "server_V" not in golden_keys(name):
        pytest.skip("fixture stores the worker outputs only (d = 16384)")
    g = load_golden(name)
    k, m = int(g["k"]), int(g["m"])
    if len(g["worker_V"]) < m:
        pytest.skip("fixture stores shard 0's basis only: see test_gpu_configs "
                    "test_c3_server_leg_m8_golden for the end-to-end server check")
    bases = [torch.from_numpy(v.astype(np.float32)).to(cuda) for v in g["worker_V"]]
    Wt = de.stack_bases(bases)
    r = de.projavg_topk(Wt, k, 1.0 / m, q0=bases[0])
    V = r.V.cpu().numpy().astype(np.float64)
    dist = ref_cpu.projector_distance(V, g["server_V"])
    assert dist <= P_TOL, f"{name}: server ||P-P_ref||_F = {dist:.3e}"
    np.testing.assert_allclose(r.evals.cpu().numpy(), g["server_evals"], rtol=EV_TOL, atol=0)


def test_topk_matches_oracle_on_sigma_hat0(cuda):
    """Eigensolver alone on the reference's own float64 Sigma_hat (rounded to fp32)."""
    import distributed_eigenspaces_amd as de
    for name in golden_names():
        if "sigma_hat0" not in golden_keys(name):
            continue
        g = load_golden(name)
        k = int(g["k"])
        S32 = g["sigma_hat0"].astype(np.float32)
        r = de.topk_eigh(torch.from_numpy(S32).to(cuda), k)
        w, v = ref_cpu.top_k_eigh(S32.astype(np.float64), k)
        assert ref_cpu.projector_distance(r.V.cpu().numpy(), v) <= P_TOL
        np.testing.assert_allclose(r.evals.cpu().numpy(), w, rtol=EV_TOL, atol=0)


@pytest.mark.parametrize("d,k", [(16, 1), (64, 16), (100, 3), (128, 128), (300, 33), (3072, 16)])
def test_topk_random_spectra(d, k, cuda):
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(d + k)
    U, _ = np.linalg.qr(rng.standard_normal((d, d)))
    lam = np.concatenate([np.linspace(10, 5, k), np.linspace(1, 0.01, d - k)])
    S = (U * lam) @ U.T
    S = ((S + S.T) / 2).astype(np.float32)
    r = de.topk_eigh(torch.from_numpy(S).to(cuda), k)
    w, v = ref_cpu.top_k_eigh(S.astype(np.float64), k)
    assert ref_cpu.projector_distance(r.V.cpu().numpy(), v) <= P_TOL
    np.testing.assert_allclose(r.evals.cpu().numpy(), w, rtol=EV_TOL, atol=0)


def test_topk_rank_deficient(cuda):
    """Tiny shards (the notebook's 8-row batches): rank(S) < subspace size."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(5)
    X = rng.standard_normal((8, 256)).astype(np.float32)
    S = de.sigma_hat(torch.from_numpy(X).to(cuda))
    r = de.topk_eigh(S, 2)
    w, v = ref_cpu.top_k_eigh(ref_cpu.sigma_hat(X.astype(np.float64)), 2)
    assert ref_cpu.projector_distance(r.V.cpu().numpy(), v) <= P_TOL
    np.testing.assert_allclose(r.evals.cpu().numpy(), w, rtol=EV_TOL, atol=0)


def test_errors(cuda):
    import distributed_eigenspaces_amd as de
    S = torch.eye(32, device=cuda)
    with pytest.raises(ValueError):
        de.topk_eigh(S, 0)
    with pytest.raises(ValueError):
        de.topk_eigh(S, 33)
    S[0, 1] = float("nan")
    with pytest.raises(ValueError):
        de.topk_eigh(S, 2)


@pytest.mark.parametrize("algo", ["bf16x6", "fp32"])
@pytest.mark.parametrize("d,p", [(16, 16), (60, 16), (256, 32), (1000, 80), (3072, 128),
                                 (4100, 48), (8192, 80)])
def test_sym_apply_sweep(d, p, algo, cuda):
    """One solver sweep Y = S Q (bf16x6 and f32 MFMA kernels) vs float64, on a
    symmetric S with tails in both d % 64 and d % 8 (d = 60, 4100)."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(d * 31 + p)
    A = rng.standard_normal((d, d)).astype(np.float32)
    S = ((A + A.T) * 0.5).astype(np.float32)
    Q = rng.standard_normal((d, p)).astype(np.float32)
    Y = de.sym_apply(torch.from_numpy(S).to(cuda), torch.from_numpy(Q).to(cuda), algo=algo,
                     alpha=0.5)
    ref = 0.5 * (S.astype(np.float64) @ Q.astype(np.float64))
    err = np.abs(Y.cpu().numpy() - ref).max() / np.abs(ref).max()
    tol = 2e-6  # both kernels form fp32-grade products
    assert err <= tol, f"sym_apply[{algo}] d={d} p={p}: rel err {err:.3e} > {tol:.1e}"


@pytest.mark.parametrize("d,p,ld", [(520, 80, 528), (300, 128, 300), (8192, 64, 8192)])
def test_sym_apply_prepared_image_reuse(d, p, ld, cuda):
    """The solver's pattern: the S image is built once (first call), later sweeps
    with new Q reuse it (DEIG_SWEEP_PREPARED); strided S rows (ld > d)."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(d + p)
    A = rng.standard_normal((d, d)).astype(np.float32)
    S = ((A + A.T) * 0.5).astype(np.float32)
    Sp = np.zeros((d, ld), np.float32)
    Sp[:, :d] = S
    Sp[:, d:] = np.nan  # padding columns must never be read
    St = torch.from_numpy(Sp).to(cuda)[:, :d]
    for it in range(3):
        Q = rng.standard_normal((d, p)).astype(np.float32)
        Y = de.sym_apply(St, torch.from_numpy(Q).to(cuda), algo="bf16x6", prepared=it > 0)
        ref = S.astype(np.float64) @ Q.astype(np.float64)
        err = np.abs(Y.cpu().numpy() - ref).max() / np.abs(ref).max()
        assert err <= 2e-6, f"prepared sweep {it}: rel err {err:.3e}"


@pytest.mark.parametrize("d,p", [(520, 80), (300, 128), (1000, 16), (8192, 80)])
def test_sym_apply_round_q(d, p, cuda):
    """The solver's mode (DEIG_SWEEP_ROUND_Q): Q is rounded in place to Q' = h + m
    (two bf16 pieces: |Q' - Q| <= 2^-17 |Q|, Q' exactly bf16(Q') + bf16(Q' - bf16(Q'))),
    and Y = S Q' to fp32 grade (five bf16 products) against float64 S @ Q'."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(7 * d + p)
    A = rng.standard_normal((d, d)).astype(np.float32)
    S = ((A + A.T) * 0.5).astype(np.float32)
    Q = rng.standard_normal((d, p)).astype(np.float32)
    St = torch.from_numpy(S).to(cuda)
    Qt = torch.from_numpy(Q).to(cuda)
    for it in range(2):
        Y = de.sym_apply(St, Qt, algo="bf16x6", prepared=it > 0, round_q=True)
        Qr = Qt.cpu().numpy()
        assert np.all(np.abs(Qr - Q) <= 2.0 ** -17 * np.abs(Q) * 1.0001), "rounding exceeds 2^-17"
        h = torch.from_numpy(Qr).to(torch.bfloat16).float()
        m = (torch.from_numpy(Qr) - h).to(torch.bfloat16).float()
        assert torch.equal(h + m, torch.from_numpy(Qr)), "Q' is not two bf16 pieces"
        ref = S.astype(np.float64) @ Qr.astype(np.float64)
        err = np.abs(Y.cpu().numpy() - ref).max() / np.abs(ref).max()
        assert err <= 2e-6, f"round_q sweep d={d} p={p} it={it}: rel err {err:.3e}"
        # idempotent: Q' is already two pieces, a second sweep leaves it unchanged
        Q = Qr


@pytest.mark.parametrize("d,p", [(520, 80), (300, 128), (1000, 16), (8192, 80), (4100, 96)])
def test_sym_apply_fast(d, p, cuda):
    """The solver's early-sweep mode (DEIG_SWEEP_FAST): Q rounded in place as in
    round_q, S taken as its two leading bf16 pieces S' = h + m from the prepared
    two-piece image, three products hh + hm + mh.  Against float64 S' @ Q' the only
    error is the dropped m m term (2^-18 per product) and fp32 accumulation; against
    the exact S @ Q' it is ~2^-16 relative."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(11 * d + p)
    A = rng.standard_normal((d, d)).astype(np.float32)
    S = ((A + A.T) * 0.5).astype(np.float32)
    Q = rng.standard_normal((d, p)).astype(np.float32)
    St = torch.from_numpy(S).to(cuda)
    Qt = torch.from_numpy(Q).to(cuda)
    Sh = torch.from_numpy(S).to(torch.bfloat16).float()
    S2 = (Sh + (torch.from_numpy(S) - Sh).to(torch.bfloat16).float()).double().numpy()
    for it in range(2):
        Y = de.sym_apply(St, Qt, prepared=it > 0, fast=True).cpu().numpy().astype(np.float64)
        Qr = Qt.cpu().numpy()
        assert np.all(np.abs(Qr - Q) <= 2.0 ** -17 * np.abs(Q) * 1.0001), "rounding exceeds 2^-17"
        ref2 = S2 @ Qr.astype(np.float64)
        ref = S.astype(np.float64) @ Qr.astype(np.float64)
        scale = np.abs(ref).max()
        assert np.abs(Y - ref2).max() / scale <= 1e-5, f"fast sweep vs S'Q' d={d} p={p} it={it}"
        assert np.abs(Y - ref).max() / scale <= 6e-5, f"fast sweep vs SQ' d={d} p={p} it={it}"
        Q = Qr
    # the exact modes still read the three-piece path after a fast call on one image
    Y6 = de.sym_apply(St, Qt, prepared=True).cpu().numpy()
    ref = S.astype(np.float64) @ Qt.cpu().numpy().astype(np.float64)
    assert np.abs(Y6 - ref).max() / np.abs(ref).max() <= 2e-6


@pytest.mark.parametrize("d,p", [(520, 80), (300, 128), (8192, 80), (4100, 96), (2048, 64), (16384, 128)])
def test_sym_apply_half(d, p, cuda):
    """The solver's first sweeps (DEIG_SWEEP_HALF, p >= 64): Q rounded in place as in
    round_q, then S and Q both taken as their leading bf16 piece (round to nearest
    even), one product.  Against float64 bf16(S) @ bf16(Q) only the fp32
    accumulation differs; against the exact S @ Q' it is ~2^-9 relative."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(13 * d + p)
    A = rng.standard_normal((d, d)).astype(np.float32)
    S = ((A + A.T) * 0.5).astype(np.float32)
    Q = rng.standard_normal((d, p)).astype(np.float32)
    St = torch.from_numpy(S).to(cuda)
    Qt = torch.from_numpy(Q).to(cuda)
    Sh = torch.from_numpy(S).to(torch.bfloat16).double().numpy()
    for it in range(2):
        Y = de.sym_apply(St, Qt, prepared=it > 0, half=True).cpu().numpy().astype(np.float64)
        Qr = Qt.cpu().numpy()
        assert np.all(np.abs(Qr - Q) <= 2.0 ** -17 * np.abs(Q) * 1.0001), "rounding exceeds 2^-17"
        # the h piece of the Q the call received (bf16(Q') can differ from it where m
        # is exactly half an ulp of h: a tie)
        Qh = torch.from_numpy(Q).to(torch.bfloat16).double().numpy()
        ref1 = Sh @ Qh
        ref = S.astype(np.float64) @ Qr.astype(np.float64)
        scale = np.abs(ref).max()
        assert np.abs(Y - ref1).max() / scale <= 1e-5, f"half sweep vs h(S)h(Q) d={d} p={p} it={it}"
        assert np.abs(Y - ref).max() / scale <= 1e-2, f"half sweep vs SQ' d={d} p={p} it={it}"
        Q = Qr
    # the other modes still read their own paths after a half call on one image
    Y3 = de.sym_apply(St, Qt, prepared=True, fast=True).cpu().numpy()
    Y6 = de.sym_apply(St, Qt, prepared=True).cpu().numpy()
    ref = S.astype(np.float64) @ Qt.cpu().numpy().astype(np.float64)
    assert np.abs(Y3 - ref).max() / np.abs(ref).max() <= 6e-5
    assert np.abs(Y6 - ref).max() / np.abs(ref).max() <= 2e-6


@pytest.mark.parametrize("d,p", [(1000, 16), (3072, 48)])
def test_sym_apply_half_below_p64_is_fast(d, p, cuda):
    """Below p = 64 (no v3 sweep kernel) DEIG_SWEEP_HALF runs the FAST mode: the same
    bits as fast=True on the same input."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(d * p)
    A = rng.standard_normal((d, d)).astype(np.float32)
    St = torch.from_numpy((A + A.T) * 0.5).to(cuda)
    Q = torch.from_numpy(rng.standard_normal((d, p)).astype(np.float32)).to(cuda)
    Q2 = Q.clone()
    Yh = de.sym_apply(St, Q, half=True)
    Yf = de.sym_apply(St, Q2, fast=True)
    assert torch.equal(Yh, Yf) and torch.equal(Q, Q2)


def test_sym_apply_rejects_bad_p(cuda):
    import distributed_eigenspaces_amd as de
    S = torch.eye(64, device=cuda)
    with pytest.raises(ValueError):
        de.sym_apply(S, torch.ones(64, 24, device=cuda))



@pytest.mark.parametrize("d,p,mode", [(512, 32, "exact"), (1000, 48, "round_q"), (3072, 32, "fast"),
                                      (8192, 80, "fast"), (2048, 128, "exact"), (8192, 80, "half"),
                                      (4096, 128, "half")])
def test_sym_power_fused_chain(d, p, mode, cuda):
    """The solver's sweep chain with the power step, the split-K reduction and the
    next sweep's Q image fused (sweep_finish_kernel) vs the same chain in float64:
    Y = S Q, Q_j <- cs_j Y_j (cs_j <= 0: column kept)."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(d + p)
    A = rng.standard_normal((d, d))
    S = ((A + A.T) / (2 * np.sqrt(d))).astype(np.float32)
    Q0 = rng.standard_normal((d, p)).astype(np.float32)
    cs = np.full(p, 0.5, dtype=np.float32)
    cs[3] = 0.0  # kept column
    steps = 4
    St = torch.from_numpy(S).to(cuda)
    Q = torch.from_numpy(Q0).to(cuda)
    kw = {"round_q": mode == "round_q", "fast": mode == "fast", "half": mode == "half"}
    Y = de.sym_power(St, Q, torch.from_numpy(cs), steps, **kw)
    Qr, S64 = Q0.astype(np.float64), S.astype(np.float64)
    for _ in range(steps):
        Yr = S64 @ Qr
        Qn = Yr * cs
        Qn[:, cs <= 0] = Qr[:, cs <= 0]
        Qr = Qn
    tol = {"exact": 6e-6, "round_q": 5e-5, "fast": 2e-4, "half": 2e-2}[mode]
    for got, ref in ((Y.cpu().numpy(), Yr), (Q.cpu().numpy(), Qr)):
        err = np.abs(got - ref).max() / np.abs(ref).max()
        assert err <= tol, f"sym_power[{mode}] d={d} p={p}: rel err {err:.3e} > {tol:.1e}"
    if mode != "exact":  # the basis stays rounded to two bf16 pieces, as sym_apply leaves it
        q = Q.cpu()
        h = q.to(torch.bfloat16).float()
        m = (q - h).to(torch.bfloat16).float()
        assert torch.equal(h + m, q)


@pytest.mark.parametrize("d", [2048, 2052, 4096])
def test_syrk_split3_variant_boundary(d, cuda):
    """Either side of the default's width switch (fused split up to d = 2048, the
    split pass above since r04), ragged n: both vs float64."""
    rng = np.random.default_rng(d)
    X = (rng.standard_normal((2085, d)) + 0.25).astype(np.float32)
    _syrk_check(X, cuda, rel=_split3_tol(2085), algo="split3")


def test_sym_apply_kernel_only_leaves_y(cuda):
    """DEIG_SWEEP_KERNEL_ONLY (measurement): the sweep kernel alone - Y untouched,
    and a following full call still returns S Q."""
    import distributed_eigenspaces_amd as de
    rng = np.random.default_rng(7)
    d, p = 1024, 48
    A = rng.standard_normal((d, d))
    S = torch.from_numpy(((A + A.T) / 2).astype(np.float32)).to(cuda)
    Q = torch.from_numpy(rng.standard_normal((d, p)).astype(np.float32)).to(cuda)
    Y = de.sym_apply(S, Q)
    Y2 = torch.full_like(Y, 7.0)
    de.sym_apply(S, Q, out=Y2, prepared=True, kernel_only=True)
    torch.cuda.synchronize()
    assert torch.all(Y2 == 7.0)
    Y3 = de.sym_apply(S, Q, prepared=True)
    assert torch.equal(Y, Y3)
