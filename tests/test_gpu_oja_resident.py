"""The block-resident Oja path (DEIG_OJA_RESIDENT, csrc/oja.hip oja_blk_kernel): one
launch per run of batches, Xb held in registers, in-launch hand-offs between the 256
workgroups.  Checked against the two-pass path (same products, other summation order)
and ref_cpu.oja_epoch (parity unpinned w.r.t. the reference: it has no Oja)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import ref_cpu

pytestmark = pytest.mark.gpu

P_TOL = 1e-4


def _data(nb, b, d, k, seed):
    from distributed_eigenspaces_amd import synthetic
    dev = torch.device("cuda", 0)
    U = synthetic.planted_basis(d, min(k, 16), seed=seed, device=dev)
    X = synthetic.spiked_samples(nb * b, U, seed=seed + 1)
    g = torch.Generator(device="cpu").manual_seed(seed + 2)
    V0 = torch.linalg.qr(torch.randn(d, k, generator=g, dtype=torch.float64))[0]
    return X, V0


def _run(X, V0, eta, b, orth, algo):
    import distributed_eigenspaces_amd as de
    V = V0.float().to(X.device).t().contiguous().t()
    de.oja_steps(X, V, eta, b, orth_every=orth, algo=algo)
    torch.cuda.synchronize()
    return V.cpu().double().numpy()


@pytest.mark.parametrize("d,k,nb,orth", [(3072, 32, 16, 8), (1024, 16, 5, 2), (512, 32, 3, 1),
                                          (2048, 20, 9, 4), (2560, 32, 4, 3), (1536, 8, 3, 8)])
def test_resident_matches_two_pass_and_oracle(d, k, nb, orth, cuda):
    b, eta = 4096, 0.02
    X, V0 = _data(nb, b, d, k, seed=d + k)
    Vr = _run(X, V0, eta, b, orth, "resident")
    Vt = _run(X, V0, eta, b, orth, "two_pass")
    assert np.isfinite(Vr).all()
    np.testing.assert_allclose(Vr.T @ Vr, np.eye(k), atol=1e-5)
    assert ref_cpu.projector_distance(Vr, Vt) <= 1e-5
    Vo = ref_cpu.oja_epoch(X.double().cpu().numpy(), V0.numpy(), eta, b)
    assert ref_cpu.projector_distance(Vr, Vo) <= P_TOL


def test_resident_deterministic_and_poisoned_workspace(cuda):
    """Bit-identical on a repeat, and every partial / image it reads was written first
    (a NaN-filled workspace changes nothing)."""
    from distributed_eigenspaces_amd import _lib
    b, d, k, nb, eta = 4096, 3072, 32, 4, 0.02
    X, V0 = _data(nb, b, d, k, seed=11)
    L = _lib.lib()
    nbytes = L.deig_oja_workspace(b, d, k)
    outs = []
    for fill in (0.0, float("nan"), float("nan")):
        ws = torch.full((nbytes // 4 + 1,), fill, dtype=torch.float32, device=X.device)
        V = V0.float().to(X.device).t().contiguous().t()
        rc = L.deig_oja_steps_ex(X.data_ptr(), nb, b, d, X.stride(0), ctypes.c_float(eta),
                                 V.data_ptr(), k, V.stride(1), 2, _lib.DEIG_OJA_RESIDENT,
                                 ws.data_ptr(), nbytes, None)
        assert rc == _lib.DEIG_OK, _lib.last_error()
        torch.cuda.synchronize()
        outs.append(V.cpu().numpy())
    assert np.isfinite(outs[0]).all()
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[1], outs[2])


def test_resident_refuses_other_shapes(cuda):
    import distributed_eigenspaces_amd as de
    X = torch.randn(2 * 2048, 1024, device="cuda")
    V = torch.linalg.qr(torch.randn(1024, 16, device="cuda"))[0].t().contiguous().t()
    with pytest.raises(ValueError, match="resident"):
        de.oja_steps(X, V, 0.02, 2048, algo="resident")
    de.oja_steps(X, V, 0.02, 2048, algo="auto")  # auto takes the two-pass path there
    assert torch.isfinite(V).all()


def test_resident_counters_reset_between_launches(cuda):
    """Each resident launch leaves its hand-off counters at zero for the next one (the
    last workgroup out resets them; only the call's first launch is preceded by a
    memset): 12 launches per call (orth_every = 1), three calls on one workspace with
    no re-initialisation between them - bit-identical results, every counter line (the
    first 65 x 128 B of the workspace) zero after each call."""
    from distributed_eigenspaces_amd import _lib
    b, d, k, nb, eta = 4096, 1024, 16, 12, 0.02
    X, V0 = _data(nb, b, d, k, seed=23)
    L = _lib.lib()
    nbytes = L.deig_oja_workspace(b, d, k)
    ws = torch.full((nbytes // 4 + 1,), float("nan"), dtype=torch.float32, device=X.device)
    outs = []
    for _ in range(3):
        V = V0.float().to(X.device).t().contiguous().t()
        rc = L.deig_oja_steps_ex(X.data_ptr(), nb, b, d, X.stride(0), ctypes.c_float(eta),
                                 V.data_ptr(), k, V.stride(1), 1, _lib.DEIG_OJA_RESIDENT,
                                 ws.data_ptr(), nbytes, None)
        assert rc == _lib.DEIG_OK, _lib.last_error()
        torch.cuda.synchronize()
        outs.append(V.cpu().numpy())
        cnt = ws[:65 * 32].view(torch.int32).cpu().numpy()
        assert not cnt.any(), f"counter lines left non-zero: {np.flatnonzero(cnt)[:8]}"
    assert np.isfinite(outs[0]).all()
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[1], outs[2])
    Vt = _run(X, V0, eta, b, 1, "two_pass")
    assert ref_cpu.projector_distance(outs[0].astype(np.float64), Vt) <= 1e-5
