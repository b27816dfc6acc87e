"""Batched worker solves (include/deig.h deig_topk_sym_batch, linalg.topk_eigh_batch):
W problems advanced in lockstep with their small Rayleigh-Ritz solves in one launch
per step must give exactly what W separate topk_eigh calls give (same kernels, same
decisions), and meet the parity bars against the float64 oracle (distributed.py:22-29
per SlaveNode shard :42-53)."""
import numpy as np
import pytest
import torch

from oracle import ref_cpu

pytestmark = pytest.mark.gpu

P_TOL, EV_TOL = 1e-4, 1e-5


def _spiked_cov(d, k, n, seed, dev, mean=0.0):
    from distributed_eigenspaces_amd import synthetic
    U = synthetic.planted_basis(d, k, seed=seed, device=dev)
    X = synthetic.spiked_samples(n, U, seed=seed + 1) + mean
    return (X.double().t() @ X.double() / n)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_batch_equals_separate_solves(dtype, cuda):
    """Four spiked problems (one with a dominant mean direction, which takes the
    deflation redo path): bit-identical V, eigenvalues and sweep counts."""
    import distributed_eigenspaces_amd as de
    d, k = 1024, 10
    Ss = [_spiked_cov(d, k, 8192, 10 * i, cuda, mean=(3.0 if i == 2 else 0.0)).to(dtype)
          for i in range(4)]
    single = [de.topk_eigh(S, k) for S in Ss]
    batch = de.topk_eigh_batch(Ss, k)
    torch.cuda.synchronize()
    for a, b in zip(single, batch):
        assert a.sweeps == b.sweeps
        assert torch.equal(a.V, b.V)
        assert torch.equal(a.evals, b.evals)


def test_batch_two_stream_groups_equal_separate_solves(cuda):
    """d >= 2048: the batch runs as two interleaved groups on two streams (capi.hip
    solve_batch, r06); an odd count (groups of 2 and 1) with one dominant-mean problem
    (deflation path): still bit-identical to separate solves, and everything is
    ordered on the caller's stream when the call returns."""
    import distributed_eigenspaces_amd as de
    d, k = 2048, 12
    Ss = [_spiked_cov(d, k, 8192, 7 + 3 * i, cuda, mean=(3.0 if i == 1 else 0.0)) for i in range(3)]
    single = [de.topk_eigh(S, k) for S in Ss]
    side = torch.cuda.Stream(cuda)
    side.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(side):  # a non-default caller stream
        for S in Ss:
            S.record_stream(side)
        batch = de.topk_eigh_batch(Ss, k)
        checks = [(b.V * 1.0).sum() for b in batch]  # work queued behind the call on `side`
    side.synchronize()
    torch.cuda.synchronize(cuda)
    for a, b, c in zip(single, batch, checks):
        assert a.sweeps == b.sweeps
        assert torch.equal(a.V, b.V)
        assert torch.equal(a.evals, b.evals)
        assert torch.equal(c, (a.V * 1.0).sum())


def test_batch_c1_shape_vs_oracle(cuda):
    """configs[0]'s worker shape: 8 byte shards (6250 x 3072, uncentered, float64
    exact covariance), k = 10, against float64 eigh of each shard."""
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    d, k, W, ni = 3072, 10, 8, 6250
    U = synthetic.planted_basis(d, k, seed=0, device=cuda)
    X = synthetic.spiked_bytes(W * ni, U, seed=1, channels=0)
    Ss = [de.sigma_hat(X[w * ni:(w + 1) * ni], dtype=torch.float64) for w in range(W)]
    rs = de.topk_eigh_batch(Ss, k)
    for w in (0, 5, 7):
        Sh = Ss[w].cpu().numpy()
        ev, V = ref_cpu.top_k_eigh(Sh, k)
        assert rs[w].converged
        assert ref_cpu.projector_distance(rs[w].V.cpu().numpy(), V) <= P_TOL
        np.testing.assert_allclose(rs[w].evals.double().cpu().numpy(), ev, rtol=EV_TOL)


def test_batch_k_above_128_and_padding(cuda):
    """k > 128 (locked blocks, the narrower last block) and d % 4 != 0 (padding)."""
    import distributed_eigenspaces_amd as de
    d, k = 1022, 150
    Ss = [_spiked_cov(1022, 150, 4096, 3 + i, cuda) for i in range(2)]
    single = [de.topk_eigh(S, k) for S in Ss]
    batch = de.topk_eigh_batch(Ss, k)
    for a, b in zip(single, batch):
        assert a.V.shape == b.V.shape == (d, k)
        assert torch.equal(a.V, b.V) and torch.equal(a.evals, b.evals)


def test_estimator_batched_workers_vs_serial(cuda):
    """DistributedEigenspaceEstimator with 4 workers per rank: the batched default
    equals the serial worker loop."""
    from distributed_eigenspaces_amd import synthetic
    from distributed_eigenspaces_amd.estimator import DistributedEigenspaceEstimator
    d, k = 768, 8
    U = synthetic.planted_basis(d, k, seed=4, device=cuda)
    X = synthetic.spiked_samples(4 * 4096, U, seed=5)
    a = DistributedEigenspaceEstimator(k, workers_per_rank=4).fit(X)
    b = DistributedEigenspaceEstimator(k, workers_per_rank=4, batched_workers=False).fit(X)
    assert torch.equal(a.Wt, b.Wt)
    assert torch.equal(a.V, b.V) and torch.equal(a.evals, b.evals)
