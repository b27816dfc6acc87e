"""The solvers stay inside the workspace they report (the f64-MFMA
Rayleigh-quotient pass wrote RQM_G = 256 partial rows while rq_workspace_bytes
reserved cdiv(d,512)*cdiv(d,8) of them - fewer than 256 for d below ~1020 - so an
explicit solve at small d wrote past its slice).

Each solve gets exactly ``deig_topk_workspace_ex`` (or ``deig_topk_batch_workspace``)
bytes followed by a canary region; the canary must come back untouched, and the pairs
must still meet the oracle's bars (reference/distributed.py:22-29)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import ref_cpu

pytestmark = pytest.mark.gpu

CANARY = 1 << 20
FILL = 0xA5


def _spd(d, seed, k=16):
    """Top-k eigenvalues 40..10 above a [0, 5) bulk: a gap at k the 1e-4 projector bar
    can resolve at the solver's 1e-6 residual."""
    rng = np.random.default_rng(seed)
    w = np.concatenate([np.linspace(40.0, 10.0, min(d, k)), rng.uniform(0.0, 5.0, d - min(d, k))])
    Q, _ = np.linalg.qr(rng.standard_normal((d, d)))
    return ((Q * w) @ Q.T).astype(np.float32)


def _solve_with_canary(S, k, algo, cuda):
    from distributed_eigenspaces_amd import _lib
    L = _lib.lib()
    d = S.shape[0]
    o = _lib.solver_opts(sweep_algo=algo)
    nbytes = L.deig_topk_workspace_ex(d, k, 0, _lib.DEIG_F32, ctypes.byref(o))
    buf = torch.full((nbytes + CANARY,), FILL, dtype=torch.uint8, device=cuda)
    V = torch.empty((k, d), dtype=torch.float32, device=cuda)
    ev = torch.empty(k, dtype=torch.float32, device=cuda)
    sw, rs = ctypes.c_int(0), ctypes.c_float(0)
    rc = L.deig_topk_sym_ex(S.data_ptr(), _lib.DEIG_F32, d, d, k, 0, 300, ctypes.c_float(1e-6), None, 0,
                            d, V.data_ptr(), d, ev.data_ptr(), ctypes.byref(sw), ctypes.byref(rs),
                            ctypes.byref(o), buf.data_ptr(), nbytes,
                            torch.cuda.current_stream().cuda_stream)
    _lib.check(rc, "deig_topk_sym_ex")
    torch.cuda.synchronize()
    tail = buf[nbytes:]
    bad = int((tail != FILL).sum())
    return V.t().cpu().numpy(), ev.cpu().numpy(), bad


@pytest.mark.parametrize("algo", ["auto", "fp32"])
@pytest.mark.parametrize("d,k", [(128, 8), (128, 64), (128, 128), (256, 32), (256, 128),
                                 (512, 64), (512, 128), (1024, 128)])
def test_topk_stays_in_workspace(d, k, algo, cuda):
    from distributed_eigenspaces_amd import _lib
    A = _spd(d, seed=d + k, k=k)
    S = torch.from_numpy(A).to(cuda)
    V, ev, bad = _solve_with_canary(S, k, _lib.SWEEP_ALGOS[algo], cuda)
    assert bad == 0, f"d={d} k={k} {algo}: {bad} canary bytes overwritten past the workspace"
    w, Vr = ref_cpu.top_k_eigh(A.astype(np.float64), k)
    assert np.max(np.abs(ev - w) / np.abs(w)) <= 1e-5
    if k < d:  # k = d: every direction, the projector is the identity either way
        assert ref_cpu.projector_distance(V, Vr) <= 1e-4


@pytest.mark.parametrize("d,k", [(128, 64), (256, 128), (512, 32)])
def test_batch_stays_in_workspace(d, k, cuda):
    """Batched solves share one allocation carved in equal slices: an overrun of one
    problem's slice lands in the next problem's (changing its result) or past the end
    (the canary).  Results must equal separate solves and the canary stay intact."""
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import _lib
    L = _lib.lib()
    W = 4
    mats = [torch.from_numpy(_spd(d, seed=100 * i + d, k=k)).to(cuda) for i in range(W)]
    o = _lib.solver_opts()
    nbytes = L.deig_topk_batch_workspace(W, d, k, 0, _lib.DEIG_F32, ctypes.byref(o))
    buf = torch.full((nbytes + CANARY,), FILL, dtype=torch.uint8, device=cuda)
    Vs = [torch.empty((k, d), dtype=torch.float32, device=cuda) for _ in range(W)]
    evs = [torch.empty(k, dtype=torch.float32, device=cuda) for _ in range(W)]
    vp = ctypes.c_void_p
    sweeps, resid, status = (ctypes.c_int * W)(), (ctypes.c_float * W)(), (ctypes.c_int * W)()
    rc = L.deig_topk_sym_batch_ex(W, (vp * W)(*[S.data_ptr() for S in mats]), _lib.DEIG_F32, d, d, k,
                                  0, 300, ctypes.c_float(1e-6), (vp * W)(*[V.data_ptr() for V in Vs]),
                                  d, (vp * W)(*[e.data_ptr() for e in evs]), sweeps, resid, status,
                                  ctypes.byref(o), buf.data_ptr(), nbytes,
                                  torch.cuda.current_stream().cuda_stream)
    _lib.check(rc, "deig_topk_sym_batch_ex")
    torch.cuda.synchronize()
    assert int((buf[nbytes:] != FILL).sum()) == 0, "batched solve wrote past its workspace"
    for i in range(W):
        r = de.topk_eigh(mats[i], k)
        assert torch.equal(r.evals, evs[i]), f"problem {i}: batch differs from a separate solve"
        assert torch.equal(r.V, Vs[i].t()), f"problem {i}: batch differs from a separate solve"
