"""NumPy emulation of the GPU solver's algorithm (capi.hip solve + rr.hip) for debugging."""
import numpy as np


def emulate(S, k, p, sweeps, dtype=np.float32, seed=0, verbose=False):
    d = S.shape[0]
    rng = np.random.default_rng(seed)
    S = S.astype(dtype)
    Q = rng.uniform(-1, 1, (d, p)).astype(dtype)
    hist = []
    for it in range(sweeps):
        Y = S @ Q
        Z = np.concatenate([Q, Y], 1)
        C = Z.T @ Z
        M, H, G = C[:p, :p], C[:p, p:], C[p:, p:]
        dsc = 1 / np.sqrt(np.diag(M))
        Mh = M * dsc[:, None] * dsc[None, :]
        L = np.linalg.cholesky(Mh.astype(np.float64)).astype(dtype)
        Li = np.linalg.inv(L.astype(np.float64)).astype(dtype)
        Ht = Li @ (H * dsc[:, None] * dsc[None, :]) @ Li.T
        Ht = (Ht + Ht.T) / 2
        lam, U = np.linalg.eigh(Ht.astype(np.float64))
        lam = lam.astype(dtype); U = U.astype(dtype)
        W = (Li.T @ U) * dsc[:, None]
        g = np.einsum('aj,ab,bj->j', W, G, W)
        order = np.argsort(-lam, kind='stable')
        lam, W, g = lam[order], W[:, order], g[order]
        qw, yw = Q @ W, Y @ W
        res = np.linalg.norm(yw[:, :k] - lam[:k] * qw[:, :k], axis=0) / abs(lam[0])
        cs = np.where(g > g.max() * 1e-10, 1 / np.sqrt(np.maximum(g, 1e-300)), 0)
        Q = np.where(cs > 0, yw * cs, qw).astype(dtype)
        hist.append(res.max())
        if verbose:
            print(it, res.max(), lam[:k])
    V = qw[:, :k][:, ::-1]
    return V, lam[:k][::-1], hist


if __name__ == "__main__":
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from tests.conftest import load_golden
    from oracle import ref_cpu
    g = load_golden('spiked_d128_k2_m5_ragged')
    lo, hi = g['ranges'][3]
    X32 = g['X'][lo:hi].astype(np.float32)
    S = (X32.T @ X32) / np.float32(hi - lo)
    V, lam, hist = emulate(S, 2, 16, 60)
    print(np.array(hist)[[0, 5, 10, 20, 30, 40, 59]])
    print('dist', ref_cpu.projector_distance(V, g['worker_V'][3]), lam, g['worker_evals'][3])
