"""NumPy fp32 emulation of the solver's outer loop (capi.hip solve) with the
Chebyshev filter between Rayleigh-Ritz steps, for choosing its parameters.

usage: python tools/emulate_cheb.py
"""
import math
import sys
import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ref_cpu  # noqa: E402


def rr(Q, Y, k, dtype):
    p = Q.shape[1]
    Z = np.concatenate([Q, Y], 1)
    C = (Z.T @ Z).astype(dtype)
    M, H, G = C[:p, :p], C[:p, p:], C[p:, p:]
    dm = np.diag(M).copy()
    dsc = np.where(dm > 0, 1 / np.sqrt(np.maximum(dm, 1e-300)), 1.0).astype(dtype)
    Mh = (M * dsc[:, None] * dsc[None, :]).astype(np.float64)
    # floored Cholesky (rr_small_kernel)
    L = np.zeros_like(Mh)
    for j in range(p):
        v = Mh[j, j] - L[j, :j] @ L[j, :j]
        v = max(v, 1e-6)
        L[j, j] = math.sqrt(v)
        L[j + 1:, j] = (Mh[j + 1:, j] - L[j + 1:, :j] @ L[j, :j]) / L[j, j]
    Li = np.linalg.inv(L).astype(dtype)
    Ht = Li @ (H * dsc[:, None] * dsc[None, :]) @ Li.T
    Ht = ((Ht + Ht.T) / 2).astype(np.float64)
    lam, U = np.linalg.eigh(Ht)
    lam = lam.astype(dtype)
    W = ((Li.T @ U.astype(dtype)) * dsc[:, None]).astype(dtype)
    g = np.einsum('aj,ab,bj->j', W, G, W)
    order = np.argsort(-lam, kind='stable')
    lam, W, g = lam[order], W[:, order], g[order]
    qw, yw = (Q @ W).astype(dtype), (Y @ W).astype(dtype)
    res = np.linalg.norm(yw[:, :k] - lam[:k] * qw[:, :k], axis=0) / abs(lam[0])
    cs = np.where(g > g.max() * 1e-10, 1 / np.sqrt(np.maximum(g, 1e-300)), 0).astype(dtype)
    Qn = np.where(cs > 0, yw * cs, qw).astype(dtype)
    return lam, qw, Qn, res.max()


def cheb_plan(lam, k, p, resid, tol, gmax, mmax, kappa=0.1, above=1e-2):
    """(cc, e, sigma1, m, theta_thr) for the next cycle, or None (power steps)."""
    if resid > above:
        return None
    gmax = min(gmax, max(10.0, kappa / max(resid, 1e-30)))
    a = 0.0
    c = lam[p - 1] if p - k >= 4 else min(lam[p - 1], 0.5 * lam[k - 1])
    if not (lam[k - 1] > c > a) or lam[0] <= c:
        return None
    cc, e = (c + a) / 2, (c - a) / 2
    t = lambda x: (x - cc) / e  # noqa: E731
    tk, t1 = t(lam[k - 1]), t(lam[0])
    rho = 1.0 / (tk + math.sqrt(tk * tk - 1))  # damping per degree, column k
    lr1, lrk = math.acosh(t1), math.acosh(tk)
    # degree: growth cap C_m(t1)/C_m(tk) ~ exp(m (acosh t1 - acosh tk)) <= gmax
    m = mmax
    if lr1 - lrk > 1e-9:
        m = min(m, max(1, int(math.log(gmax) / (lr1 - lrk))))
    need = math.log(max(tol * 0.3 / max(resid, 1e-30), 1e-30)) / math.log(rho)
    m = max(1, min(m, int(math.ceil(need))))
    # active columns: C_m(t1)/C_m(tj) <= gmax  <=>  acosh(tj) >= acosh(t1) - log(gmax)/m
    thr_t = math.cosh(max(lr1 - math.log(gmax) / m, 0.0))
    return cc, e, 1.0 / t1, m, cc + thr_t * e


def solve(S, k, p, max_sweeps=300, tol=1e-6, dtype=np.float32, cheb=True, gmax=100.0,
          mmax=16, rr_every=4, seed=0, verbose=False, kappa=0.1, above=1e-2):
    d = S.shape[0]
    S = S.astype(dtype)
    rng = np.random.default_rng(seed)
    Q = rng.uniform(-1, 1, (d, p)).astype(dtype)
    sweeps, rrs = 0, 0
    resid = np.inf
    lam = None
    hist = []
    while sweeps < max_sweeps:
        plan = cheb_plan(lam, k, p, resid, tol, gmax, mmax, kappa, above) if (cheb and lam is not None) else None
        if plan is not None:
            cc, e, s1, m, thr = plan
            act = (lam >= thr)[None, :]
            Xp, X = Q, Q
            sig = s1
            for j in range(m):
                Y = (S @ X).astype(dtype)
                sweeps += 1
                if j == 0:
                    Xn = (s1 / e) * (Y - cc * X)
                    sig_n = s1
                else:
                    sig_n = 1.0 / (2.0 / s1 - sig)
                    Xn = (2 * sig_n / e) * (Y - cc * X) - (sig * sig_n) * Xp
                Xn = np.where(act, Xn, X).astype(dtype)
                Xp, X, sig = X, Xn, sig_n
            Q = X
        elif lam is not None:
            for _ in range(rr_every - 1):
                Y = (S @ Q).astype(dtype)
                sweeps += 1
                Q = Y / np.linalg.norm(Y, axis=0)
        Y = (S @ Q).astype(dtype)
        sweeps += 1
        lam, qw, Q, resid = rr(Q, Y, k, dtype)
        rrs += 1
        hist.append((sweeps, float(resid)))
        if verbose:
            print(sweeps, resid, plan[3] if plan else None)
        if resid <= tol:
            break
    V = qw[:, :k][:, ::-1]
    return V, lam[:k][::-1], sweeps, rrs, resid, hist


def spectrum_matrix(lams, seed=0):
    d = len(lams)
    U = np.linalg.qr(np.random.default_rng(seed).standard_normal((d, d)))[0]
    return (U * lams) @ U.T


def cases(d=1024):
    rng = np.random.default_rng(1)
    out = {}
    k = 16
    # spiked covariance (c2/c3 like): spikes 9..5, MP bulk ~[0.7, 1.4]
    bulk = np.sort(rng.uniform(0.7, 1.4, d - k))[::-1]
    out["spiked"] = (np.concatenate([np.linspace(9, 5, k), bulk]), k)
    # small gap: lambda_{k+1}/lambda_k = 0.95, flat tail down to 0.5
    out["gap0.95"] = (np.concatenate([np.linspace(2, 1, k), np.linspace(0.95, 0.5, d - k)]), k)
    out["gap0.99"] = (np.concatenate([np.linspace(2, 1, k), np.linspace(0.99, 0.5, d - k)]), k)
    # power law (image-like) with a dominant mean direction, k = 10
    j = np.arange(1, d)
    out["powerlaw+mean"] = (np.concatenate([[3e4], 1e3 * j ** -1.2]), 10)
    # projector-average-like: k ones, rest small
    out["projavg"] = (np.concatenate([1 - 1e-3 * rng.random(k), 1e-2 * rng.random(d - k)]), k)
    return out


if __name__ == "__main__":
    for name, (lams, k) in cases().items():
        S = spectrum_matrix(np.asarray(lams, dtype=np.float64))
        w, Vr = ref_cpu.top_k_eigh(S, k)
        p = ((k + max(8, k // 4) + 15) // 16) * 16
        for cheb, g, kap in [(False, 0, 0), (True, 1e4, 0.01), (True, 1e4, 0.1), (True, 1e4, 1.0), (True, 1e6, 1.0)]:
            V, lam, sw, nrr, res, _ = solve(S, k, p, cheb=cheb, gmax=g or 100.0, kappa=kap)
            print(f"{name:14s} p={p:3d} cheb={cheb!s:5s} gmax={g:6.0f} kap={kap} sweeps={sw:4d} rr={nrr:3d} "
                  f"resid={res:.2e} P={ref_cpu.projector_distance(V, Vr):.2e} "
                  f"ev={np.max(np.abs(lam - w) / w):.1e}")
