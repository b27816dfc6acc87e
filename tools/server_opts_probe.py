"""Server-solve schedule A/B through deig_solver_opts (no rebuild): m worker bases of a
config's shape (spiked data, the default worker solve), then the projector-average
solve (linalg.projavg_topk, warm start V_1 as bench.py / the estimator call it) under
several option sets - median time, sweeps, residual, and the distance of each
variant's projector from the default's and from the planted basis.  Measurement tooling.

  python tools/server_opts_probe.py [--case c5|c3] [--reps R] [--variants name:key=val;key=val,...]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="c5")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="default:")
    a = ap.parse_args()
    import torch
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import _lib, synthetic
    n, d, k, m = {"c5": (65536, 16384, 128, 8), "c3": (1 << 18, 8192, 64, 8)}[a.case]
    dev = torch.device("cuda", 0)
    U = synthetic.planted_basis(d, k, seed=0, device=dev)
    bases = []
    for w in range(m):
        X = synthetic.spiked_samples(n, U, seed=1 + w)
        S = de.sigma_hat(X)
        del X
        bases.append(de.topk_eigh(S, k, check_finite=False).V)
        del S
    Wt = de.stack_bases(bases)
    torch.cuda.synchronize()

    def proj_dist(A, B):  # ||A A^T - B B^T||_F for orthonormal d x k bases
        sv = torch.linalg.svdvals(A.double().t() @ B.double()).clamp(max=1)
        return float(((1 - sv.pow(2)).clamp(min=0).sum() * 2).sqrt())

    ref = None
    for item in a.variants.split(","):
        name, _, kv = item.partition(":")
        fields = {kk: (int(v) if v.lstrip("-").isdigit() else float(v))
                  for kk, v in (x.split("=") for x in kv.split(";") if x)}
        o = _lib.solver_opts(**fields)
        ts, r = [], None
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = de.projavg_topk(Wt, k, 1.0 / m, q0=Wt[:k].t(), opts=o)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        if ref is None:
            ref = r
        print(json.dumps({"case": a.case, "variant": name, "ms": round(statistics.median(ts), 3),
                          "sweeps": r.sweeps, "resid": r.resid, "converged": r.converged,
                          "P_dist_vs_first": proj_dist(r.V, ref.V),
                          "evals_rel_vs_first": float(((r.evals - ref.evals).abs() / ref.evals.abs()).max()),
                          "sin_theta_planted": float(torch.linalg.svdvals(r.V.double().t() @ U.double())
                                                     .clamp(max=1).pow(2).neg().add(1).clamp(min=0)
                                                     .max().sqrt())}), flush=True)


if __name__ == "__main__":
    main()
